"""Which joined-forward geometries run on the chunked stencil (no materialised join)?
Counts sehip.functional._join_raw calls per geometry (both join orders)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speech-enhancement_amd"))
import torch  # noqa: E402

from sehip import functional as F  # noqa: E402

calls = []
raw = F._join_raw
F._join_raw = lambda *a, **k: calls.append(1) or raw(*a, **k)
dev = torch.device("cuda")
cases = [
    # (x shape, s shape, kernel, stride, padding, output_padding, cat)
    ((2, 64, 16, 31), (2, 64, 17, 33), (7, 5), (2, 2), (3, 2), (0, 0), True),
    ((2, 64, 16, 33), (2, 64, 16, 33), (7, 5), (2, 2), (3, 2), (0, 0), False),
    ((2, 32, 9, 23), (2, 32, 9, 23), (5, 2), (2, 1), (2, 0), (0, 0), True),
    ((2, 32, 9, 23), (2, 32, 9, 23), (5, 2), (2, 1), (2, 0), (0, 0), False),
    ((2, 32, 9, 23), (2, 32, 9, 23), (5, 2), (2, 1), (2, 0), (1, 0), False),
    ((2, 32, 9, 24), (2, 32, 9, 23), (5, 2), (2, 1), (2, 0), (1, 0), False),
    ((2, 32, 9, 23), (2, 32, 9, 23), (5, 3), (2, 1), (2, 1), (0, 0), False),
]
for xs, ss, k, st, p, op, cat in cases:
    x, s = torch.randn(xs, device=dev), torch.randn(ss, device=dev)
    cin = 2 * xs[1]
    wr = torch.randn(cin // 2, 1, *k, device=dev) * 0.05
    wi = torch.randn(cin // 2, 1, *k, device=dev) * 0.05
    n0 = len(calls)
    with torch.no_grad():
        F.conv2d_joined(x, s, wr, wi, out_channels=2, kernel=k, stride=st, padding=p, output_padding=op,
                        transposed=True, cat=cat)
    torch.cuda.synchronize()
    print(xs, ss, k, st, p, op, "cat" if cat else "complex_concat", "materialised" if len(calls) > n0 else "stencil",
          flush=True)
