"""ComplexLSTM fwd+bwd at FRCRN B=64 / 4 s (128 stacked sequences x 403
frames, H = 128, 2 layers, real+imag LSTMs): HIP recurrence vs MIOpen."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speech-enhancement_amd"))
import torch  # noqa: E402

from sehip import complex_nn  # noqa: E402
from sehip import functional as F  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = complex_nn.ComplexLSTM(256, 256, num_layers=2, batch_first=True).to(dev)
x = torch.randn(64, 403, 256, device=dev, requires_grad=True)


def run(hip, iters=5):
    orig = complex_nn._hip_lstm_ok
    if not hip:
        complex_nn._hip_lstm_ok = lambda mod: False
    try:
        for _ in range(2):
            m(x).sum().backward()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            m(x).sum().backward()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / iters * 1e3
    finally:
        complex_nn._hip_lstm_ok = orig


timer = F.OpTimer()
print(f"MIOpen nn.LSTM   fwd+bwd {run(False):8.2f} ms")
print(f"HIP recurrence   fwd+bwd {run(True):8.2f} ms")
F.set_op_timer(timer)
run(True, iters=3)
F.set_op_timer(None)
for k, v in timer.summary().items():
    print(f"  {k:10s} {v['ms'] / v['calls']:8.3f} ms/call  ({v['calls']} calls)  "
          f"{v['ms'] / v['calls'] * 1e3 / 403:6.2f} us/step")
