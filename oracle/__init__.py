"""ORACLE — test infrastructure only, never the product.

A CPU restatement (plain PyTorch on the CPU, fp32 by default, fp64 on
request) of shs2783/Speech-Enhancement's complex-spectral hot path, written
from the reference's *behaviour* with file:line citations into
/root/reference. It keeps the reference's constructor signatures and
state_dict keys so a state_dict moves freely between the reference, this
oracle and the HIP product path (speech-enhancement_amd/sehip).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker (or as the timed CPU baseline,
cpu_baseline.kind = "port"). The product path never imports it.

Parity pinning: tests/test_oracle_golden.py checks every module here against
tests/golden/*.npz, which tests/golden/gen_golden.py produced by importing
the reference itself.
"""
