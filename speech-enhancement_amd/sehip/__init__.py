"""sehip — MI355X-native complex-spectral speech-enhancement hot path.

Python host mirroring shs2783/Speech-Enhancement's module surface
(conv_stft, modules.complex_nn, modules.ccbam, the FRCRN/DCCRN/DCUNet/CARN/
CRN models, losses, the training step) on top of libsehip.so, a C-ABI
library of hand-written HIP kernels for gfx950 (include/sehip.h).
"""
__version__ = "0.1.0"
