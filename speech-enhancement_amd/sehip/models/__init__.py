"""Model zoo on the HIP path (mirrors /root/reference/models/__init__.py:1-23
for the complex-spectral models in scope)."""
from .carn import CARN, GCARN
from .crn import CRN
from .dccrn import DCCRN
from .dcunet import DCUNet, dcunet_architecture
from .frcrn import FRCRN
from ..complex_nn import ComplexBatchNorm2d, ComplexConv2d, ComplexLeakyReLU, ComplexReLU
from ..conv_stft import ConvSTFT, ConviSTFT

__all__ = ["CRN", "DCUNet", "DCCRN", "CARN", "GCARN", "FRCRN",
           "ComplexConv2d", "ComplexBatchNorm2d", "ComplexReLU", "ComplexLeakyReLU",
           "ConvSTFT", "ConviSTFT", "dcunet_architecture"]
