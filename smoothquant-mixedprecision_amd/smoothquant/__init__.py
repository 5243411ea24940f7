"""MI355X-native drop-in for adithyab100/smoothquant-mixedprecision's `smoothquant` package.

The hot path (W4A4Linear.from_float / forward) runs HIP kernels for gfx950 through the C
ABI in include/sqmp_w4a4.h; see DESIGN.md.  Same public surface as the reference's
smoothquant/__init__.py:1-4.
"""
from .smooth import smooth_lm
from .fake_quant import quantize_model

__all__ = ["smooth_lm", "quantize_model"]
