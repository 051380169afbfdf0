"""Python wrappers over the gfx950 HIP kernels in ``streamml._C``."""
from ._ext import gpu_available, has_c, load_c, load_io  # noqa: F401
