"""Native operators: HIP kernels for gfx950 + the C++ CPU kernel, bound through a C ABI (``_lib``)."""
from ._lib import kernels_available, io_available, cpu_available, NativeError  # noqa: F401
