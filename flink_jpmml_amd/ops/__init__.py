"""Native HIP kernel library (``_pmml_kernels.so``, gfx950) and its ctypes ABI.

Kernels (``csrc/``): ``tree.hip`` (perfect / pointer / wide tree-ensemble traversal, split
reduce), ``cluster.hip`` (center-based clustering), ``linear.hip`` (regression tables + links),
``mlp.hip`` (fused all-layer MFMA MLP, bf16 and fp32), ``svm.hip`` (kernel eval + votes),
``host.hip`` (zero-copy / copy helpers). Shared device code: ``common.h`` (field preparation,
LDS staging), ``epilogue.h`` (fused target decode).
"""

from ._lib import KernelLibraryError, LIB_PATH, build, host_device_ptr, is_stale, load

__all__ = ["KernelLibraryError", "LIB_PATH", "build", "host_device_ptr", "is_stale", "load"]
