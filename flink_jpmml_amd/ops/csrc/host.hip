// Host-side helpers exported with the kernel library (they bind to the HIP runtime instance that
// torch already loaded, so stream handles and pointers are shared).
#include "common.h"

// Device-visible address of pinned (hipHostMalloc'ed) host memory, for zero-copy kernel writes
// straight into the host sink buffers. Returns a hipError_t.
PMML_API int pmml_host_device_ptr(void* host, void** dev) {
  return (int)hipHostGetDevicePointer(dev, host, 0);
}

PMML_API int pmml_memcpy_async(void* dst, const void* src, size_t bytes, int kind, hipStream_t stream) {
  return (int)hipMemcpyAsync(dst, src, bytes, (hipMemcpyKind)kind, stream);
}

PMML_API int pmml_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
