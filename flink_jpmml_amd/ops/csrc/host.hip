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

// Page-lock an existing host range (e.g. a memory-mapped file in the page cache) so copy engines
// DMA straight from it: flags = hipHostRegister* (ReadOnly for PROT_READ mappings). Returns a
// hipError_t.
PMML_API int pmml_host_register(void* p, size_t bytes, unsigned flags) {
  return (int)hipHostRegister(p, bytes, flags);
}

PMML_API int pmml_host_unregister(void* p) { return (int)hipHostUnregister(p); }

PMML_API int pmml_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Pull copy: a grid-stride kernel reading pinned host memory through its device-visible address
// (PCIe reads issued by the CUs instead of an SDMA engine). Used by the ingest probe and as the
// kernel-pull H2D mode of the streaming engine.
__global__ __launch_bounds__(256) void pull_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        size_t n16) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256;
  for (; i + 3 * stride < n16; i += 4 * stride) {  // 4 independent 16-B loads in flight per lane
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

PMML_API int pmml_pull_copy(hipStream_t stream, const void* src_dev, void* dst, size_t bytes, int blocks) {
  if (bytes == 0) return 0;
  if ((bytes & 15) != 0 || (((uintptr_t)src_dev | (uintptr_t)dst) & 15) != 0) return -2;
  if (blocks <= 0) blocks = 1024;
  hipLaunchKernelGGL(pull_copy_kernel, dim3(blocks), dim3(256), 0, stream, (const uint4*)src_dev, (uint4*)dst,
                     bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
