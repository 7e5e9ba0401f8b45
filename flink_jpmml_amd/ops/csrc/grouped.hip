// Mixed-model micro-batches: device-side grouping of rows by model and the ungrouping epilogue.
//
// The reference's dynamic operator serves many models from one operator and picks the model per
// event (`S/package.scala:107-119`, `S/api/functions/EvaluationCoFunction.scala:106-117`). A
// columnar micro-batch here carries one model code per row. Instead of gathering each model's rows
// on the host (a 128-byte row copy per record through host memory), the rows cross PCIe once in
// arrival order and are grouped in HBM:
//
//   group_rows_kernel:  pos = cursor[code] + rank of the row among its workgroup's rows of that
//                       code (LDS atomics); Xg[pos] = X[row]; inv[row] = pos.
//                       cursor[k] enters as the exclusive prefix of the per-code row counts (known
//                       on the host, which needs them to size each model's launch) and advances by
//                       ONE global atomic per (workgroup, code), not one per row.
//   <one launch per model over its contiguous rows of Xg, epilogues into sg / vg>
//   ungroup_kernel:     out[j] = sg[inv[j]] — reads gathered from HBM, writes contiguous (the
//                       outputs usually live in pinned host memory, written zero-copy over PCIe:
//                       coalesced 4-byte stores there, scattered reads only on the HBM side).
//
// The order of rows inside a group depends on atomic timing; every row's score depends only on
// its own features, so the ungrouped result is deterministic.

#include "common.h"

namespace {

constexpr int GROUP_TB = 256;
constexpr int GROUP_MAXK = 1024;

template <typename CodeT, bool VEC4>
__global__ __launch_bounds__(GROUP_TB) void group_rows_kernel(const float* __restrict__ X, int ldx, int F, int n,
                                                              const CodeT* __restrict__ codes, int K,
                                                              int* __restrict__ cursor, float* __restrict__ Xg,
                                                              int* __restrict__ inv) {
  __shared__ int cnt[GROUP_MAXK];
  __shared__ int base[GROUP_MAXK];
  __shared__ int pos_s[GROUP_TB];
  const int tid = threadIdx.x;
  const int row0 = blockIdx.x * GROUP_TB;
  for (int k = tid; k < K; k += GROUP_TB) cnt[k] = 0;
  __syncthreads();
  const int row = row0 + tid;
  int code = -1, rank = 0;
  if (row < n) {
    code = (int)codes[row];
    if (code < 0 || code >= K) code = -1;  // never produced by the host; scored as EmptyScore
    else rank = atomicAdd(&cnt[code], 1);
  }
  __syncthreads();
  for (int k = tid; k < K; k += GROUP_TB)
    if (cnt[k]) base[k] = atomicAdd(&cursor[k], cnt[k]);
  __syncthreads();
  const int pos = code >= 0 ? base[code] + rank : -1;
  pos_s[tid] = pos;
  if (row < n) inv[row] = pos;
  __syncthreads();
  const int rows = min(GROUP_TB, n - row0);
  if (VEC4) {  // F % 4 == 0, ldx % 4 == 0, 16-byte aligned bases: float4 moves
    const int F4 = F >> 2;
    const int total = rows * F4;
    for (int e = tid; e < total; e += GROUP_TB) {
      const int r = e / F4, c = e - r * F4;
      const int p = pos_s[r];
      if (p >= 0) {
        const float4 v = *reinterpret_cast<const float4*>(X + (size_t)(row0 + r) * ldx + 4 * c);
        *reinterpret_cast<float4*>(Xg + (size_t)p * F + 4 * c) = v;
      }
    }
  } else {
    const int total = rows * F;
    for (int e = tid; e < total; e += GROUP_TB) {
      const int r = e / F, c = e - r * F;
      const int p = pos_s[r];
      if (p >= 0) Xg[(size_t)p * F + c] = X[(size_t)(row0 + r) * ldx + c];
    }
  }
}

__global__ __launch_bounds__(GROUP_TB) void ungroup_kernel(const float* __restrict__ sg, const uint8_t* __restrict__ vg,
                                                           const int* __restrict__ inv, int n, float* out_s,
                                                           uint8_t* out_v, float* out_s2, uint8_t* out_v2) {
  const int j = blockIdx.x * GROUP_TB + threadIdx.x;
  if (j >= n) return;
  const int p = inv[j];
  const float s = p >= 0 ? sg[p] : __builtin_nanf("");
  const uint8_t v = p >= 0 ? vg[p] : (uint8_t)0;
  out_s[j] = s;
  out_v[j] = v;
  if (out_s2) out_s2[j] = s;
  if (out_v2) out_v2[j] = v;
}

template <typename T>
void launch_group(hipStream_t stream, bool vec4, dim3 grid, const float* X, int ldx, int F, int n, const void* codes,
                  int K, int* cursor, float* Xg, int* inv) {
  if (vec4)
    hipLaunchKernelGGL((group_rows_kernel<T, true>), grid, dim3(GROUP_TB), 0, stream, X, ldx, F, n,
                       (const T*)codes, K, cursor, Xg, inv);
  else
    hipLaunchKernelGGL((group_rows_kernel<T, false>), grid, dim3(GROUP_TB), 0, stream, X, ldx, F, n,
                       (const T*)codes, K, cursor, Xg, inv);
}

}  // namespace

// code_bytes: 1 (uint8), 2 (int16) or 4 (int32) per row. cursor: K ints on the device holding the
// exclusive prefix of the per-code counts (consumed). Xg: [n, F] dense; inv: [n].
PMML_API int pmml_group_rows(hipStream_t stream, const float* X, int ldx, int F, int n, const void* codes,
                             int code_bytes, int K, int* cursor, float* Xg, int* inv) {
  if (n <= 0) return 0;
  if (K < 1 || K > GROUP_MAXK || F < 1 || ldx < F) return -2;
  const dim3 grid((n + GROUP_TB - 1) / GROUP_TB);
  const bool vec4 = (F & 3) == 0 && (ldx & 3) == 0 && ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Xg)) & 15) == 0;
  switch (code_bytes) {
    case 1: launch_group<uint8_t>(stream, vec4, grid, X, ldx, F, n, codes, K, cursor, Xg, inv); break;
    case 2: launch_group<int16_t>(stream, vec4, grid, X, ldx, F, n, codes, K, cursor, Xg, inv); break;
    case 4: launch_group<int32_t>(stream, vec4, grid, X, ldx, F, n, codes, K, cursor, Xg, inv); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

PMML_API int pmml_ungroup(hipStream_t stream, const float* sg, const uint8_t* vg, const int* inv, int n, float* out_s,
                          uint8_t* out_v, float* out_s2, uint8_t* out_v2) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ungroup_kernel, dim3((n + GROUP_TB - 1) / GROUP_TB), dim3(GROUP_TB), 0, stream, sg, vg, inv, n,
                     out_s, out_v, out_s2, out_v2);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
