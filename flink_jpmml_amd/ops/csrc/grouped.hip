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

// ---- device-counted path (ONE tree launch per slice: tree_common.h::tree_grouped_wide_kernel) ----
//
//   group_count_kernel: per-code row counts of the slice (LDS histogram, one global atomic per
//     (workgroup, code)); the LAST workgroup to finish (ticket) reads and clears the counts and
//     writes the exclusive prefixes: cursor / row_start (grouped rows by code) and tile_start (the
//     entries' tiles, entry order = launch order, ceil(count / tile_rows) each). The host never
//     reads a count: it sizes the grid from the row count alone.
//   group_place_kernel: like group_rows_kernel, but rows of codes without a model (tile_rows 0:
//     unknown / deleted ids, EmptyScore) are answered on the spot in the arrival-order outputs and
//     the kernel records perm[pos] = row for the tree epilogue's scatter (no ungroup pass).

constexpr int COUNT_ROWS = 4096;  // rows per counting workgroup

// In-place exclusive prefix of v[0, L) (LDS, L <= GROUP_MAXK) by one workgroup; returns the total.
// Each thread owns a contiguous run; the GROUP_TB run sums are scanned by thread 0.
__device__ int block_exclusive_scan(int* v, int L, int* part) {
  const int tid = threadIdx.x;
  const int per = (L + GROUP_TB - 1) / GROUP_TB;
  const int a = min(L, tid * per), b = min(L, a + per);
  int run = 0;
  for (int i = a; i < b; ++i) run += v[i];
  part[tid] = run;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int i = 0; i < GROUP_TB; ++i) {
      const int x = part[i];
      part[i] = acc;
      acc += x;
    }
    part[GROUP_TB] = acc;
  }
  __syncthreads();
  int acc = part[tid];
  for (int i = a; i < b; ++i) {
    const int x = v[i];
    v[i] = acc;
    acc += x;
  }
  const int total = part[GROUP_TB];
  __syncthreads();
  return total;
}

template <typename CodeT>
__global__ __launch_bounds__(GROUP_TB) void group_count_kernel(const CodeT* __restrict__ codes, int n, int K,
                                                               const int* __restrict__ tile_rows,
                                                               const int* __restrict__ order, int n_entries,
                                                               int* counts, unsigned int* ticket, int* cursor,
                                                               int* row_start, int* tile_start) {
  __shared__ int cnt[GROUP_MAXK];
  __shared__ int tiles[GROUP_MAXK];
  __shared__ int part[GROUP_TB + 1];
  __shared__ int is_last;
  const int tid = threadIdx.x;
  for (int k = tid; k < K; k += GROUP_TB) cnt[k] = 0;
  __syncthreads();
  const int r0 = blockIdx.x * COUNT_ROWS;
  const int r1 = min(n, r0 + COUNT_ROWS);
  for (int i = r0 + tid; i < r1; i += GROUP_TB) {
    const int c = (int)codes[i];
    if (c >= 0 && c < K && tile_rows[c] > 0) atomicAdd(&cnt[c], 1);
  }
  __syncthreads();
  for (int k = tid; k < K; k += GROUP_TB)
    if (cnt[k]) atomicAdd(&counts[k], cnt[k]);
  __threadfence();
  __syncthreads();
  if (tid == 0) is_last = atomicAdd(ticket, 1u) == gridDim.x - 1u;
  __syncthreads();
  if (!is_last) return;
  __threadfence();
  // the last workgroup: every other workgroup's counts are visible; read + clear them
  for (int k = tid; k < K; k += GROUP_TB) cnt[k] = atomicExch(&counts[k], 0);
  __syncthreads();
  // per-entry tile counts (launch order) next to the per-code row counts
  for (int e = tid; e < n_entries; e += GROUP_TB) {
    const int c = order[e];
    const int tr = tile_rows[c];
    tiles[e] = tr > 0 ? (cnt[c] + tr - 1) / tr : 0;
  }
  __syncthreads();
  const int rows_total = block_exclusive_scan(cnt, K, part);
  const int tiles_total = block_exclusive_scan(tiles, n_entries, part);
  for (int k = tid; k < K; k += GROUP_TB) {
    cursor[k] = cnt[k];
    row_start[k] = cnt[k];
  }
  for (int e = tid; e < n_entries; e += GROUP_TB) tile_start[e] = tiles[e];
  if (tid == 0) {
    row_start[K] = rows_total;
    tile_start[n_entries] = tiles_total;
    *ticket = 0u;  // ready for the next slice (stream order)
  }
}

template <typename CodeT, bool VEC4>
__global__ __launch_bounds__(GROUP_TB) void group_place_kernel(const float* __restrict__ X, int ldx, int F, int n,
                                                               const CodeT* __restrict__ codes, int K,
                                                               const int* __restrict__ tile_rows,
                                                               int* __restrict__ cursor, float* __restrict__ Xg,
                                                               int* __restrict__ perm, float* __restrict__ out_s,
                                                               uint8_t* __restrict__ out_v) {
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
    if (code < 0 || code >= K || tile_rows[code] <= 0) {
      code = -1;  // no model behind this code: EmptyScore right here
      out_s[row] = __builtin_nanf("");
      out_v[row] = 0;
    } else {
      rank = atomicAdd(&cnt[code], 1);
    }
  }
  __syncthreads();
  for (int k = tid; k < K; k += GROUP_TB)
    if (cnt[k]) base[k] = atomicAdd(&cursor[k], cnt[k]);
  __syncthreads();
  const int pos = code >= 0 ? base[code] + rank : -1;
  pos_s[tid] = pos;
  if (pos >= 0) perm[pos] = row;
  __syncthreads();
  const int rows = min(GROUP_TB, n - row0);
  if (VEC4) {
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

// Device-counted grouping of one slice (see above). counts: K ints, zero before the first call (the
// kernel leaves them zero); ticket: one zeroed uint. cursor / row_start: K / K + 1 ints;
// tile_start: n_entries + 1 ints; order: n_entries codes (launch order of the tree entries);
// tile_rows: K ints (0 = no model). Xg: [n, F]; perm: n ints; out_s / out_v: the slice's
// arrival-order outputs (rows without a model are written here).
PMML_API int pmml_group_slice(hipStream_t stream, const float* X, int ldx, int F, int n, const void* codes,
                              int code_bytes, int K, const int* tile_rows, const int* order, int n_entries,
                              int* counts, unsigned int* ticket, int* cursor, int* row_start, int* tile_start,
                              float* Xg, int* perm, float* out_s, uint8_t* out_v) {
  if (n <= 0) return 0;
  if (K < 1 || K > GROUP_MAXK || F < 1 || ldx < F || n_entries < 0 || n_entries > K) return -2;
  const dim3 cgrid((n + COUNT_ROWS - 1) / COUNT_ROWS);
  const dim3 grid((n + GROUP_TB - 1) / GROUP_TB);
  const bool vec4 = (F & 3) == 0 && (ldx & 3) == 0 &&
                    ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Xg)) & 15) == 0;
#define PMML_SLICE(T)                                                                                    \
  hipLaunchKernelGGL(group_count_kernel<T>, cgrid, dim3(GROUP_TB), 0, stream, (const T*)codes, n, K, tile_rows, \
                     order, n_entries, counts, ticket, cursor, row_start, tile_start);                   \
  if (vec4)                                                                                              \
    hipLaunchKernelGGL((group_place_kernel<T, true>), grid, dim3(GROUP_TB), 0, stream, X, ldx, F, n,     \
                       (const T*)codes, K, tile_rows, cursor, Xg, perm, out_s, out_v);                   \
  else                                                                                                   \
    hipLaunchKernelGGL((group_place_kernel<T, false>), grid, dim3(GROUP_TB), 0, stream, X, ldx, F, n,    \
                       (const T*)codes, K, tile_rows, cursor, Xg, perm, out_s, out_v);
  switch (code_bytes) {
    case 1: PMML_SLICE(uint8_t) break;
    case 2: PMML_SLICE(int16_t) break;
    case 4: PMML_SLICE(int32_t) break;
    default: return -3;
  }
#undef PMML_SLICE
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
