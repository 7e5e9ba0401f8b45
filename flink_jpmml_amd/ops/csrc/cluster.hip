// Center-based ClusteringModel scoring: per-row distance to K centres + argmin/argmax.
//
// The centre table is tiny compared to the row stream and every lane of a wave needs the same
// centre element at the same time, so centres are read with wave-uniform addresses (scalar loads,
// broadcast to all lanes) — no LDS round trip. The row tile is staged in LDS [F][256] by the shared
// preparation/staging helper. Missing inputs are skipped and the sum rescaled by Σq / Σq_present
// (PMML ClusteringModel missing-value adjustment). Large K×F with complete rows goes through the
// MFMA path (‖x‖² − 2x·C + ‖C‖²) in a later revision.
#include "common.h"

namespace {

constexpr int TB = 256;

enum : int { M_SQEUCLID = 0, M_EUCLID = 1, M_CITY = 2, M_CHEBY = 3, M_MINKOWSKI = 4 };
enum : int { CF_ABSDIFF = 0, CF_GAUSS = 1, CF_DELTA = 2, CF_EQUAL = 3 };

struct ClusterArgs {
  const float* X;
  int n_rows, n_feat, ldx, K;
  const FieldPrep* prep;
  const float* centers;   // [K][F]
  const float* weights;   // [F]
  const float* scales;    // [F] gaussSim similarity scale
  const float* qweights;  // [F] missing-value weights
  const int* cfun;        // [F] compare function codes
  const float* table;     // [K] entity id parsed as double (NaN = not numeric)
  int metric, similarity;  // similarity: argmax instead of argmin
  float p;                 // minkowski p
  int pad;
  float* score;
  uint8_t* valid;
  int* label;              // [n] winning cluster index (nullable)
  float* affinity;         // [n] winning distance (nullable)
};

__device__ __forceinline__ float compare(int cf, float d, float s) {
  switch (cf) {
    case CF_GAUSS: return __expf(-0.69314718056f * d * d / (s * s));
    case CF_DELTA: return d != 0.f ? 1.f : 0.f;
    case CF_EQUAL: return d == 0.f ? 1.f : 0.f;
    default: return fabsf(d);
  }
}

template <int METRIC>
__global__ __launch_bounds__(TB) void cluster_kernel(ClusterArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  const int row0 = blockIdx.x * TB;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  const int tid = threadIdx.x;
  const int row = row0 + tid;
  if (row >= a.n_rows) return;
  const int F = a.n_feat;
  float qsum = 0.f, qpresent = 0.f;
  for (int f = 0; f < F; ++f) {
    const float q = a.qweights[f];
    qsum += q;
    if (feat[f * TB + tid] == feat[f * TB + tid]) qpresent += q;
  }
  const float adj = qpresent > 0.f ? qsum / qpresent : __builtin_nanf("");
  float best = a.similarity ? -__builtin_inff() : __builtin_inff();
  int best_k = -1;
  for (int k = 0; k < a.K; ++k) {
    const float* c = a.centers + (size_t)k * F;
    float s = 0.f;
    for (int f = 0; f < F; ++f) {
      const float x = feat[f * TB + tid];
      if (x != x) continue;
      const float v = compare(a.cfun[f], x - c[f], a.scales[f]);
      const float w = a.weights[f];
      if (METRIC == M_SQEUCLID || METRIC == M_EUCLID) s = fmaf(w * v, v, s);
      else if (METRIC == M_CITY) s = fmaf(w, v, s);
      else if (METRIC == M_CHEBY) s = fmaxf(s, w * v);
      else s = fmaf(w, __powf(v, a.p), s);
    }
    if (METRIC != M_CHEBY) s *= adj;
    if (METRIC == M_EUCLID) s = sqrtf(s);
    else if (METRIC == M_MINKOWSKI) s = __powf(s, 1.0f / a.p);
    const bool better = a.similarity ? (s > best) : (s < best);
    if (better) { best = s; best_k = k; }
  }
  bool ok = (bad[tid] == 0) && (qpresent > 0.f) && (best_k >= 0);
  float sc = ok ? a.table[best_k] : __builtin_nanf("");
  ok = ok && (sc == sc);
  a.score[row] = ok ? sc : __builtin_nanf("");
  a.valid[row] = ok ? 1 : 0;
  if (a.label) a.label[row] = best_k;
  if (a.affinity) a.affinity[row] = best;
}

}  // namespace

PMML_API int pmml_cluster_args_size() { return (int)sizeof(ClusterArgs); }

PMML_API int pmml_cluster_launch(hipStream_t stream, const ClusterArgs* args) {
  const ClusterArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_feat > 128) return -4;
  const size_t lds = (size_t)a.n_feat * TB * 4 + TB * 4;
  dim3 grid((a.n_rows + TB - 1) / TB);
  switch (a.metric) {
    case M_SQEUCLID: hipLaunchKernelGGL(cluster_kernel<M_SQEUCLID>, grid, dim3(TB), lds, stream, a); break;
    case M_EUCLID: hipLaunchKernelGGL(cluster_kernel<M_EUCLID>, grid, dim3(TB), lds, stream, a); break;
    case M_CITY: hipLaunchKernelGGL(cluster_kernel<M_CITY>, grid, dim3(TB), lds, stream, a); break;
    case M_CHEBY: hipLaunchKernelGGL(cluster_kernel<M_CHEBY>, grid, dim3(TB), lds, stream, a); break;
    case M_MINKOWSKI: hipLaunchKernelGGL(cluster_kernel<M_MINKOWSKI>, grid, dim3(TB), lds, stream, a); break;
    default: return -6;
  }
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
