// Center-based ClusteringModel scoring: per-row distance to K centres + argmin/argmax.
//
// The centre table is tiny compared to the row stream and every lane of a wave needs the same
// centre element at the same time, so centres are read with wave-uniform addresses (scalar loads,
// broadcast to all lanes) — no LDS round trip. The row tile is staged in LDS [F][256] by the shared
// preparation/staging helper. Missing inputs are skipped and the sum rescaled by Σq / Σq_present
// (PMML ClusteringModel missing-value adjustment).
//
// MFMA path (squared / plain Euclidean, absDiff, many clusters): Σ_f w_f (x_f - c_kf)² =
// ‖x‖²_w − 2 x·(w∘c_k) + ‖c_k‖²_w, the cross term as a [K×F]·[F×rows] product on the matrix cores
// (exact-fp32 v_mfma_f32_32x32x2_f32: clusters on M, rows on N, so each lane ends up holding 16
// cluster distances of ONE row and the argmin is lane-local plus one lane^32 exchange). Rows with a
// missing value take the exact VALU path (skip + Σq/Σq_present rescale) in the same wave.
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


typedef float f32x16_t __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(TB) void cluster_mfma_kernel(ClusterArgs a, const float* __restrict__ wc,
                                                          const float* __restrict__ cc, int Kp, int Fp,
                                                          int euclid) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  const int row0 = blockIdx.x * TB;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int half = lane >> 5;
  const int F = a.n_feat;
  // the wave's 64 rows are two 32-row N tiles sharing every A (centre) operand load
  const int rb = wave * 64 + (lane & 31);
  float xx[2] = {0.f, 0.f};
  bool missing[2] = {false, false};
  for (int f = 0; f < F; ++f) {
    const float w = a.weights[f];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float x = feat[f * TB + rb + 32 * h];
      missing[h] = missing[h] || (x != x);
      xx[h] = fmaf(w * x, x, xx[h]);
    }
  }
  float bests[2] = {__builtin_inff(), __builtin_inff()};
  int bks[2] = {-1, -1};
  for (int k0 = 0; k0 < Kp; k0 += 32) {
    f32x16_t acc0 = {}, acc1 = {};
    const float* wrow = wc + (size_t)(k0 + (lane & 31)) * Fp;
    for (int f0 = 0; f0 < Fp; f0 += 2) {
      const int f = f0 + half;
      float x0 = f < F ? feat[f * TB + rb] : 0.f;
      float x1 = f < F ? feat[f * TB + rb + 32] : 0.f;
      x0 = (x0 != x0) ? 0.f : x0;  // rows with missing values are redone exactly below
      x1 = (x1 != x1) ? 0.f : x1;
      const float av = wrow[f];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, x0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, x1, acc1, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // D[cluster (i&3)+8(i>>2)+4*half][row lane&31]
      const int k = k0 + (i & 3) + 8 * (i >> 2) + 4 * half;
      const float ck = cc[k];
      const float d0 = fmaf(-2.f, acc0[i], xx[0]) + ck;
      const float d1 = fmaf(-2.f, acc1[i], xx[1]) + ck;
      if (d0 < bests[0]) { bests[0] = d0; bks[0] = k; }
      if (d1 < bests[1]) { bests[1] = d1; bks[1] = k; }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rl = rb + 32 * h;
    const bool miss = missing[h];
    float best = bests[h];
    int best_k = bks[h];
    const float ob = __shfl_xor(best, 32);
    const int okk = __shfl_xor(best_k, 32);
    if (ob < best || (ob == best && okk < best_k)) { best = ob; best_k = okk; }
    const int row = row0 + rl;
    if (half == 0 && row < a.n_rows) {
      bool ok = bad[rl] == 0;
      if (miss) {  // exact path: skip missing fields, rescale by Σq / Σq_present
        float qsum = 0.f, qpresent = 0.f;
        for (int f = 0; f < F; ++f) {
          qsum += a.qweights[f];
          if (feat[f * TB + rl] == feat[f * TB + rl]) qpresent += a.qweights[f];
        }
        const float adj = qpresent > 0.f ? qsum / qpresent : __builtin_nanf("");
        ok = ok && qpresent > 0.f;
        best = __builtin_inff();
        best_k = -1;
        for (int k = 0; k < a.K; ++k) {
          const float* c = a.centers + (size_t)k * F;
          float sacc = 0.f;
          for (int f = 0; f < F; ++f) {
            const float x = feat[f * TB + rl];
            if (x != x) continue;
            const float v = x - c[f];
            sacc = fmaf(a.weights[f] * v, v, sacc);
          }
          sacc *= adj;
          if (euclid) sacc = sqrtf(sacc);  // per cluster, as the VALU kernel (same tie order)
          if (sacc < best) { best = sacc; best_k = k; }
        }
      } else {
        best = fmaxf(best, 0.f);  // the expansion can dip below 0 by rounding at a centre
        if (euclid) best = sqrtf(best);
      }
      ok = ok && best_k >= 0;
      float sc = ok ? a.table[best_k] : __builtin_nanf("");
      ok = ok && (sc == sc);
      a.score[row] = ok ? sc : __builtin_nanf("");
      a.valid[row] = ok ? 1 : 0;
      if (a.label) a.label[row] = best_k;
      if (a.affinity) a.affinity[row] = best;
    }
  }
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

// MFMA path: wc [Kp][Fp] = w ∘ centres (zero padded), cc [Kp] = Σ_f w_f c_kf² (+inf on padding).
PMML_API int pmml_cluster_mfma_launch(hipStream_t stream, const ClusterArgs* args, const float* wc, const float* cc,
                                      int Kp, int Fp) {
  const ClusterArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_feat > 128 || (Kp & 31) || (Fp & 1) || Fp < a.n_feat || Kp < a.K) return -4;
  if (a.metric != M_SQEUCLID && a.metric != M_EUCLID) return -6;
  const size_t lds = (size_t)a.n_feat * TB * 4 + TB * 4;
  dim3 grid((a.n_rows + TB - 1) / TB);
  hipLaunchKernelGGL(cluster_mfma_kernel, grid, dim3(TB), lds, stream, a, wc, cc, Kp, Fp,
                     a.metric == M_EUCLID ? 1 : 0);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
