// NearestNeighborModel with k > 1: per-row distances to the training instances, a register top-k,
// then the PMML aggregation (majority / weighted majority vote, average / median / weighted average).
//
// Same comparison machinery as the clustering kernels (cluster.hip): metric x compareFunction x
// fieldWeight, missing inputs skipped. Two observations keep the inner loop lean:
//   * the missing-value rescale Σq/Σq_present, the final sqrt (euclidean) and the 1/p power
//     (minkowski) are monotone per row, so the top-k is selected on the raw sums and only the k
//     winners are finished;
//   * the top-k list is a fixed-size register array (KMAX in {8, 32}, runtime k <= KMAX) kept
//     sorted by (key, instance index) — a candidate that does not beat the current k-th key costs
//     one compare; a winner bubbles in with an unrolled, predicated compare-exchange chain (no
//     dynamic register indexing, so nothing spills to scratch).
//
// VALU path: instances are read with wave-uniform addresses (scalar loads, broadcast), rows are
// staged in LDS [F][256]. MFMA path (squared / plain euclidean, absDiff, distance measure, many
// instances): Σ_f w_f (x_f - c_if)² = ‖x‖²_w − 2 x·(w∘c_i) + ‖c_i‖²_w with the cross term on the
// matrix cores (v_mfma_f32_32x32x2_f32, instances on M, rows on N). Each lane then holds 16
// instance distances of one row per 32-instance tile and feeds them into its own top-k; the two
// half-waves' lists of a row are merged through lane^32 shuffles. Rows with a missing value redo
// the exact form in the same wave.
#include "common.h"
#include "epilogue.h"

namespace {

constexpr int TB = 256;

enum : int { M_SQEUCLID = 0, M_EUCLID = 1, M_CITY = 2, M_CHEBY = 3, M_MINKOWSKI = 4 };
enum : int { CF_ABSDIFF = 0, CF_GAUSS = 1, CF_DELTA = 2, CF_EQUAL = 3 };
enum : int { AGG_MAJORITY = 0, AGG_WMAJORITY = 1, AGG_AVERAGE = 2, AGG_MEDIAN = 3, AGG_WAVERAGE = 4 };

struct KnnArgs {
  const float* X;
  int n_rows, n_feat, ldx, n_inst;
  const FieldPrep* prep;
  const float* inst;        // [N][F] training instances
  const float* weights;     // [F]
  const float* scales;      // [F] gaussSim similarity scale
  const float* qweights;    // [F] missing-value weights
  const int* cfun;          // [F] compare function codes
  const float* inst_value;  // [N] regression target of each instance
  const int* inst_class;    // [N] class index of each instance (classification)
  const float* class_table; // [C] class label parsed as double (NaN = not numeric)
  int metric, similarity;   // similarity: larger is nearer
  float p;                  // minkowski p
  int k;                    // neighbours (<= KMAX, <= n_inst)
  int agg;                  // AGG_*
  float threshold;          // weighting: 1 / (d + threshold)
  Epilogue epi;             // Target stage of a regression value (tgt flags only)
  float* score;
  uint8_t* valid;
};

__device__ __forceinline__ float compare(int cf, float d, float s) {
  switch (cf) {
    case CF_GAUSS: return __expf(-0.69314718056f * d * d / (s * s));
    case CF_DELTA: return d != 0.f ? 1.f : 0.f;
    case CF_EQUAL: return d == 0.f ? 1.f : 0.f;
    default: return fabsf(d);
  }
}

// Insert (ck, ci) into the sorted list key/id of length k (ties: lower instance index first).
template <int KMAX>
__device__ __forceinline__ void topk_insert(float (&key)[KMAX], int (&id)[KMAX], int k, float ck, int ci) {
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    if (j < k) {
      const bool sw = ck < key[j] || (ck == key[j] && ci < id[j]);
      const float tk = key[j];
      const int ti = id[j];
      key[j] = sw ? ck : tk;
      id[j] = sw ? ci : ti;
      ck = sw ? tk : ck;
      ci = sw ? ti : ci;
    }
  }
}

// Last (k-th) entry of the sorted list, written as a running max over the live prefix: an
// `index == k - 1` select chain is folded by LLVM into a dynamic array index (-> scratch memory).
template <int KMAX>
__device__ __forceinline__ float kth(const float (&key)[KMAX], int k) {
  float w = -__builtin_inff();
#pragma unroll
  for (int j = 0; j < KMAX; ++j) w = (j < k) ? fmaxf(w, key[j]) : w;
  return w;
}

// (key, id) of the k-th entry under the list's lexicographic order.
template <int KMAX>
__device__ __forceinline__ void kth_pair(const float (&key)[KMAX], const int (&id)[KMAX], int k, float* wk,
                                         int* wi) {
  float w = -__builtin_inff();
  int wid = -1;
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    const bool later = j < k && (key[j] > w || (key[j] == w && id[j] > wid));
    w = later ? key[j] : w;
    wid = later ? id[j] : wid;
  }
  *wk = w;
  *wi = wid;
}

// Raw sum of one instance (before rescale / root); `feat` points at the row's LDS column.
template <int METRIC>
__device__ __forceinline__ float raw_distance(const KnnArgs& a, const float* feat, int stride, const float* c) {
  float s = 0.f;
  for (int f = 0; f < a.n_feat; ++f) {
    const float x = feat[f * stride];
    if (x != x) continue;
    const float v = compare(a.cfun[f], x - c[f], a.scales[f]);
    const float w = a.weights[f];
    if (METRIC == M_SQEUCLID || METRIC == M_EUCLID) s = fmaf(w * v, v, s);
    else if (METRIC == M_CITY) s = fmaf(w, v, s);
    else if (METRIC == M_CHEBY) s = fmaxf(s, w * v);
    else s = fmaf(w, __powf(v, a.p), s);
  }
  return s;
}

// Finished distance of a raw sum (the oracle's value: rescaled, rooted; similarity keeps its sign).
__device__ __forceinline__ float finish_distance(int metric, float s, float adj, float p) {
  if (metric != M_CHEBY) s *= adj;
  if (metric == M_EUCLID) s = sqrtf(fmaxf(s, 0.f));
  else if (metric == M_MINKOWSKI) s = __powf(s, 1.0f / p);
  return s;
}

// Aggregate the k nearest (sorted by key) into the row's score / validity.
template <int KMAX>
__device__ __forceinline__ void knn_finish(const KnnArgs& a, const float (&key)[KMAX], const int (&id)[KMAX],
                                           float adj, bool ok, int row) {
  const int k = a.k;
  float d[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    // key is the raw sum (distance) or minus the raw sum (similarity)
    const float raw = a.similarity ? -key[j] : key[j];
    d[j] = finish_distance(a.metric, raw, adj, a.p);
    if (j < k) ok = ok && __builtin_isfinite(d[j]) && id[j] >= 0 && id[j] < a.n_inst;
  }
  float s = __builtin_nanf("");
  if (ok) {
    if (a.agg == AGG_MAJORITY || a.agg == AGG_WMAJORITY) {
      int cls[KMAX];
      float w[KMAX];
      bool any_exact = false;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        cls[j] = j < k ? a.inst_class[id[j]] : -1;
        w[j] = a.agg == AGG_WMAJORITY ? 1.0f / (fabsf(d[j]) + a.threshold) : 1.0f;
        any_exact = any_exact || (j < k && !__builtin_isfinite(w[j]));
      }
      // an exact match (weight 1 / (0 + threshold 0)) dominates: the weighted vote's limit is the
      // vote of the exact neighbours alone, each counting once (models/knn.py, same rule)
#pragma unroll
      for (int j = 0; j < KMAX; ++j)
        if (any_exact) w[j] = __builtin_isfinite(w[j]) ? 0.f : 1.f;
      // votes of neighbour j's class, summed in rank order; the first rank reaching the maximum
      // names the winner (= the tied class whose best member ranks first)
      float best = -1.f;
      int best_c = -1;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        if (j < k) {
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < KMAX; ++i)
            if (i < k && cls[i] == cls[j]) v += w[i];
          if (v > best) {
            best = v;
            best_c = cls[j];
          }
        }
      }
      s = best_c >= 0 ? a.class_table[best_c] : __builtin_nanf("");
      ok = s == s;
    } else {
      float y[KMAX];
#pragma unroll
      for (int j = 0; j < KMAX; ++j) y[j] = j < k ? a.inst_value[id[j]] : __builtin_inff();
      if (a.agg == AGG_AVERAGE) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
          if (j < k) acc += y[j];
        s = acc / (float)k;
      } else if (a.agg == AGG_WAVERAGE) {
        float num = 0.f, den = 0.f, num0 = 0.f, den0 = 0.f;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if (j < k) {
            const float w = 1.0f / (fabsf(d[j]) + a.threshold);
            if (__builtin_isfinite(w)) {
              num = fmaf(w, y[j], num);
              den += w;
            } else {  // exact match: see the vote above
              num0 += y[j];
              den0 += 1.f;
            }
          }
        }
        s = den0 > 0.f ? num0 / den0 : num / den;
      } else {  // median: odd-even transposition sort of the k values (+inf padding sorts last)
#pragma unroll
        for (int pass = 0; pass < KMAX; ++pass) {
#pragma unroll
          for (int j = pass & 1; j + 1 < KMAX; j += 2) {
            const float lo = fminf(y[j], y[j + 1]), hi = fmaxf(y[j], y[j + 1]);
            y[j] = lo;
            y[j + 1] = hi;
          }
        }
        // sorted ascending: the (k-1)/2-th and k/2-th values are maxima of prefixes (no dynamic index)
        float m0 = -__builtin_inff(), m1 = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          m0 = j <= (k - 1) / 2 ? fmaxf(m0, y[j]) : m0;
          m1 = j <= k / 2 ? fmaxf(m1, y[j]) : m1;
        }
        s = (k & 1) ? m0 : 0.5f * (m0 + m1);
      }
      ok = __builtin_isfinite(s);
    }
  }
  if (a.agg >= AGG_AVERAGE && a.epi.tgt) {
    if (ok) s = apply_target(a.epi, s);
    if (!ok && (a.epi.tgt & TGT_DEFAULT)) {
      s = a.epi.dflt;
      ok = true;
    }
  }
  a.score[row] = ok ? s : __builtin_nanf("");
  a.valid[row] = ok ? 1 : 0;
}

__device__ __forceinline__ float row_adjust(const KnnArgs& a, const float* feat, int stride, float* qpresent_out) {
  float qsum = 0.f, qpresent = 0.f;
  for (int f = 0; f < a.n_feat; ++f) {
    const float q = a.qweights[f];
    qsum += q;
    if (feat[f * stride] == feat[f * stride]) qpresent += q;
  }
  *qpresent_out = qpresent;
  return qpresent > 0.f ? qsum / qpresent : __builtin_nanf("");
}

template <int METRIC, int KMAX>
__global__ __launch_bounds__(TB) void knn_kernel(KnnArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  const int row0 = blockIdx.x * TB;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  const int tid = threadIdx.x;
  const int row = row0 + tid;
  if (row >= a.n_rows) return;
  const float* fr = feat + tid;
  float qpresent;
  const float adj = row_adjust(a, fr, TB, &qpresent);
  float key[KMAX];
  int id[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    key[j] = __builtin_inff();
    id[j] = 0x7fffffff;
  }
  // instances arrive in increasing index, so a tie with the k-th entry never displaces it
  float worst = __builtin_inff();
  for (int i = 0; i < a.n_inst; ++i) {
    const float s = raw_distance<METRIC>(a, fr, TB, a.inst + (size_t)i * a.n_feat);
    const float ck = a.similarity ? -s : s;
    if (ck < worst) {
      topk_insert<KMAX>(key, id, a.k, ck, i);
      worst = kth<KMAX>(key, a.k);
    }
  }
  knn_finish<KMAX>(a, key, id, adj, bad[tid] == 0 && qpresent > 0.f, row);
}

typedef float f32x16_t __attribute__((ext_vector_type(16)));

// One row of the MFMA kernel: keep the expansion's top-k, or redo it exactly for a row with a
// missing value (skip missing fields, rescale by Σq / Σq_present).
template <int KMAX>
__device__ __forceinline__ void mfma_row_finish(const KnnArgs& a, const float* feat, const int* bad,
                                                float (&key)[KMAX], int (&id)[KMAX], bool missing, int rl,
                                                int row0) {
  const int row = row0 + rl;
  if (row >= a.n_rows) return;
  float qpresent = 1.f, adj = 1.f;
  if (missing) {
    adj = row_adjust(a, feat + rl, TB, &qpresent);
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      key[j] = __builtin_inff();
      id[j] = 0x7fffffff;
    }
    float worst = __builtin_inff();
    for (int i = 0; i < a.n_inst; ++i) {
      const float s = raw_distance<M_SQEUCLID>(a, feat + rl, TB, a.inst + (size_t)i * a.n_feat);
      if (s < worst) {
        topk_insert<KMAX>(key, id, a.k, s, i);
        worst = kth<KMAX>(key, a.k);
      }
    }
  }
  knn_finish<KMAX>(a, key, id, adj, bad[rl] == 0 && qpresent > 0.f, row);
}

template <int KMAX>
__global__ __launch_bounds__(TB) void knn_mfma_kernel(KnnArgs a, const float* __restrict__ wc,
                                                      const float* __restrict__ cc, int Np, int Fp) {
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
  const int k = a.k;
  const int rb = wave * 64 + (lane & 31);  // this lane's two rows: rb, rb + 32
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
  float key0[KMAX], key1[KMAX];
  int id0[KMAX], id1[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    key0[j] = key1[j] = __builtin_inff();
    id0[j] = id1[j] = 0x7fffffff;
  }
  float worst0 = __builtin_inff(), worst1 = __builtin_inff();
  for (int i0 = 0; i0 < Np; i0 += 32) {
    f32x16_t acc0 = {}, acc1 = {};
    const float* wrow = wc + (size_t)(i0 + (lane & 31)) * Fp;
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
    for (int r = 0; r < 16; ++r) {  // D[instance (r&3)+8(r>>2)+4*half][row lane&31]
      const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * half;
      const float ci = cc[i];
      const float d0 = fmaxf(fmaf(-2.f, acc0[r], xx[0]) + ci, 0.f);
      const float d1 = fmaxf(fmaf(-2.f, acc1[r], xx[1]) + ci, 0.f);
      // within a lane instances arrive in increasing index: strict < keeps the lower index on ties
      if (d0 < worst0) {
        topk_insert<KMAX>(key0, id0, k, d0, i);
        worst0 = kth<KMAX>(key0, k);
      }
      if (d1 < worst1) {
        topk_insert<KMAX>(key1, id1, k, d1, i);
        worst1 = kth<KMAX>(key1, k);
      }
    }
  }
  // merge the partner half-wave's lists (same rows, the other instances of every tile)
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    const float o0 = __shfl_xor(key0[j], 32);
    const int p0 = __shfl_xor(id0[j], 32);
    const float o1 = __shfl_xor(key1[j], 32);
    const int p1 = __shfl_xor(id1[j], 32);
    if (half == 0 && j < k) {
      float w0, w1;
      int i0, i1;
      kth_pair<KMAX>(key0, id0, k, &w0, &i0);
      kth_pair<KMAX>(key1, id1, k, &w1, &i1);
      if (o0 < w0 || (o0 == w0 && p0 < i0)) topk_insert<KMAX>(key0, id0, k, o0, p0);
      if (o1 < w1 || (o1 == w1 && p1 < i1)) topk_insert<KMAX>(key1, id1, k, o1, p1);
    }
  }
  if (half != 0) return;
  mfma_row_finish<KMAX>(a, feat, bad, key0, id0, missing[0], rb, row0);
  mfma_row_finish<KMAX>(a, feat, bad, key1, id1, missing[1], rb + 32, row0);
}

template <int KMAX>
int launch_valu(hipStream_t stream, const KnnArgs& a, dim3 grid, size_t lds) {
  switch (a.metric) {
    case M_SQEUCLID: hipLaunchKernelGGL((knn_kernel<M_SQEUCLID, KMAX>), grid, dim3(TB), lds, stream, a); break;
    case M_EUCLID: hipLaunchKernelGGL((knn_kernel<M_EUCLID, KMAX>), grid, dim3(TB), lds, stream, a); break;
    case M_CITY: hipLaunchKernelGGL((knn_kernel<M_CITY, KMAX>), grid, dim3(TB), lds, stream, a); break;
    case M_CHEBY: hipLaunchKernelGGL((knn_kernel<M_CHEBY, KMAX>), grid, dim3(TB), lds, stream, a); break;
    case M_MINKOWSKI: hipLaunchKernelGGL((knn_kernel<M_MINKOWSKI, KMAX>), grid, dim3(TB), lds, stream, a); break;
    default: return -6;
  }
  return 0;
}
}  // namespace

PMML_API int pmml_knn_args_size() { return (int)sizeof(KnnArgs); }

// wc / cc: MFMA operands (see ClusterPlan.mfma_operands: wc [Np][Fp] = w∘c zero padded, cc [Np] =
// Σ_f w_f c_f² with +inf on padded instances) or null for the VALU kernel.
PMML_API int pmml_knn_launch(hipStream_t stream, const KnnArgs* args, const float* wc, const float* cc, int Np,
                             int Fp) {
  const KnnArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_feat > 128 || a.k < 1 || a.k > 32 || a.k > a.n_inst || a.agg < 0 || a.agg > AGG_WAVERAGE) return -4;
  const size_t lds = (size_t)a.n_feat * TB * 4 + TB * 4;
  dim3 grid((a.n_rows + TB - 1) / TB);
  int rc = 0;
  if (wc) {
    if ((Np & 31) || (Fp & 1) || Fp < a.n_feat || Np < a.n_inst || a.similarity) return -4;
    if (a.metric != M_SQEUCLID && a.metric != M_EUCLID) return -6;
    if (a.k <= 8) hipLaunchKernelGGL(knn_mfma_kernel<8>, grid, dim3(TB), lds, stream, a, wc, cc, Np, Fp);
    else hipLaunchKernelGGL(knn_mfma_kernel<32>, grid, dim3(TB), lds, stream, a, wc, cc, Np, Fp);
  } else {
    rc = a.k <= 8 ? launch_valu<8>(stream, a, grid, lds) : launch_valu<32>(stream, a, grid, lds);
  }
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
