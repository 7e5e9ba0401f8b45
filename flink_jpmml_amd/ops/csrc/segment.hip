// MiningModel segmentations the fused ensemble kernels refuse: ONE kernel for the segment
// predicates and the aggregation over the K segment outputs (runtime/segmented.py).
//
// The reference evaluates any Segmentation JPMML supports (`S/api/PmmlModel.scala:159-160`). Each
// segment model runs as its own plan and writes its scores (and, for probability methods, its
// class probabilities) into [K][n] buffers; this kernel then does, per row, what
// MiningEvaluator._select / _regress / _classify do in the float64 oracle (models/mining.py):
//
//   * segment predicates: postfix programs over PMML's three-valued logic (TRUE / FALSE / UNKNOWN,
//     2 bits per stack entry), fp64 comparisons of the fp32 inputs (the oracle compares float64);
//   * selectFirst, sum / average / weightedAverage / max / min / median / weightedMedian
//     (regression, fp64), majority / weighted-majority votes and average / weightedAverage / max /
//     median of the probability vectors (classification), missingPredictionTreatment;
//   * the regression Target stage (clip, rescale, castInteger, defaultValue) and the label table.
//
// One lane per row, every per-row array in registers / scratch: the <64, 64> instantiation for
// K, C <= 64 segments / classes, the <256, 256> one (bitmask words, scratch arrays) up to 256.

#include "common.h"

namespace {

constexpr int SEG_TB = 256;
constexpr int SEG_WIDE = 256;  // segments / classes of the wide instantiation

enum : int {
  SP_END = 0, SP_TRUE, SP_FALSE, SP_CMP, SP_ISMISS, SP_NOTMISS, SP_SET, SP_AND, SP_OR, SP_XOR, SP_SURR,
};
enum : int { CMP_EQ = 0, CMP_NE, CMP_LT, CMP_LE, CMP_GT, CMP_GE };
enum : int {
  SM_SELECT = 0, SM_SUM, SM_AVG, SM_WAVG, SM_MAX, SM_MIN, SM_MEDIAN, SM_WMEDIAN,
  SM_VOTE, SM_WVOTE, SM_PAVG, SM_PWAVG, SM_PMAX, SM_PMEDIAN,
};
constexpr uint32_t SV_F = 0u, SV_T = 1u, SV_U = 2u;

struct SegArgs {
  const float* X;          // [n, ldx] prepared (augmented) input
  int n_rows, ldx;
  const float* S;          // [K][n] segment scores (class index for classification segments)
  const uint8_t* V;        // [K][n] segment validity
  const float* P;          // probability methods: segment i at P + coff[i] * n, [n][C_i]
  const long long* coff;   // [K + 1] prefix of the segments' probability widths
  const int4* prog;        // {op | arg << 8, col / n, pool offset, count}
  const double* pool;      // comparison values / set members
  const int* pc;           // [K] program start of each segment's predicate
  const double* weights;   // [K]
  const int* remap;        // [K][SEG_MAXC + 1] segment class -> ensemble class (-1 none)
  const float* table;      // [C] label table (classification)
  int K, C, method, classification;
  int skip;                // missingPredictionTreatment == skipSegment
  int tgt;                 // regression Target flags (TGT_*), 0 = none
  double lo, hi, ta, tb, dflt;
  float* score;
  uint8_t* valid;
  float* score2;           // optional device mirrors
  uint8_t* valid2;
  int remap_stride, pad;   // remap row length: (max classes of the instantiation) + 1
};

__device__ uint32_t seg_predicate(const SegArgs& a, int pc, const float* xrow) {
  uint64_t st = 0;
  for (;; ++pc) {
    const int4 in = a.prog[pc];
    const int op = in.x & 0xFF;
    const int arg = in.x >> 8;
    uint32_t v;
    if (op == SP_END) return (uint32_t)(st & 3u);
    if (op >= SP_AND) {
      bool any_t = false, any_f = false, any_u = false;
      uint32_t par = 0u, sur = SV_U;
      for (int i = 0; i < in.y; ++i) {
        const uint32_t e = (uint32_t)(st & 3u);
        st >>= 2;
        any_t |= e == SV_T;
        any_f |= e == SV_F;
        any_u |= e == SV_U;
        par ^= (e == SV_T) ? 1u : 0u;
        if (e != SV_U) sur = e;  // popped last-first: ends at the first child with a known value
      }
      if (op == SP_AND) v = any_f ? SV_F : (any_u ? SV_U : SV_T);
      else if (op == SP_OR) v = any_t ? SV_T : (any_u ? SV_U : SV_F);
      else if (op == SP_XOR) v = any_u ? SV_U : par;
      else v = sur;
    } else if (op == SP_TRUE) {
      v = SV_T;
    } else if (op == SP_FALSE) {
      v = SV_F;
    } else {
      const double x = (double)xrow[in.y];
      const bool miss = x != x;
      if (op == SP_ISMISS) {
        v = miss ? SV_T : SV_F;
      } else if (op == SP_NOTMISS) {
        v = miss ? SV_F : SV_T;
      } else if (miss) {
        v = SV_U;
      } else if (op == SP_CMP) {
        const double t = a.pool[in.z];
        bool r;
        switch (arg) {
          case CMP_EQ: r = x == t; break;
          case CMP_NE: r = x != t; break;
          case CMP_LT: r = x < t; break;
          case CMP_LE: r = x <= t; break;
          case CMP_GT: r = x > t; break;
          default: r = x >= t; break;
        }
        v = r ? SV_T : SV_F;
      } else {  // SP_SET: arg 1 = isIn, 0 = isNotIn
        bool inside = false;
        for (int i = 0; i < in.w; ++i) inside = inside || (a.pool[in.z + i] == x);
        v = (inside == (arg != 0)) ? SV_T : SV_F;
      }
    }
    st = (st << 2) | v;
  }
}

__device__ __forceinline__ double seg_target(const SegArgs& a, double v) {
  if ((a.tgt & TGT_LO) && v < a.lo) v = a.lo;
  if ((a.tgt & TGT_HI) && v > a.hi) v = a.hi;
  v = v * a.ta + a.tb;
  switch ((a.tgt >> TGT_CAST_SHIFT) & 3) {
    case CAST_ROUND: v = floor(v + 0.5); break;
    case CAST_CEIL: v = ceil(v); break;
    case CAST_FLOOR: v = floor(v); break;
    default: break;
  }
  return v;
}

// numpy-style median of the first m values of w (sorted in place): mean of the two middle values
__device__ double seg_median(double* w, int m) {
  for (int i = 1; i < m; ++i) {  // insertion sort, m <= 256
    const double x = w[i];
    int j = i - 1;
    while (j >= 0 && w[j] > x) {
      w[j + 1] = w[j];
      --j;
    }
    w[j + 1] = x;
  }
  if (m == 0) return __builtin_nan("");
  return (w[(m - 1) / 2] + w[m / 2]) * 0.5;
}

template <int MK>
struct SegMask {  // one bit per segment, MK / 64 words
  uint64_t w[MK / 64];
  __device__ __forceinline__ SegMask() {
#pragma unroll
    for (int i = 0; i < MK / 64; ++i) w[i] = 0ull;
  }
  __device__ __forceinline__ void set(int k) { w[k >> 6] |= 1ull << (k & 63); }
  __device__ __forceinline__ bool get(int k) const { return (w[k >> 6] >> (k & 63)) & 1ull; }
  __device__ __forceinline__ bool any() const {
    uint64_t o = 0ull;
#pragma unroll
    for (int i = 0; i < MK / 64; ++i) o |= w[i];
    return o != 0ull;
  }
  __device__ __forceinline__ int first() const {  // lowest set bit, -1 if none
#pragma unroll
    for (int i = 0; i < MK / 64; ++i)
      if (w[i]) return 64 * i + __ffsll((unsigned long long)w[i]) - 1;
    return -1;
  }
};

template <int MK, int MC>
__global__ __launch_bounds__(SEG_TB) void segment_reduce_kernel(SegArgs a) {
  const int row = blockIdx.x * SEG_TB + threadIdx.x;
  if (row >= a.n_rows) return;
  const size_t n = (size_t)a.n_rows;
  const float* xrow = a.X + (size_t)row * a.ldx;
  const int K = a.K;
  const int RS = a.remap_stride;
  SegMask<MK> tmask, okmask, use;
  bool anymiss = false;
  for (int i = 0; i < K; ++i) {
    const bool t = seg_predicate(a, a.pc[i], xrow) == SV_T;
    const float s = a.S[i * n + row];
    const bool okk = a.V[i * n + row] && s == s;
    if (t) tmask.set(i);
    if (okk) okmask.set(i);
    if (t && okk) use.set(i);
    anymiss = anymiss || (t && !okk);
  }
  double out = __builtin_nan("");
  bool ok = false;
  const int m = a.method;
  if (m == SM_SELECT) {
    const int f = tmask.first();
    if (f >= 0) {
      ok = okmask.get(f);
      const float s = a.S[f * n + row];
      if (a.classification) {
        const int lab = s == s ? a.remap[f * RS + (int)s] : -1;
        ok = ok && lab >= 0;
        out = lab >= 0 ? (double)a.table[lab] : __builtin_nan("");
        ok = ok && out == out;
      } else {
        out = (double)s;
        ok = ok && isfinite(out);
        if (a.tgt) out = seg_target(a, out);
      }
    } else if (!a.classification && a.tgt) {
      out = seg_target(a, out);
    }
    if (!a.classification && (a.tgt & TGT_DEFAULT) && !ok) {
      out = a.dflt;
      ok = true;
    }
  } else if (!a.classification) {
    double w[MK];
    int cnt = 0;
    double acc = 0.0, wsum = 0.0;
    double best = m == SM_MAX ? -__builtin_inf() : __builtin_inf();
    for (int i = 0; i < K; ++i) {
      if (!use.get(i)) continue;
      const double s = (double)a.S[i * n + row];
      ++cnt;
      if (m == SM_SUM || m == SM_AVG) acc += s;
      else if (m == SM_WAVG) {
        acc += s * a.weights[i];
        wsum += a.weights[i];
      } else if (m == SM_MAX) best = s > best ? s : best;
      else if (m == SM_MIN) best = s < best ? s : best;
      else w[cnt - 1] = s;
    }
    if (m == SM_SUM) out = acc;
    else if (m == SM_AVG) out = acc / (double)cnt;
    else if (m == SM_WAVG) out = acc / wsum;
    else if (m == SM_MAX || m == SM_MIN) out = best;
    else if (m == SM_MEDIAN) out = seg_median(w, cnt);
    else {  // weightedMedian: first value (stable ascending order) whose cumulative weight reaches half
      int idx[MK];
      int c2 = 0;
      double total = 0.0;
      for (int i = 0; i < K; ++i)
        if (use.get(i)) {
          idx[c2++] = i;
          total += a.weights[i];
        }
      for (int p = 1; p < c2; ++p) {  // stable insertion sort by value
        const int x = idx[p];
        const double xv = (double)a.S[x * n + row];
        int q = p - 1;
        while (q >= 0 && (double)a.S[idx[q] * n + row] > xv) {
          idx[q + 1] = idx[q];
          --q;
        }
        idx[q + 1] = x;
      }
      double cw = 0.0;
      int below = 0;
      for (int p = 0; p < c2; ++p) {
        cw += a.weights[idx[p]];
        if (cw < 0.5 * total) ++below;
      }
      out = c2 ? (double)a.S[idx[min(below, c2 - 1)] * n + row] : __builtin_inf();
    }
    ok = cnt > 0 && (a.skip || !anymiss) && isfinite(out);
    if (a.tgt) {
      out = seg_target(a, out);
      if ((a.tgt & TGT_DEFAULT) && !ok) {
        out = a.dflt;
        ok = true;
      }
    }
  } else {
    const int C = a.C;
    double acc[MC];
    for (int c = 0; c < C; ++c) acc[c] = 0.0;
    if (m == SM_VOTE || m == SM_WVOTE) {
      for (int i = 0; i < K; ++i) {
        if (!use.get(i)) continue;
        const int lab = a.remap[i * RS + (int)a.S[i * n + row]];
        if (lab >= 0) acc[lab] += m == SM_WVOTE ? a.weights[i] : 1.0;
      }
    } else if (m == SM_PAVG || m == SM_PWAVG) {
      double wu = 0.0;
      for (int i = 0; i < K; ++i) {
        if (!use.get(i)) continue;
        const double wi = m == SM_PWAVG ? a.weights[i] : 1.0;
        wu += wi;
        const int Ci = (int)(a.coff[i + 1] - a.coff[i]);
        const float* pr = a.P + a.coff[i] * n + (size_t)row * Ci;
        for (int j = 0; j < Ci; ++j) {
          const int c = a.remap[i * RS + j];
          const float p = pr[j];
          if (c >= 0) acc[c] += (p == p ? (double)p : 0.0) * wi;
        }
      }
      for (int c = 0; c < C; ++c) acc[c] /= wu;
    } else if (m == SM_PMAX) {
      for (int i = 0; i < K; ++i) {
        if (!use.get(i)) continue;
        const int Ci = (int)(a.coff[i + 1] - a.coff[i]);
        const float* pr = a.P + a.coff[i] * n + (size_t)row * Ci;
        for (int j = 0; j < Ci; ++j) {
          const int c = a.remap[i * RS + j];
          const float p = pr[j];
          if (c >= 0) {
            const double v = p == p ? (double)p : 0.0;
            acc[c] = v > acc[c] ? v : acc[c];
          }
        }
      }
    } else {  // SM_PMEDIAN: per class, the median over the using segments (NaN entries dropped)
      for (int c = 0; c < C; ++c) {
        double w[MK];
        int cnt = 0;
        for (int i = 0; i < K; ++i) {
          if (!use.get(i)) continue;
          const int Ci = (int)(a.coff[i + 1] - a.coff[i]);
          const float* pr = a.P + a.coff[i] * n + (size_t)row * Ci;
          for (int j = 0; j < Ci; ++j)
            if (a.remap[i * RS + j] == c && pr[j] == pr[j]) w[cnt++] = (double)pr[j];
        }
        acc[c] = seg_median(w, cnt);
      }
    }
    int lab = 0;
    double bv = -__builtin_inf();
    for (int c = 0; c < C; ++c) {
      const double v = acc[c] == acc[c] ? acc[c] : -1.0;  // nan_to_num(nan=-1) before argmax
      if (v > bv) {
        bv = v;
        lab = c;
      }
    }
    ok = use.any() && (a.skip || !anymiss);
    out = (double)a.table[lab];
    ok = ok && out == out;
  }
  const float s = ok ? (float)out : __builtin_nanf("");
  a.score[row] = s;
  a.valid[row] = ok ? 1 : 0;
  if (a.score2) a.score2[row] = s;
  if (a.valid2) a.valid2[row] = ok ? 1 : 0;
}

}  // namespace

PMML_API int pmml_segment_args_size() { return (int)sizeof(SegArgs); }

// remap_stride selects the instantiation: 65 -> <64, 64> (K, C <= 64), 257 -> <256, 256>.
PMML_API int pmml_segment_reduce(hipStream_t stream, const SegArgs* args) {
  const SegArgs& a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.method < SM_SELECT || a.method > SM_PMEDIAN || a.K < 1) return -2;
  const dim3 grid((a.n_rows + SEG_TB - 1) / SEG_TB);
  if (a.remap_stride == 64 + 1) {
    if (a.K > 64 || a.C > 64) return -2;
    hipLaunchKernelGGL((segment_reduce_kernel<64, 64>), grid, dim3(SEG_TB), 0, stream, a);
  } else if (a.remap_stride == SEG_WIDE + 1) {
    if (a.K > SEG_WIDE || a.C > SEG_WIDE) return -2;
    hipLaunchKernelGGL((segment_reduce_kernel<SEG_WIDE, SEG_WIDE>), grid, dim3(SEG_TB), 0, stream, a);
  } else {
    return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
