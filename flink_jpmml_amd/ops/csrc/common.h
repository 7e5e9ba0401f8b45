// Shared device helpers for the PMML scoring kernels (gfx950 / CDNA4, wave64).
//
// Every kernel consumes a row-major [rows, F] fp32 feature matrix (NaN = missing) that arrives
// straight from the host ingest buffer, and applies the MiningField / DataField preparation
// (missing replacement, validity interval + invalidValueTreatment, outliers) *while staging the
// tile into LDS* — there is no separate "prepare" pass over HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PMML_API extern "C" __attribute__((visibility("default")))

// FieldPrep.flags bits
enum : uint32_t {
  FP_HAS_MISSING_REPL = 1u << 0,   // NaN -> missing_repl
  FP_HAS_INTERVAL = 1u << 1,       // validity interval [lo, hi] (closure bits below)
  FP_LO_OPEN = 1u << 2,
  FP_HI_OPEN = 1u << 3,
  FP_INVALID_RETURN = 1u << 4,     // invalid -> whole row invalid (returnInvalid)
  FP_INVALID_AS_MISSING = 1u << 5, // invalid -> NaN (then missing replacement)
  FP_INVALID_AS_VALUE = 1u << 6,   // invalid -> invalid_repl
  FP_OUTLIER_AS_MISSING = 1u << 7, // x < out_lo | x > out_hi -> NaN
  FP_OUTLIER_AS_EXTREME = 1u << 8, // clamp to [out_lo, out_hi]
  FP_INTEGER = 1u << 9,            // non-integral value is invalid
  FP_CODE_RANGE = 1u << 10,        // categorical codes: valid iff 0 <= x < hi (string vocabularies)
  FP_ROW_INVALID = 1u << 11,       // field definition rejects every value (e.g. Interval on categorical)
  FP_MISSING_VALUE = 1u << 12,     // x == pad is a missing value (DataField <Value property="missing">)
  FP_VALUE_MASK = 1u << 13,        // numeric categories: valid iff x integral, lo <= x < lo + 64 and
                                   // bit (x - lo) of the 64-bit mask in the out_lo / out_hi words
  FP_VALUE_LIST = 1u << 14,        // DataField <Value property="missing"/"invalid"> lists: the pad word
                                   // holds {offset 16 | n_missing 8 | n_invalid 8}; the values are
                                   // fp32 words `offset` floats past this record (same buffer)
};

struct FieldPrep {
  uint32_t flags;
  float lo, hi;          // validity interval (or code range in hi)
  float missing_repl;
  float invalid_repl;
  float out_lo, out_hi;  // outlier bounds (continuous) / FP_VALUE_MASK bits 0-31, 32-63 (categorical)
  float pad;             // FP_MISSING_VALUE: the field's explicit missing value;
                         // FP_VALUE_LIST: {offset, n_missing, n_invalid} of its value lists
};
static_assert(sizeof(FieldPrep) == 32, "FieldPrep must stay 32 bytes (host mirror in ops/_lib.py)");

// Prepare one raw value. Sets *bad when the row must be rejected (returnInvalid).
__device__ __forceinline__ float prep_value(float x, const FieldPrep& p, bool* bad) {
  const uint32_t fl = p.flags;
  if (fl == 0u) return x;
  if (fl & FP_ROW_INVALID) { *bad = true; return x; }
  bool miss = (x != x) || ((fl & FP_MISSING_VALUE) && x == p.pad);
  const float* vlist = nullptr;
  uint32_t n_miss = 0u, n_inv = 0u;
  if (fl & FP_VALUE_LIST) {
    const uint32_t w = __float_as_uint(p.pad);
    vlist = reinterpret_cast<const float*>(&p) + (w & 0xFFFFu);
    n_miss = (w >> 16) & 0xFFu;
    n_inv = w >> 24;
    for (uint32_t i = 0; i < n_miss; ++i) miss = miss || (x == vlist[i]);
  }
  if (!miss) {
    bool invalid = false;
    for (uint32_t i = 0; i < n_inv; ++i) invalid = invalid || (x == vlist[n_miss + i]);
    if (fl & FP_HAS_INTERVAL) {
      bool lo_ok = (fl & FP_LO_OPEN) ? (x > p.lo) : (x >= p.lo);
      bool hi_ok = (fl & FP_HI_OPEN) ? (x < p.hi) : (x <= p.hi);
      invalid = !(lo_ok && hi_ok);
    }
    if (fl & FP_CODE_RANGE) invalid = invalid || !(x >= 0.f && x < p.hi);
    if (fl & FP_INTEGER) invalid = invalid || (floorf(x) != x);
    if (fl & FP_VALUE_MASK) {
      const float d = x - p.lo;
      bool in = d >= 0.f && d < 64.f && floorf(x) == x;
      if (in) {
        const int k = (int)d;
        in = (__float_as_uint(k < 32 ? p.out_lo : p.out_hi) >> (k & 31)) & 1u;
      }
      invalid = invalid || !in;
    }
    if (invalid) {
      if (fl & FP_INVALID_RETURN) *bad = true;
      else if (fl & FP_INVALID_AS_MISSING) miss = true;
      else if (fl & FP_INVALID_AS_VALUE) x = p.invalid_repl;
    } else {
      if (fl & FP_OUTLIER_AS_MISSING) miss = (x < p.out_lo) || (x > p.out_hi);
      else if (fl & FP_OUTLIER_AS_EXTREME) x = fminf(fmaxf(x, p.out_lo), p.out_hi);
    }
  }
  if (miss) x = (fl & FP_HAS_MISSING_REPL) ? p.missing_repl : __builtin_nanf("");
  return x;
}

__device__ __forceinline__ float fast_sigmoid(float z) { return 1.0f / (1.0f + __expf(-z)); }

// Epilogue modes shared by the model kernels.
enum : int {
  EPI_AFFINE = 0,       // score = link(a * acc0 + b)
  EPI_LOGISTIC2 = 1,    // p0 = link(a * acc0 + b), p1 = 1 - p0; label = p0 >= thr ? 0 : 1
  EPI_ARGMAX = 2,       // label = argmax_c acc_c (ties -> lowest c); probs = acc * a
  EPI_SOFTMAX = 3,      // probs = softmax(acc); label = argmax
  EPI_CUMULATIVE = 4,   // ordinal: cum_c = link(acc_c) (c < C-1), cum_{C-1} = 1; p_c = cum_c - cum_{c-1}
  EPI_LINKMAX = 5,      // > 2 tables, element-wise link: p_c = link(acc_c); label = first argmax; any
                        // non-finite p_c voids the row (models/regression.py finish)
};

struct Epilogue {
  int mode;
  int n_classes;        // accumulator slots C
  float a, b;           // affine
  float thr;            // EPI_LOGISTIC2 threshold
  int has_table;        // score = table[label] (class label parsed as double), NaN -> invalid
  const float* table;   // [C]
  int write_probs;      // also write probs[row, C]
  int link;             // LINK_* applied after the affine map (EPI_AFFINE, EPI_LOGISTIC2)
  float* score2;        // optional mirror outputs (e.g. device copy beside a zero-copy host sink)
  uint8_t* valid2;
  int tgt;              // TGT_* flags: PMML Target post-processing of an EPI_AFFINE value
  float dflt;           // TargetValue defaultValue (rows without a prediction)
  double lo, hi;        // Target min / max (clip, applied first)
  double ta, tb;        // Target rescaleFactor / rescaleConstant (after the clip)
                        // fp64 like the oracle: a clipped value rescales to the exact constant
                        // (fp32 -0.2 * 10 + 3 lands below 1.0 and floors to 0)
};

// Target post-processing (JPMML TargetUtil order): clip to [min, max], rescale, castInteger;
// a row without a prediction takes the default value when one is declared.
enum : int { TGT_ON = 1, TGT_LO = 2, TGT_HI = 4, TGT_DEFAULT = 8, TGT_CAST_SHIFT = 4 };
enum : int { CAST_NONE = 0, CAST_ROUND = 1, CAST_CEIL = 2, CAST_FLOOR = 3 };

enum : int { LINK_NONE = 0, LINK_LOGIT = 1, LINK_EXP = 2, LINK_PROBIT = 3, LINK_CLOGLOG = 4, LINK_LOGLOG = 5,
             LINK_CAUCHIT = 6 };

__device__ __forceinline__ float apply_link(int link, float y) {
  switch (link) {
    case LINK_LOGIT: return 1.0f / (1.0f + expf(-y));
    case LINK_EXP: return expf(y);
    case LINK_PROBIT: return 0.5f * erfcf(-y * 0.70710678118654752f);
    case LINK_CLOGLOG: return 1.0f - expf(-expf(y));
    case LINK_LOGLOG: return expf(-expf(-y));
    case LINK_CAUCHIT: return 0.5f + atanf(y) * 0.31830988618379067f;
    default: return y;
  }
}

// Stage TB rows x F features of a row-major [n_rows, ldx] matrix into LDS as [F][TB] (lane-major,
// so lane r reading feature f hits bank (f*TB + r) % 64 — conflict free for any mix of features),
// applying the field preparation and flagging rejected rows in bad[TB]. Ends with a barrier.
template <int TB>
__device__ __forceinline__ void stage_rows_T(const float* __restrict__ X, int n_rows, int F, int ldx,
                                             const FieldPrep* __restrict__ prep, float* __restrict__ feat,
                                             int* __restrict__ bad, int row0) {
  bad[threadIdx.x] = 0;
  __syncthreads();
  // 16-byte aligned rows: lane = row (consecutive lanes, consecutive rows), one float4 of 4
  // consecutive columns per load, then 4 plane stores of 32 consecutive rows each — conflict-free
  // (a lane-per-column order stores 32 lanes into one bank: 32-way conflicts, measured 16 % of the
  // SVM kernel)
  if ((ldx & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0) {
    const int F4 = (F + 3) >> 2;
    for (int e = threadIdx.x; e < TB * F4; e += TB) {
      const int fq = e / TB;
      const int r = e - fq * TB;
      const int row = row0 + r;
      float4 v = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
      if (row < n_rows) v = *reinterpret_cast<const float4*>(X + (size_t)row * ldx + 4 * fq);
      const float vv[4] = {v.x, v.y, v.z, v.w};
      bool b = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int f = 4 * fq + k;
        if (f < F) {
          float x = vv[k];
          if (row < n_rows && prep) x = prep_value(x, prep[f], &b);
          feat[f * TB + r] = x;
        }
      }
      if (b) bad[r] = 1;
    }
    __syncthreads();
    return;
  }
  const int total = TB * F;
  for (int e = threadIdx.x; e < total; e += TB) {
    const int r = e / F;
    const int f = e - r * F;
    const int row = row0 + r;
    float x = __builtin_nanf("");
    bool b = false;
    if (row < n_rows) {
      x = X[(size_t)row * ldx + f];
      if (prep) x = prep_value(x, prep[f], &b);
    }
    feat[f * TB + r] = x;
    if (b) bad[r] = 1;
  }
  __syncthreads();
}

// stage_rows_T where thread t stages ITS OWN row t (same loads and values as stage_rows_T's
// aligned path; unaligned rows are read a column at a time) and returns the row's rejected flag in
// a register: no bad[TB] array, so a kernel's LDS is the feature planes alone — 32 features x 256
// rows = exactly 32 KiB, five workgroups per CU instead of four. Ends with a barrier.
template <int TB>
__device__ __forceinline__ bool stage_rows_own(const float* __restrict__ X, int n_rows, int F, int ldx,
                                               const FieldPrep* __restrict__ prep, float* __restrict__ feat, int row0) {
  const int r = threadIdx.x;
  const int row = row0 + r;
  const bool in = row < n_rows;
  bool b = false;
  if ((ldx & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0) {
    const int F4 = (F + 3) >> 2;
    for (int fq = 0; fq < F4; ++fq) {
      float4 v = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
      if (in) v = *reinterpret_cast<const float4*>(X + (size_t)row * ldx + 4 * fq);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int f = 4 * fq + k;
        if (f < F) {
          float x = vv[k];
          if (in && prep) x = prep_value(x, prep[f], &b);
          feat[f * TB + r] = x;
        }
      }
    }
  } else {
    for (int f = 0; f < F; ++f) {
      float x = __builtin_nanf("");
      if (in) {
        x = X[(size_t)row * ldx + f];
        if (prep) x = prep_value(x, prep[f], &b);
      }
      feat[f * TB + r] = x;
    }
  }
  __syncthreads();
  return b;
}
