// Fused per-row epilogue: ensemble/linear accumulators -> PMML target value (+ probabilities).
#pragma once
#include "common.h"

__device__ __forceinline__ float apply_target(const Epilogue& e, float s) {
  double v = (double)s;
  if ((e.tgt & TGT_LO) && v < e.lo) v = e.lo;  // compare form: a NaN stays NaN (no prediction)
  if ((e.tgt & TGT_HI) && v > e.hi) v = e.hi;
  v = v * e.ta + e.tb;
  switch ((e.tgt >> TGT_CAST_SHIFT) & 3) {
    case CAST_ROUND: v = floor(v + 0.5); break;
    case CAST_CEIL: v = ceil(v); break;
    case CAST_FLOOR: v = floor(v); break;
    default: break;
  }
  return (float)v;
}

// acc: C accumulator values of this row (registers or LDS, read through the accessor).
template <typename Acc>
__device__ __forceinline__ void apply_epilogue(const Epilogue& e, Acc acc, bool row_ok, int row, int n_rows,
                                               float* __restrict__ score, uint8_t* __restrict__ valid,
                                               float* __restrict__ probs) {
  float s = __builtin_nanf("");
  bool ok = row_ok;
  int label = 0;
  if (e.mode == EPI_AFFINE) {
    s = apply_link(e.link, fmaf(e.a, acc(0), e.b));
    ok = ok && __builtin_isfinite(s);  // the oracle's regression rule: a non-finite value is no prediction
    if (e.tgt) s = apply_target(e, s);  // on the model value, after its validity (oracle order)
    if (!ok && (e.tgt & TGT_DEFAULT)) {
      s = e.dflt;
      ok = true;
    }
    if (e.write_probs && probs) probs[row] = s;
  } else if (e.mode == EPI_LOGISTIC2) {
    float p0 = apply_link(e.link, fmaf(e.a, acc(0), e.b));
    label = (p0 >= e.thr) ? 0 : 1;
    if (e.write_probs && probs) {
      probs[(size_t)row * 2 + 0] = p0;
      probs[(size_t)row * 2 + 1] = 1.0f - p0;
    }
    ok = ok && (p0 == p0);
  } else if (e.mode == EPI_LINKMAX) {
    const int C = e.n_classes;
    float best = -__builtin_inff();
    for (int c = 0; c < C; ++c) {
      const float pv = apply_link(e.link, acc(c));
      if (pv > best) { best = pv; label = c; }  // NaN never wins (the oracle's nan -> -inf)
      ok = ok && __builtin_isfinite(pv);
      if (e.write_probs && probs) probs[(size_t)row * C + c] = pv;
    }
  } else if (e.mode == EPI_CUMULATIVE) {
    const int C = e.n_classes;
    float best = -__builtin_inff();
    float prev = 0.f;
    for (int c = 0; c < C; ++c) {
      const float cum = c < C - 1 ? apply_link(e.link, acc(c)) : 1.0f;
      const float pv = cum - prev;
      prev = cum;
      if (pv > best) { best = pv; label = c; }
      ok = ok && (pv == pv);
      if (e.write_probs && probs) probs[(size_t)row * C + c] = pv;
    }
  } else {
    const int C = e.n_classes;
    float best = -__builtin_inff();
    float mx = -__builtin_inff();
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, acc(c));
    float denom = 0.f;
    if (e.mode == EPI_SOFTMAX) {
      for (int c = 0; c < C; ++c) denom += __expf(acc(c) - mx);
    }
    for (int c = 0; c < C; ++c) {
      float v = acc(c);
      if (v > best) { best = v; label = c; }
      if (e.write_probs && probs) {
        float pv = (e.mode == EPI_SOFTMAX) ? __expf(v - mx) / denom : v * e.a;
        probs[(size_t)row * C + c] = pv;
      }
    }
    ok = ok && (best == best) && (best > -__builtin_inff());
  }
  if (e.mode != EPI_AFFINE) {
    s = e.has_table ? e.table[label] : (float)label;
    ok = ok && (s == s);
  }
  const float so = ok ? s : __builtin_nanf("");
  score[row] = so;
  valid[row] = ok ? 1 : 0;
  if (e.score2) {
    e.score2[row] = so;
    e.valid2[row] = ok ? 1 : 0;
  }
}
