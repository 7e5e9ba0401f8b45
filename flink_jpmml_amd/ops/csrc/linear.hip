// RegressionModel / GeneralRegressionModel (dense numeric tables): y_k = b_k + Σ_f W[f][k]·x_f,
// then the fused link / normalisation epilogue (regression link, binary link, softmax, simplemax).
//
// One lane per row; W and b are read with wave-uniform addresses (scalar loads, broadcast), the
// row tile comes from the shared LDS staging helper. A missing numeric predictor makes the row's
// prediction missing (PMML RegressionModel rule).
#include "epilogue.h"

namespace {

constexpr int TB = 256;
constexpr int KMAX = 16;

struct LinearArgs {
  const float* X;
  int n_rows, n_feat, ldx, K;
  const FieldPrep* prep;
  const float* W;      // [F][K]
  const float* bias;   // [K]
  int simplemax, pad;
  Epilogue epi;
  float* score;
  uint8_t* valid;
  float* probs;
};

__global__ __launch_bounds__(TB) void linear_kernel(LinearArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  const int row0 = blockIdx.x * TB;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  const int tid = threadIdx.x;
  const int row = row0 + tid;
  if (row >= a.n_rows) return;
  float acc[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) acc[k] = (k < a.K) ? a.bias[k] : 0.f;
  bool miss = false;
  for (int f = 0; f < a.n_feat; ++f) {
    const float x = feat[f * TB + tid];
    miss = miss || (x != x);
    const float* w = a.W + (size_t)f * a.K;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < a.K) acc[k] = fmaf(w[k], x, acc[k]);
  }
  if (a.simplemax) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < a.K) s += acc[k];
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < a.K) acc[k] /= s;
  }
  apply_epilogue(a.epi, [&](int c) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) v = (k == c) ? acc[k] : v;
    return v;
  }, (bad[tid] == 0) && !miss, row, a.n_rows, a.score, a.valid, a.probs);
}

}  // namespace

PMML_API int pmml_linear_args_size() { return (int)sizeof(LinearArgs); }

PMML_API int pmml_linear_launch(hipStream_t stream, const LinearArgs* args) {
  const LinearArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.K > KMAX || a.n_feat > 128) return -4;
  const size_t lds = (size_t)a.n_feat * TB * 4 + TB * 4;
  dim3 grid((a.n_rows + TB - 1) / TB);
  hipLaunchKernelGGL(linear_kernel, grid, dim3(TB), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
