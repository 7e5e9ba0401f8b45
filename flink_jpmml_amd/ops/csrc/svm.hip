// SupportVectorMachineModel scoring: kernel evaluation against every support vector + dual
// coefficients + machine votes, fused in one pass.
//
// One lane per row; the row's (prepared) features live in registers (FMAX template bucket, zero
// padded) so the per-support-vector dot product needs no memory traffic besides the support
// vector itself, which every lane reads at the same address (scalar loads, broadcast). Machines
// (<= MMAX) accumulate in registers. fp32 throughout (parity path; the SV x row product is tiny
// compared to the tree and MLP workloads, see profiles/).
#include "epilogue.h"

namespace {

constexpr int TB = 256;
constexpr int MMAX = 8;

enum : int { K_LINEAR = 0, K_POLY = 1, K_RBF = 2, K_SIGMOID = 3 };

struct SvmArgs {
  const float* X;
  int n_rows, n_feat, ldx, n_sv;
  const FieldPrep* prep;
  const int* in_index;     // [n_in] active-field index of each vector field
  const float* sv;         // [n_sv][FMAX] (zero padded)
  const float* sv_norm;    // [n_sv] squared norms (RBF)
  const float* coef;       // [n_sv][MMAX] dual coefficients per machine (zero padded)
  const float* intercept;  // [MMAX]
  const float* thr;        // [MMAX] decision threshold per machine
  const int* tgt;          // [MMAX] category index voted when D < thr
  const int* alt;          // [MMAX] category index voted otherwise (-1: none)
  int n_in, n_machines, kernel, classification;
  float gamma, coef0, degree;
  int max_wins, n_classes, pad;
  Epilogue epi;  // table: category -> score
  float* score;
  uint8_t* valid;
  float* decision;  // optional [n_rows][n_machines]
};

template <int FMAX>
__global__ __launch_bounds__(TB) void svm_kernel(SvmArgs a) {
  const int row = blockIdx.x * TB + threadIdx.x;
  if (row >= a.n_rows) return;
  float x[FMAX];
  bool bad = false, miss = false;
  float xn = 0.f;
#pragma unroll
  for (int f = 0; f < FMAX; ++f) {
    float v = 0.f;
    if (f < a.n_in) {
      const int c = a.in_index[f];
      v = a.X[(size_t)row * a.ldx + c];
      if (a.prep) v = prep_value(v, a.prep[c], &bad);
      miss = miss || (v != v);
    }
    x[f] = v;
    xn = fmaf(v, v, xn);
  }
  float acc[MMAX];
#pragma unroll
  for (int m = 0; m < MMAX; ++m) acc[m] = a.intercept[m];
  for (int j = 0; j < a.n_sv; ++j) {
    const float* s = a.sv + (size_t)j * FMAX;
    float dot = 0.f;
#pragma unroll
    for (int f = 0; f < FMAX; ++f) dot = fmaf(x[f], s[f], dot);
    float k;
    switch (a.kernel) {
      case K_POLY: k = __powf(fmaf(a.gamma, dot, a.coef0), a.degree); break;
      case K_RBF: k = __expf(-a.gamma * fmaxf(xn - 2.f * dot + a.sv_norm[j], 0.f)); break;
      case K_SIGMOID: k = tanhf(fmaf(a.gamma, dot, a.coef0)); break;
      default: k = dot;
    }
    const float* cj = a.coef + (size_t)j * MMAX;
#pragma unroll
    for (int m = 0; m < MMAX; ++m) acc[m] = fmaf(cj[m], k, acc[m]);
  }
  if (a.decision) {
    for (int m = 0; m < a.n_machines; ++m) a.decision[(size_t)row * a.n_machines + m] = acc[m];
  }
  bool ok = !bad && !miss;
  float sc;
  if (!a.classification) {
    sc = acc[0];
  } else {
    int votes[16];
    for (int c = 0; c < 16; ++c) votes[c] = 0;
#pragma unroll
    for (int m = 0; m < MMAX; ++m) {
      if (m < a.n_machines) {
        bool first = acc[m] < a.thr[m];
        if (a.max_wins) first = !first;
        if (first) votes[a.tgt[m] & 15] += 1;
        else if (a.alt[m] >= 0) votes[a.alt[m] & 15] += 1;
      }
    }
    int best = 0;
    for (int c = 1; c < a.n_classes && c < 16; ++c)
      if (votes[c] > votes[best]) best = c;
    sc = a.epi.table[best];
  }
  ok = ok && (sc == sc);
  const float so = ok ? sc : __builtin_nanf("");
  a.score[row] = so;
  a.valid[row] = ok ? 1 : 0;
  if (a.epi.score2) {
    a.epi.score2[row] = so;
    a.epi.valid2[row] = ok ? 1 : 0;
  }
}

}  // namespace

PMML_API int pmml_svm_args_size() { return (int)sizeof(SvmArgs); }

PMML_API int pmml_svm_launch(hipStream_t stream, const SvmArgs* args, int fmax) {
  const SvmArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_machines > MMAX || a.n_classes > 16) return -4;
  dim3 grid((a.n_rows + TB - 1) / TB);
  switch (fmax) {
    case 8: hipLaunchKernelGGL(svm_kernel<8>, grid, dim3(TB), 0, stream, a); break;
    case 16: hipLaunchKernelGGL(svm_kernel<16>, grid, dim3(TB), 0, stream, a); break;
    case 32: hipLaunchKernelGGL(svm_kernel<32>, grid, dim3(TB), 0, stream, a); break;
    case 64: hipLaunchKernelGGL(svm_kernel<64>, grid, dim3(TB), 0, stream, a); break;
    default: return -6;
  }
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
