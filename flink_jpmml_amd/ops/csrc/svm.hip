// SupportVectorMachineModel scoring: kernel evaluation against every support vector + dual
// coefficients + machine votes, fused in one pass.
//
// Two kernels, fp32 throughout (parity path):
//  * svm_mfma_kernel (>= 32 support vectors, the common case): the x . sv products on the matrix
//    cores (exact-fp32 MFMA, support vectors on M, rows on N), kernel function and dual
//    coefficients applied on the accumulator registers — see its comment below;
//  * svm_kernel (few support vectors): one lane per row, the row's (prepared) features in
//    registers (FMAX template bucket, zero padded), every support vector read by all lanes at the
//    same address (broadcast); machines (<= MMAX) accumulate in registers.
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

// Decision values -> machine votes / regression score, validity, outputs (both kernels).
__device__ __forceinline__ void svm_finish(const SvmArgs& a, int row, const float (&acc)[MMAX], bool ok) {
  if (a.decision) {
    for (int m = 0; m < a.n_machines; ++m) a.decision[(size_t)row * a.n_machines + m] = acc[m];
  }
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

template <int KT>
__device__ __forceinline__ float svm_kernel_t(const SvmArgs& a, float dot, float xx, float svn) {
  if constexpr (KT == K_POLY) return __powf(fmaf(a.gamma, dot, a.coef0), a.degree);
  if constexpr (KT == K_RBF)  // exp(-g d) as one v_exp_f32 of d * (-g log2 e)
    return __builtin_amdgcn_exp2f(fmaxf(xx - 2.f * dot + svn, 0.f) * (-a.gamma * 1.4426950408889634f));
  if constexpr (KT == K_SIGMOID) return tanhf(fmaf(a.gamma, dot, a.coef0));
  return dot;
}

__device__ __forceinline__ float svm_kernel_fn(const SvmArgs& a, float dot, float xx, float svn) {
  switch (a.kernel) {
    case K_POLY: return __powf(fmaf(a.gamma, dot, a.coef0), a.degree);
    case K_RBF: return __expf(-a.gamma * fmaxf(xx - 2.f * dot + svn, 0.f));
    case K_SIGMOID: return tanhf(fmaf(a.gamma, dot, a.coef0));
    default: return dot;
  }
}

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
    const float k = svm_kernel_fn(a, dot, xn, a.kernel == K_RBF ? a.sv_norm[j] : 0.f);
    const float* cj = a.coef + (size_t)j * MMAX;
#pragma unroll
    for (int m = 0; m < MMAX; ++m) acc[m] = fmaf(cj[m], k, acc[m]);
  }
  svm_finish(a, row, acc, !bad && !miss);
}


// Matrix-core path (n_sv >= 32): the x . sv products of 32 support vectors (M) x 32 rows (N) per
// exact-fp32 `v_mfma_f32_32x32x2f32`, a wave's 64 rows as two N tiles sharing every A (support
// vector) operand; the kernel function and the dual-coefficient products run on the accumulator
// registers (lane = one row, 16 support vectors), the two lane halves (other 16 support vectors
// of each 32) are added once at the end. Rows staged transposed in LDS (fused field preparation).
// sv / coef are padded on the host to whole 32-vector tiles with zero coefficients; support
// vectors (row stride FMAX + 1: conflict-free A fragments), coefficients and norms are staged in
// LDS once per workgroup (global A-operand loads per MFMA left the chain latency-bound: 0.67 ms
// per 1M rows at 256 support vectors, no faster than the VALU kernel).
typedef float f32x16_t __attribute__((ext_vector_type(16)));

// NM: machines evaluated per support vector (1: binary / regression; MMAX: any, the padded
// machines' coefficients are zero) — unconditional FMAs on a vector LDS read, no per-machine branch
template <int FMAX, int KT, int NM>
__global__ __launch_bounds__(TB) void svm_mfma_kernel(SvmArgs a, int n_svp) {
  constexpr int SVS = FMAX + 1;  // padded support-vector row: the 32 rows of an A fragment hit 32 banks
  extern __shared__ __align__(16) uint32_t smem[];
  // LDS: [feat n_feat x TB][bad TB][sv n_svp x SVS][coef n_svp x MMAX][sv_norm n_svp]
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  float* svs = reinterpret_cast<float*>(bad + TB);
  float* cof = svs + n_svp * SVS;
  float* svn = cof + n_svp * MMAX;
  for (int e = threadIdx.x; e < n_svp * FMAX; e += TB) svs[(e / FMAX) * SVS + e % FMAX] = a.sv[e];
  for (int e = threadIdx.x; e < n_svp * MMAX; e += TB) cof[e] = a.coef[e];
  for (int e = threadIdx.x; e < n_svp; e += TB) svn[e] = a.sv_norm[e];
  const int row0 = blockIdx.x * TB;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);  // barriers both sides
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int half = lane >> 5;
  const int rb = (tid >> 6) * 64 + (lane & 31);
  // B operand columns: vector field f -> staged active field in_index[f] (zero beyond n_in)
  float xb[2][FMAX / 2];
  float xx[2] = {0.f, 0.f};
  bool miss[2] = {false, false};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int q = 0; q < FMAX / 2; ++q) {
      const int f = 2 * q + half;
      float x = 0.f;
      if (f < a.n_in) x = feat[a.in_index[f] * TB + rb + 32 * h];
      miss[h] = miss[h] || (x != x);
      xb[h][q] = (x != x) ? 0.f : x;  // a missing value invalidates the row (below)
      xx[h] = fmaf(xb[h][q], xb[h][q], xx[h]);
    }
    xx[h] += __shfl_xor(xx[h], 32);  // the other half's fields
    const uint64_t mb = __ballot(miss[h]);  // either half of the row's fields
    miss[h] = (((mb >> (lane & 31)) | (mb >> ((lane & 31) + 32))) & 1ull) != 0ull;
  }
  float acc[2][MMAX];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int m = 0; m < MMAX; ++m) acc[h][m] = 0.f;
  for (int k0 = 0; k0 < n_svp; k0 += 32) {
    f32x16_t d0 = {}, d1 = {};
    const float* srow = svs + (k0 + (lane & 31)) * SVS + half;
    float av[FMAX / 2];
#pragma unroll
    for (int q = 0; q < FMAX / 2; ++q) av[q] = srow[2 * q];
#pragma unroll
    for (int q = 0; q < FMAX / 2; ++q) {
      d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], xb[0][q], d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], xb[1][q], d1, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // D[sv (i&3)+8(i>>2)+4*half][row lane&31]
      const int k = k0 + (i & 3) + 8 * (i >> 2) + 4 * half;
      const float sn = svn[k];
      const float k0v = svm_kernel_t<KT>(a, d0[i], xx[0], sn);
      const float k1v = svm_kernel_t<KT>(a, d1[i], xx[1], sn);
      const float* cj = cof + k * MMAX;
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        acc[0][m] = fmaf(cj[m], k0v, acc[0][m]);
        acc[1][m] = fmaf(cj[m], k1v, acc[1][m]);
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float tot[MMAX];
#pragma unroll
    for (int m = 0; m < MMAX; ++m) tot[m] = a.intercept[m] + (acc[h][m] + __shfl_xor(acc[h][m], 32));
    const int rl = rb + 32 * h;
    const int row = row0 + rl;
    if (half == h && row < a.n_rows) svm_finish(a, row, tot, bad[rl] == 0 && !miss[h]);
  }
}

template <int FMAX, int KT>
int launch_svm_mfma_k(hipStream_t stream, const SvmArgs& a, int n_svp, dim3 grid, size_t lds) {
  auto k = a.n_machines == 1 ? svm_mfma_kernel<FMAX, KT, 1> : svm_mfma_kernel<FMAX, KT, MMAX>;
  if (lds > 65536 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return -5;
  hipLaunchKernelGGL(k, grid, dim3(TB), lds, stream, a, n_svp);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

template <int FMAX>
int launch_svm_mfma(hipStream_t stream, const SvmArgs& a, int n_svp, dim3 grid, size_t lds) {
  switch (a.kernel) {
    case K_POLY: return launch_svm_mfma_k<FMAX, K_POLY>(stream, a, n_svp, grid, lds);
    case K_RBF: return launch_svm_mfma_k<FMAX, K_RBF>(stream, a, n_svp, grid, lds);
    case K_SIGMOID: return launch_svm_mfma_k<FMAX, K_SIGMOID>(stream, a, n_svp, grid, lds);
    default: return launch_svm_mfma_k<FMAX, K_LINEAR>(stream, a, n_svp, grid, lds);
  }
}
}  // namespace

PMML_API int pmml_svm_args_size() { return (int)sizeof(SvmArgs); }

// n_svp: support vectors padded to whole 32-vector tiles (sv / coef rows; 0 = VALU kernel only)
PMML_API int pmml_svm_launch(hipStream_t stream, const SvmArgs* args, int fmax, int n_svp) {
  const SvmArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_machines > MMAX || a.n_classes > 16) return -4;
  dim3 grid((a.n_rows + TB - 1) / TB);
  const size_t lds = (size_t)a.n_feat * TB * 4 + TB * 4 + (size_t)n_svp * (fmax + 1 + MMAX + 1) * 4;
  if (n_svp >= 32 && (n_svp & 31) == 0 && a.n_feat <= 64 && lds <= 160 * 1024 && a.kernel >= 0 && a.kernel <= 3) {
    switch (fmax) {
      case 8: return launch_svm_mfma<8>(stream, a, n_svp, grid, lds);
      case 16: return launch_svm_mfma<16>(stream, a, n_svp, grid, lds);
      case 32: return launch_svm_mfma<32>(stream, a, n_svp, grid, lds);
      case 64: return launch_svm_mfma<64>(stream, a, n_svp, grid, lds);
      default: return -6;
    }
  }
  switch (fmax) {
    case 8: hipLaunchKernelGGL(svm_kernel<8>, grid, dim3(TB), 0, stream, a); break;
    case 16: hipLaunchKernelGGL(svm_kernel<16>, grid, dim3(TB), 0, stream, a); break;
    case 32: hipLaunchKernelGGL(svm_kernel<32>, grid, dim3(TB), 0, stream, a); break;
    case 64: hipLaunchKernelGGL(svm_kernel<64>, grid, dim3(TB), 0, stream, a); break;
    default: return -6;
  }
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
