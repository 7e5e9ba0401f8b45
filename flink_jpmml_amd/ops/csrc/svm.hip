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
  if (!a.classification && a.epi.tgt) {  // PMML Target of a regression SVM (epilogue.h order)
    sc = apply_target(a.epi, sc);
    if (!ok && (a.epi.tgt & TGT_DEFAULT)) {
      sc = a.epi.dflt;
      ok = true;
    }
  }
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

// ------------------------------------------------------------------------------------------
// Wide SVM kernel: any number of machines (one-against-one over many classes), up to 64 classes,
// up to 128 vector fields, any number of support vectors — the chained two-GEMM form of the
// decision function fused in one pass, both GEMMs on the exact-fp32 matrix cores:
//   G^T = S . X^T      (32 support vectors x 32 rows per MFMA tile, K = fields)
//   K   = kfun(G)      (on the accumulator registers, VALU)
//   D^T = A^T . K^T    (32 machines x 32 rows per tile, K = support vectors)
// The first product's accumulator IS the second product's B operand: lane l of the G tile holds
// G[sv p(i, l>>5)][row l&31] for i < 16 (p(i, h) = (i&3) + 8(i>>2) + 4h), and MFMA step j of the
// second product takes k = l>>5 — so step j feeds register j of every lane as B, and the host
// permutes the dual coefficients to match (A operand of lane l at step j = coef[p(j, l>>5)][l&31]).
// No [rows x support vectors] kernel matrix ever leaves the registers (the library-GEMM plan
// writes and re-reads it through HBM). Operands are pre-swizzled on the host so each lane streams
// contiguous 16-byte loads: svA [tile][lane][FMAX/2], coefA [tile][mtile][lane][16], svnP
// [tile][half][16]. Machines run in groups of MT tiles (acc registers); a model with more
// machines loops over groups, recomputing G per group. Votes go to packed u16 LDS counters.
struct SvmWideArgs {
  SvmArgs s;              // rows, preparation, intercept / thr / tgt / alt ([n_groups*MT*32]), outputs
  const float* svA;       // [n_tiles][64][FMAX/2]
  const float* coefA;     // [n_tiles][n_mtiles][64][16]
  const float* svnP;      // [n_tiles][2][16]
  int n_tiles, n_mtiles, n_groups, pad;
};

constexpr int WTB = 512;  // wide kernel: 8 waves x 32 rows (one MFMA N tile per wave) = TB rows

template <int FMAX, int MT>
__global__ __launch_bounds__(WTB) void svm_wide_kernel(SvmWideArgs w) {
  const SvmArgs& a = w.s;
  constexpr int Q = FMAX / 2;
  extern __shared__ __align__(16) uint32_t votes[];  // [TB][CW] packed u16 class counters
  const int CW = (a.n_classes + 1) >> 1;
  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, l31 = lane & 31;
  const int rl = (tid >> 6) * 32 + l31;  // this lane's row within the tile (both halves share it)
  const int row = blockIdx.x * TB + rl;
  for (int e = tid; e < TB * CW; e += WTB) votes[e] = 0u;
  // B operand of the first product: vector field 2q + half of the row (prepared, zero padded)
  float xb[Q];
  bool bad;
  float xx;
  {
    const float* xr = a.X + (size_t)min(row, a.n_rows - 1) * a.ldx;
    bool b = false;
    if (a.prep)  // row rejection by ANY active field's preparation (the halves split the columns)
      for (int c = half; c < a.n_feat; c += 2) (void)prep_value(xr[c], a.prep[c], &b);
    float sq = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int f = 2 * q + half;
      float x = 0.f;
      if (f < a.n_in) {
        const int c = a.in_index[f];
        x = xr[c];
        if (a.prep) x = prep_value(x, a.prep[c], &b);
        if (x != x) { b = true; x = 0.f; }  // a missing vector field invalidates the row
      }
      xb[q] = x;
      sq = fmaf(x, x, sq);
    }
    xx = sq + __shfl_xor(sq, 32);
    const uint64_t mb = __ballot(b);
    bad = (((mb >> l31) | (mb >> (l31 + 32))) & 1ull) != 0ull;
  }
  __syncthreads();  // vote counters zeroed
  const int M = a.n_machines;
  float reg = 0.f;
  for (int g = 0; g < w.n_groups; ++g) {
    f32x16_t acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x16_t{};
    for (int t = 0; t < w.n_tiles; ++t) {
      f32x16_t d = {};
      const float* sa = w.svA + ((size_t)t * 64 + lane) * Q;
#pragma unroll
      for (int q0 = 0; q0 < Q; q0 += 4) {
        const float4 v = *reinterpret_cast<const float4*>(sa + q0);
        d = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, xb[q0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, xb[q0 + 1], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, xb[q0 + 2], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, xb[q0 + 3], d, 0, 0, 0);
      }
      // kernel function in place: register i <-> support vector 32t + p(i, half)
      const float* sn = w.svnP + ((size_t)t * 2 + half) * 16;
      switch (a.kernel) {  // wave-uniform
        case K_POLY:
#pragma unroll
          for (int i = 0; i < 16; ++i) d[i] = svm_kernel_t<K_POLY>(a, d[i], xx, 0.f);
          break;
        case K_RBF:
#pragma unroll
          for (int i = 0; i < 16; ++i) d[i] = svm_kernel_t<K_RBF>(a, d[i], xx, sn[i]);
          break;
        case K_SIGMOID:
#pragma unroll
          for (int i = 0; i < 16; ++i) d[i] = svm_kernel_t<K_SIGMOID>(a, d[i], xx, 0.f);
          break;
        default:
          break;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float4* ca = reinterpret_cast<const float4*>(
            w.coefA + (((size_t)t * w.n_mtiles + g * MT + mt) * 64 + lane) * 16);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 c = ca[u];
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(c.x, d[4 * u], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(c.y, d[4 * u + 1], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(c.z, d[4 * u + 2], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(c.w, d[4 * u + 3], acc[mt], 0, 0, 0);
        }
      }
    }
    // this group's decision values: the lane holds machines (g*MT + mt)*32 + p(i, half) of its row
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = (g * MT + mt) * 32 + (i & 3) + 8 * (i >> 2) + 4 * half;
        if (m >= M) continue;
        const float dv = acc[mt][i] + a.intercept[m];
        if (a.decision && row < a.n_rows) a.decision[(size_t)row * M + m] = dv;
        if (!a.classification) {
          reg = dv;  // M == 1: machine 0 sits in half 0, register 0
          continue;
        }
        bool first = dv < a.thr[m];
        if (a.max_wins) first = !first;
        const int c = first ? a.tgt[m] : a.alt[m];
        if (c >= 0) atomicAdd(&votes[rl * CW + (c >> 1)], 1u << (16 * (c & 1)));
      }
    }
  }
  __syncthreads();
  if (half != 0 || row >= a.n_rows) return;
  float sc;
  if (a.classification) {
    int best = 0;
    uint32_t bv = votes[rl * CW] & 0xFFFFu;
    for (int c = 1; c < a.n_classes; ++c) {
      const uint32_t v = (votes[rl * CW + (c >> 1)] >> (16 * (c & 1))) & 0xFFFFu;
      if (v > bv) { bv = v; best = c; }  // ties: the first category
    }
    sc = a.epi.table[best];
  } else {
    sc = reg;
  }
  bool ok = !bad && (sc == sc);
  if (!a.classification && a.epi.tgt) {  // PMML Target of a regression SVM (epilogue.h order)
    sc = apply_target(a.epi, sc);
    if (!ok && (a.epi.tgt & TGT_DEFAULT)) {
      sc = a.epi.dflt;
      ok = true;
    }
  }
  const float so = ok ? sc : __builtin_nanf("");
  a.score[row] = so;
  a.valid[row] = ok ? 1 : 0;
  if (a.epi.score2) {
    a.epi.score2[row] = so;
    a.epi.valid2[row] = ok ? 1 : 0;
  }
}

template <int FMAX, int MT>
int launch_svm_wide_t(hipStream_t stream, const SvmWideArgs& w, dim3 grid, size_t lds) {
  auto k = svm_wide_kernel<FMAX, MT>;
  if (lds > 65536 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return -5;
  hipLaunchKernelGGL(k, grid, dim3(WTB), lds, stream, w);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

template <int FMAX>
int launch_svm_wide_f(hipStream_t stream, const SvmWideArgs& w, int mt, dim3 grid, size_t lds) {
  switch (mt) {
    case 1: return launch_svm_wide_t<FMAX, 1>(stream, w, grid, lds);
    case 2: return launch_svm_wide_t<FMAX, 2>(stream, w, grid, lds);
    case 4: return launch_svm_wide_t<FMAX, 4>(stream, w, grid, lds);
    default: return -6;
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

PMML_API int pmml_svm_wide_args_size() { return (int)sizeof(SvmWideArgs); }

// fmax in {16, 32, 64, 128} (vector fields padded), mt in {1, 2, 4} (machine tiles per group);
// intercept / thr / tgt / alt hold n_groups * mt * 32 entries; n_classes <= 256 (votes: TB x 128
// packed u16 counters = 128 KiB of LDS at most), at most 65535 machines per classifier.
PMML_API int pmml_svm_wide_launch(hipStream_t stream, const SvmWideArgs* args, int fmax, int mt) {
  const SvmWideArgs w = *args;
  const SvmArgs& a = w.s;
  if (a.n_rows <= 0) return 0;
  if (a.n_in > fmax || a.n_classes > 256) return -4;
  if (a.classification && (a.n_classes < 1 || a.n_machines > 0xFFFF)) return -4;
  if (w.n_tiles < 1 || w.n_groups < 1 || w.n_mtiles != w.n_groups * mt || a.n_machines > w.n_mtiles * 32) return -4;
  if (!a.classification && a.n_machines != 1) return -4;
  if (a.kernel < 0 || a.kernel > 3) return -4;
  dim3 grid((a.n_rows + TB - 1) / TB);
  const size_t lds = (size_t)TB * ((a.n_classes + 1) / 2 > 0 ? (a.n_classes + 1) / 2 : 1) * 4;
  switch (fmax) {
    case 16: return launch_svm_wide_f<16>(stream, w, mt, grid, lds);
    case 32: return launch_svm_wide_f<32>(stream, w, mt, grid, lds);
    case 64: return launch_svm_wide_f<64>(stream, w, mt, grid, lds);
    case 128: return launch_svm_wide_f<128>(stream, w, mt, grid, lds);
    default: return -6;
  }
}
