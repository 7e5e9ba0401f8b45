// NeuralNetwork (MLP) scoring on the matrix cores: all layers fused in one kernel.
//
// Data rows sit on the MFMA N dimension (lanes) and neurons on M (registers): each layer computes
// Zᵀ[units, 32 rows] = Wᵀ[units, K] · Hᵀ[K, 32 rows]. With that orientation the 32x32 accumulator
// of one layer (rows of Zᵀ in registers, data rows on lanes) is directly the B operand of the next
// layer's MFMA — no LDS round trip, no lane shuffles between layers (cdna_hip_programming.md §3,
// "An accumulator tile as the next MFMA's operand"). The A operands (weights) are pre-permuted on
// the host into exactly the k order the accumulator registers provide and streamed from L2.
//
// Two precisions:
//   BF16 = true : v_mfma_f32_32x32x16_bf16 (bf16 in, fp32 accumulate) — the throughput path;
//   BF16 = false: v_mfma_f32_32x32x2_f32  (exact fp32 FMA chain)     — the parity path.
// One wave owns 32 data rows; a 256-thread workgroup owns 128. Input normalisation
// (NormContinuous as scale/shift), missing handling, activations, output layer normalisation
// (softmax) and the target decode are fused.
#include "epilogue.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVES = 4;
constexpr int MT = 8;          // max 32-unit tiles per layer -> 256 units
constexpr int MAXL = 4;        // max layers

enum : int { A_IDENTITY = 0, A_LOGISTIC = 1, A_TANH = 2, A_RELU = 3, A_EXP = 4, A_RECIP = 5, A_SQUARE = 6,
             A_GAUSS = 7, A_SINE = 8, A_COSINE = 9, A_ELLIOTT = 10, A_ARCTAN = 11, A_THRESHOLD = 12 };

struct LayerMeta {
  int kp;      // padded K (inputs), multiple of 16 (bf16) / 2 (f32)
  int mp;      // padded M (units), multiple of 32
  int mreal;   // real units
  int w_off;   // offset of this layer's A fragments (elements of the weight type)
  int b_off;   // offset into biases
  int act;     // activation code
  float thr;   // threshold activation parameter
  int pad;
};

struct MlpArgs {
  const float* X;
  int n_rows, n_feat, ldx, n_layers;
  const float* in_scale;    // [n_in]
  const float* in_shift;    // [n_in]
  const float* in_missing;  // [n_in] replacement for a missing input (NaN = invalidates the row)
  const int* in_index;      // [n_in] active-field index of each NN input
  int n_in, k0;             // inputs, padded K of layer 0
  const void* weights;
  const float* biases;
  const LayerMeta* layers;  // [n_layers]
  float out_scale, out_shift;
  int final_norm, n_out;    // final_norm: 0 none, 1 softmax, 2 simplemax
  Epilogue epi;
  float* score;
  uint8_t* valid;
  float* probs;
};

__device__ __forceinline__ float activate(int a, float z, float thr) {
  switch (a) {
    case A_LOGISTIC: return 1.0f / (1.0f + __expf(-z));
    case A_TANH: return tanhf(z);
    case A_RELU: return fmaxf(z, 0.0f);
    case A_EXP: return __expf(z);
    case A_RECIP: return 1.0f / z;
    case A_SQUARE: return z * z;
    case A_GAUSS: return __expf(-z * z);
    case A_SINE: return __sinf(z);
    case A_COSINE: return __cosf(z);
    case A_ELLIOTT: return z / (1.0f + fabsf(z));
    case A_ARCTAN: return 0.63661977236758134f * atanf(z);
    case A_THRESHOLD: return z > thr ? 1.0f : 0.0f;
    default: return z;
  }
}

// row (unit) index inside a 32x32 accumulator tile held by register r of lane half h
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <bool BF16>
__global__ __launch_bounds__(64 * WAVES, BF16 ? 2 : 1) void mlp_kernel(MlpArgs a) {
  extern __shared__ __align__(16) float xs[];  // [WAVES][32][stride]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int col = lane & 31;
  const int stride = BF16 ? a.k0 + 4 : a.k0 + 1;
  float* xw = xs + wave * 32 * stride;
  const int row0 = (blockIdx.x * WAVES + wave) * 32;
  if (row0 >= a.n_rows) return;

  // ---- stage + normalise this wave's 32 input rows: xw[r][k], k < k0 (zero padded)
  for (int e = lane; e < 32 * a.k0; e += 64) {
    const int r = e / a.k0;
    const int k = e - r * a.k0;
    const int row = row0 + r;
    float v = 0.f;
    if (k < a.n_in && row < a.n_rows) {
      const float x = a.X[(size_t)row * a.ldx + a.in_index[k]];
      v = (x != x) ? a.in_missing[k] : fmaf(x, a.in_scale[k], a.in_shift[k]);
    }
    xw[r * stride + k] = v;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes are done
  __builtin_amdgcn_wave_barrier();
  bool bad = false;
  for (int k = 0; k < a.n_in; ++k) bad = bad || (xw[col * stride + k] != xw[col * stride + k]);

  // Named registers instead of arrays: hipcc demoted f32x16 acc[8] / bf16x8 pb[8][2] arrays to
  // scratch (mixed whole-vector and element accesses); one variable per tile stays in VGPR/AGPRs.
#define TILES(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define DECL(i) f32x16 acc##i = {}; bf16x8 pb##i##a = {}, pb##i##b = {}; f32x16 pf##i = {};
  TILES(DECL)
#undef DECL
  int ptiles = 0;

#pragma unroll
  for (int L = 0; L < MAXL; ++L) {
    if (L >= a.n_layers) break;
    const LayerMeta m = a.layers[L];
    const int mtiles = m.mp >> 5;
    const bool last = (L == a.n_layers - 1);
#define INIT(i)                                                                        \
    if (i < mtiles) {                                                                  \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) acc##i[r] = a.biases[m.b_off + 32 * i + acc_row(r, h)]; \
    }
    TILES(INIT)
#undef INIT
    if (BF16) {
      const bf16x8* W = reinterpret_cast<const bf16x8*>(a.weights) + m.w_off / 8;
      const int ksteps = m.kp >> 4;
#define MF(t, B, S) \
      if (t < mtiles) acc##t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(W[(t * ksteps + (S)) * 64 + lane], B, acc##t, 0, 0, 0);
#define MF_ALL(B, S) MF(0, B, S) MF(1, B, S) MF(2, B, S) MF(3, B, S) MF(4, B, S) MF(5, B, S) MF(6, B, S) MF(7, B, S)
      if (L == 0) {
        for (int s = 0; s < ksteps; ++s) {
          const float* src = xw + col * stride + 16 * s + 8 * h;
          bf16x8 b;
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = (__bf16)src[j];
          MF_ALL(b, s)
        }
      } else {
#define LTP(tp) \
        if (tp < ptiles) { MF_ALL(pb##tp##a, 2 * tp) MF_ALL(pb##tp##b, 2 * tp + 1) }
        TILES(LTP)
#undef LTP
      }
#undef MF_ALL
#undef MF
    } else {
      const float* W = reinterpret_cast<const float*>(a.weights) + m.w_off;
      const int ksteps = m.kp >> 1;
#define MF(t, B, S) \
      if (t < mtiles) acc##t = __builtin_amdgcn_mfma_f32_32x32x2f32(W[(t * ksteps + (S)) * 64 + lane], B, acc##t, 0, 0, 0);
#define MF_ALL(B, S) MF(0, B, S) MF(1, B, S) MF(2, B, S) MF(3, B, S) MF(4, B, S) MF(5, B, S) MF(6, B, S) MF(7, B, S)
      if (L == 0) {
        for (int s = 0; s < ksteps; ++s) {
          const float b = xw[col * stride + 2 * s + h];
          MF_ALL(b, s)
        }
      } else {
#define LTP(tp) \
        if (tp < ptiles) { _Pragma("unroll") for (int r = 0; r < 16; ++r) { MF_ALL(pf##tp[r], 16 * tp + r) } }
        TILES(LTP)
#undef LTP
      }
#undef MF_ALL
#undef MF
    }
    // activation (padded units: zero weights + zero bias; their activations only ever meet zero
    // weight columns of the next layer)
#define ACT(i)                                                                         \
    if (i < mtiles) {                                                                  \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                 \
        const float v = activate(m.act, acc##i[r], m.thr);                             \
        if (last) acc##i[r] = v;                                                       \
        else if (BF16) { if (r < 8) pb##i##a[r] = (__bf16)v; else pb##i##b[r - 8] = (__bf16)v; } \
        else pf##i[r] = v;                                                             \
      }                                                                                \
    }
    TILES(ACT)
#undef ACT
    ptiles = mtiles;
  }
  const f32x16 out0 = acc0;
#undef TILES

  // ---- output layer: units 0..n_out-1 live in tile 0; lanes l and l^32 hold the two halves
  const int row = row0 + col;
  const bool in_range = row < a.n_rows;
  if (a.final_norm == 0 && a.n_out == 1) {
    if (h == 0 && in_range) {
      apply_epilogue(a.epi, [&](int) { return out0[0]; }, !bad, row, a.n_rows, a.score, a.valid, a.probs);
    }
    return;
  }
  float mx = -__builtin_inff();
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (acc_row(r, h) < a.n_out) mx = fmaxf(mx, out0[r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  float p[16];
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const bool u = acc_row(r, h) < a.n_out;
    float v = out0[r];
    if (a.final_norm == 1) v = __expf(v - mx);
    p[r] = u ? v : 0.f;
    sum += p[r];
  }
  sum += __shfl_xor(sum, 32);
  float best = -__builtin_inff();
  int best_u = 1 << 30;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int u = acc_row(r, h);
    if (u < a.n_out) {
      if (a.final_norm != 0) p[r] /= sum;
      if (p[r] > best || (p[r] == best && u < best_u)) { best = p[r]; best_u = u; }
      if (a.probs && in_range) a.probs[(size_t)row * a.n_out + u] = p[r];
    }
  }
  const float ob = __shfl_xor(best, 32);
  const int ou = __shfl_xor(best_u, 32);
  if (ob > best || (ob == best && ou < best_u)) { best = ob; best_u = ou; }
  if (h == 0 && in_range) {
    bool ok = !bad && best == best && best_u < a.n_out;
    float sc = ok ? (a.epi.has_table ? a.epi.table[best_u] : (float)best_u) : __builtin_nanf("");
    ok = ok && (sc == sc);
    a.score[row] = ok ? sc : __builtin_nanf("");
    a.valid[row] = ok ? 1 : 0;
    if (a.epi.score2) {
      a.epi.score2[row] = ok ? sc : __builtin_nanf("");
      a.epi.valid2[row] = ok ? 1 : 0;
    }
  }
}

}  // namespace

PMML_API int pmml_mlp_args_size() { return (int)sizeof(MlpArgs); }
PMML_API int pmml_mlp_layer_meta_size() { return (int)sizeof(LayerMeta); }

PMML_API int pmml_mlp_launch(hipStream_t stream, const MlpArgs* args, int bf16) {
  const MlpArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_layers < 1 || a.n_layers > MAXL || a.n_out > 32 || a.k0 > 256) return -4;
  const int stride = bf16 ? a.k0 + 4 : a.k0 + 1;
  const size_t lds = (size_t)WAVES * 32 * stride * 4;
  dim3 grid((a.n_rows + 32 * WAVES - 1) / (32 * WAVES));
  if (bf16) hipLaunchKernelGGL(mlp_kernel<true>, grid, dim3(64 * WAVES), lds, stream, a);
  else hipLaunchKernelGGL(mlp_kernel<false>, grid, dim3(64 * WAVES), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
