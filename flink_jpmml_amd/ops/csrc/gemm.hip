// Wide NeuralNetwork layers on the matrix cores: a tiled bf16 MFMA GEMM with the bias, the
// activation and (for the output layer) the whole PMML output decode fused into its epilogue.
//
// The fused MLP kernel (mlp.hip) keeps every activation in registers, which caps a layer at 256
// units. Beyond that each layer is one launch of this kernel:
//
//   H_{l+1}[rows, M] = act(H_l[rows, K] · W_l[K, M] + b_l)      (bf16 in / out, fp32 accumulate)
//
// * Block tile 256 rows x BN units (BN = 256 for hidden layers, 32 for the output layer), K staged
//   in BK = 64 slices through two LDS buffers with direct global->LDS loads
//   (__builtin_amdgcn_global_load_lds, 16 B per lane): the load of slice k+1 is in flight while
//   slice k feeds the MFMAs. 512 threads = 8 waves; a hidden-layer wave owns a 128 x 64 sub-tile
//   (4 x 2 accumulators of v_mfma_f32_32x32x16_bf16).
// * LDS images are [row][64 k] with the 16-byte chunks XOR-swizzled by (row & 7) — the swizzle is
//   applied to the per-lane GLOBAL source address (the LDS side of an LDS-DMA is lane-linear), so
//   the ds_read_b128 fragment reads of 32 consecutive rows hit distinct banks.
// * Weights are stored unit-major (Wᵀ, [M][K]) so both MFMA operands read 8 consecutive k.
// * Tile order is XCD-aware: consecutive tiles (the column tiles of one row tile, which share the
//   A slice) are placed on the same XCD, so the A tile is fetched into one L2 once.
// * Epilogue (hidden): + bias, activation, bf16, lane pairs merged into 4-byte stores.
// * fp32 operands (the default fp32 precision policy): the same tiles, LDS images and schedule on
//   the exact-fp32 v_mfma_f32_32x32x2f32 — a BK slice is 32 floats (still 128 B per row); a lane
//   reads one 16-byte chunk (4 k) per operand tile and feeds it to 4 consecutive MFMAs, the k order
//   permuted identically in A and B (k = 4 * chunk + element, chunk = 2 g + half), so the dot
//   products are unchanged; activations stay fp32 between layers.
// * The input stage is its own small kernel: one lane per (row, 8 inputs), validity by ballot.
//   Epilogue (output layer): + bias into an LDS row tile, then one thread per row applies the
//   output activation, softmax / simplemax, label table or regression affine + Target stage and
//   writes score / valid / probabilities (the zero-copy sink pointers of the pipeline).
//
// Which kernel takes a layer (pmml_gemm_launch / pmml_gemm_fused_head_launch):
//   bf16 hidden, K = 64          gemm_k64p_kernel  persistent over row tiles, weights staged once,
//                                                   non-temporal 128-byte row-segment stores
//   bf16 hidden, K >= 128        gemm8p_kernel     persistent 256 x 256 phase-interleaved walk
//                                                   (LDS-DMA slice stream across tiles, SADDR asm)
//   last hidden + output layer   gemm8p_kernel<true> (n_out <= 4) / gemm8_kernel<true>: the output
//                                                   layer folded into the accumulators, no H store
//   output layer / fp32 / flags  gemm_kernel       the 2-buffer loop described above
//   bit 12 (A/B reference)       gemm8_kernel / gemm_kernel, one tile per workgroup
// Every alternative path stays selectable by a flag bit of GemmArgs.f32 and is pinned bit for bit
// against the default by tests/test_wide_mlp.py.
#include "epilogue.h"
#include "nn_act.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 256;  // rows per block
constexpr int BK = 64;   // bf16 k per LDS slice (128 B per row); fp32: 32
constexpr int SLICE_B = 128;  // bytes of one row in one LDS slice
constexpr int NT = 512;  // threads (8 waves)
constexpr int HEAD_LD = 33;
constexpr int NN_MAX_INPUTS = 16384;  // network inputs of the wide-layer input stage (padded to 64)

struct GemmArgs {
  const void* A;          // [rows_p][lda] activations (bf16 or fp32), rows_p = rows rounded up to BM
  const void* Wt;         // [Mp][ldw] weights, unit-major, Mp a multiple of BN
  const float* bias;      // [Mp]
  void* C;                // hidden layer output [rows_p][ldc]
  int rows, rows_p, K, Mp;  // K: multiple of the slice (64 bf16 / 32 fp32)
  int lda, ldw, ldc, act;
  float thr;              // threshold activation parameter
  int n_out, final_norm;  // output layer: real units, 0 none / 1 softmax / 2 simplemax
  int f32;                // bit 0: operand / activation type (0 bf16, 1 fp32); experiment bits (A/B tests,
                          // WideMlpPlan.gemm_flags): 5 wave-private LDS epilogue, 6 K = 64 on the 256 x 256
                          // tile, 7 force the phase-interleaved kernel, 8 direct [row][unit] stores instead of
                          // store_hidden_t, 9 one K = 64 tile per workgroup instead of gemm_k64p_kernel,
                          // 10 gemm_k64p_kernel with store_hidden_t instead of the row-segment stores,
                          // 11 the same for gemm8_kernel<false, true>, 12 one tile per workgroup
                          // (gemm8_kernel) instead of the persistent gemm8p_kernel, 13 gemm8p_kernel
                          // without its epilogue stores (timing only: the layer output is not written),
                          // 14 gemm_k64p_kernel with ordinary instead of non-temporal stores, 15
                          // gemm8p_kernel storing each tile in two halves (deferred, measured slower),
                          // 16 gemm8p_kernel also above K = 1024 (experiment)
  const uint8_t* row_ok;  // [rows] input-stage validity (output layer)
  Epilogue epi;           // output layer decode (affine + Target, or label table)
  float* score;
  uint8_t* valid;
  float* probs;
};

struct PrepArgs {
  const float* X;
  int n_rows, rows_p, ldx, n_in;
  const int* in_index;     // [n_in] active-field column of each network input
  const float* in_scale;   // [n_in] NormContinuous as an affine map
  const float* in_shift;
  const float* in_missing; // [n_in] value for a missing input (NaN: the row has no prediction)
  void* H;                 // [rows_p][ldh] bf16 or fp32
  int ldh, k0;             // k0: padded width (zero columns past n_in)
  uint8_t* row_ok;         // [rows_p]
  int f32;
  int contig;              // in_index[k] == in_index[0] + k, in_index[0] % 4 == 0 (host); X 16-byte rows (launch)
};

// Input layer: gather the network inputs, normalise, replace missing, bf16. A row's 8-input
// chunks are spread over GP consecutive lanes (GP = chunks rounded up to a power of two, at most
// 64: beyond 512 inputs a lane takes every 64th chunk), so its reads and its 16-byte stores are
// contiguous, and the row's validity is the AND over its lane group (one wave ballot). The affine
// / missing-value tables of the first NN_PREP_LDS inputs are staged in LDS (16-byte reads instead
// of three 4-byte vector loads per input), and a contiguous, aligned input map reads a chunk's 8
// inputs as two 16-byte loads.
constexpr int NN_PREP_LDS = 1024;
template <bool F32>
__global__ __launch_bounds__(256) void nn_prep_kernel(PrepArgs a, int gp_log2) {
  __shared__ __align__(16) float tb[3][NN_PREP_LDS];  // scale, shift, missing (zero past n_in)
  const int GP = 1 << gp_log2;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int row = t >> gp_log2;
  const int lc = t & (GP - 1);
  const int nchunk = a.k0 >> 3;
  const bool live_row = row < a.n_rows;
  const bool active = row < a.rows_p;
  const bool lds_tab = a.k0 <= NN_PREP_LDS;
  if (lds_tab) {
    for (int k = threadIdx.x; k < a.k0; k += 256) {
      const bool in = k < a.n_in;
      tb[0][k] = in ? a.in_scale[k] : 0.f;
      tb[1][k] = in ? a.in_shift[k] : 0.f;
      tb[2][k] = in ? a.in_missing[k] : 0.f;
    }
    __syncthreads();
  }
  const int c0 = a.contig ? a.in_index[0] : 0;
  bool bad = false;
  for (int chunk = lc; active && chunk < nchunk; chunk += GP) {
    const float* x = a.X + (size_t)(live_row ? row : 0) * a.ldx;
    float v[8];
    if (lds_tab && a.contig && chunk * 8 + 8 <= a.n_in) {  // a full chunk: vector loads
      const float4 x0 = *reinterpret_cast<const float4*>(x + c0 + chunk * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(x + c0 + chunk * 8 + 4);
      const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      float sc[8], sh[8], ms[8];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float4 s4 = *reinterpret_cast<const float4*>(&tb[0][chunk * 8 + 4 * q]);
        const float4 h4 = *reinterpret_cast<const float4*>(&tb[1][chunk * 8 + 4 * q]);
        const float4 m4 = *reinterpret_cast<const float4*>(&tb[2][chunk * 8 + 4 * q]);
        sc[4 * q] = s4.x, sc[4 * q + 1] = s4.y, sc[4 * q + 2] = s4.z, sc[4 * q + 3] = s4.w;
        sh[4 * q] = h4.x, sh[4 * q + 1] = h4.y, sh[4 * q + 2] = h4.z, sh[4 * q + 3] = h4.w;
        ms[4 * q] = m4.x, ms[4 * q + 1] = m4.y, ms[4 * q + 2] = m4.z, ms[4 * q + 3] = m4.w;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float z = 0.f;
        if (live_row) {
          const float xv = xs[j];
          z = xv == xv ? fmaf(xv, sc[j], sh[j]) : ms[j];
          bad = bad || (z != z);
          z = z == z ? z : 0.f;
        }
        v[j] = z;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = chunk * 8 + j;
        float z = 0.f;
        if (live_row && k < a.n_in) {
          const float xv = x[a.in_index[k]];
          const float scale = lds_tab ? tb[0][k] : a.in_scale[k];
          const float shift = lds_tab ? tb[1][k] : a.in_shift[k];
          const float miss = lds_tab ? tb[2][k] : a.in_missing[k];
          z = xv == xv ? fmaf(xv, scale, shift) : miss;
          bad = bad || (z != z);
          z = z == z ? z : 0.f;
        }
        v[j] = z;
      }
    }
    if constexpr (F32) {
      f32x4* o = reinterpret_cast<f32x4*>(static_cast<float*>(a.H) + (size_t)row * a.ldh + chunk * 8);
      o[0] = f32x4{v[0], v[1], v[2], v[3]};
      o[1] = f32x4{v[4], v[5], v[6], v[7]};
    } else {
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = (__bf16)v[j];
      *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.H) + (size_t)row * a.ldh + chunk * 8) = b;
    }
  }
  const unsigned long long m = __ballot(bad);
  const int lane = threadIdx.x & 63;
  const int g0 = lane & ~(GP - 1);
  const unsigned long long grp = GP == 64 ? ~0ull : ((1ull << GP) - 1) << g0;
  if (active && lc == 0) a.row_ok[row] = (live_row && (m & grp) == 0) ? 1 : 0;
}

__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// Stage one 128-byte-per-row slice of `nrows` rows of a matrix with row pitch `ldb` bytes,
// starting at byte column `kb0`, into a swizzled LDS image.
// Instruction q of the block covers 1 KiB = 8 rows; lane L lands at byte q*1024 + 16 L.
// LDS chunk swizzle of row r: (r >> 1) & 7. Two 128-byte rows share one 256-byte bank row, so the
// 16 rows a ds_read_b128 lane group reads need 16 distinct (row parity, chunk) slots — this is
// conflict-free; r & 7 left rows r and r + 8 on one slot (2-way: SQ_LDS_BANK_CONFLICT 1.9e9 -> 0,
// LDS busy -40 %, same wall time in this barrier-bound loop, profiles/r3ak).
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

template <int NROWS, int NW = 8>
__device__ __forceinline__ void stage_slice(const unsigned char* src, size_t ldb, size_t kb0, unsigned char* img,
                                            int wave, int lane) {
  constexpr int NINSTR = NROWS / 8;
  constexpr int PER_WAVE = (NINSTR + NW - 1) / NW;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int q = wave * PER_WAVE + i;
    if (NINSTR % NW == 0 || q < NINSTR) {
      const int p = q * 64 + lane;
      const int r = p >> 3;
      const int c = (p & 7) ^ swz(r);
      glds16(src + (size_t)r * ldb + kb0 + 16 * c, img + q * 1024);
    }
  }
}

template <typename V = bf16x8>
__device__ __forceinline__ V frag(const unsigned char* img, int r, int c) {
  return *reinterpret_cast<const V*>(img + r * SLICE_B + (((c ^ swz(r)) & 7) << 4));
}

__device__ __noinline__ float activate_any(int act, float z, float thr) { return activate(act, z, thr); }

// Two floats -> one word of two bf16 (round to nearest even, lo = a): ONE v_cvt_pk_bf16_f32
// (scalar (__bf16) casts cost a conversion per value plus an SDWA or to merge them).
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}

template <int ACT>
__device__ __forceinline__ float act_of(float z, int act, float thr) {
  if constexpr (ACT == A_IDENTITY) return z;
  else if constexpr (ACT == A_RELU) return fmaxf(z, 0.f);
  else if constexpr (ACT == A_LOGISTIC) return 1.0f / (1.0f + __expf(-z));
  else if constexpr (ACT == A_TANH) return tanhf(z);
  else return activate_any(act, z, thr);
}

// Hidden-layer epilogue: D[row][unit] (unit = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h) +
// bias, activation, bf16; even lanes store the (unit, unit + 1) pair as one 32-bit word, straight
// from the registers. (Staging the 256 x 256 tile through LDS for full-row 16-byte stores was
// measured SLOWER — 3.02 vs 2.62 ms for a 1024 x 1024 layer over 1M rows, profiles/r3l: with one
// workgroup per CU the block-wide barrier exposes the whole store phase, while direct stores
// drain behind the other waves' MFMAs.)
template <int ACT, int TM, int TN, bool F32>
__device__ __forceinline__ void store_hidden(const GemmArgs& a, const f32x16 (&acc)[TM][TN], int row0, int col0,
                                             int wm, int wn, int lane) {
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int unit = col0 + (wn * TN + j) * 32 + l32;
    const float b = a.bias[unit];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = row0 + (wm * TM + i) * 32 + 4 * h;
      if constexpr (F32) {  // 32 consecutive units per half-wave: one 128-byte segment per store.
        // One running pointer (rows rb + 0..3, +8..11, ...) instead of a 64-bit address per store.
        float* p = static_cast<float*>(a.C) + (size_t)rb * a.ldc + unit;
        const size_t ld = (size_t)a.ldc;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          *p = act_of<ACT>(acc[i][j][r] + b, a.act, a.thr);
          p += (r & 3) == 3 ? 5 * ld : ld;
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = act_of<ACT>(acc[i][j][r] + b, a.act, a.thr);
        const float o = __shfl_xor(v, 1);
        const uint32_t lo = __builtin_bit_cast(uint16_t, (__bf16)v);
        const uint32_t hi = __builtin_bit_cast(uint16_t, (__bf16)o);
        if ((lane & 1) == 0) {
          const int row = rb + (r & 3) + 8 * (r >> 2);
          *reinterpret_cast<uint32_t*>(static_cast<__bf16*>(a.C) + (size_t)row * a.ldc + unit) = lo | (hi << 16);
        }
      }
    }
  }
}

// Hidden-layer epilogue for TRANSPOSED accumulators (the operands swapped, mma_quad<true>: the
// tile is [unit][row] — a row per lane, units (r & 3) + 8 (r >> 2) + 4 h in the registers). After
// bias, activation and bf16 a lane holds four 8-byte unit runs of its row; one v_permlane32_swap per
// dword pair trades runs between the lane halves so that every lane owns two whole 16-byte runs
// (units 0-7 and 16-23 in the low half, 8-15 and 24-31 in the high half) and stores them straight
// from the registers: 2 full-width stores per lane per 32 x 32 tile instead of 16 two-unit stores
// by half the lanes, no LDS, no barrier. Default for the bf16 hidden kernels; flag bit 8 (0x100)
// selects store_hidden.
// LB: bl holds the column tile's 256 biases in LDS (16-byte reads) instead of a.bias.
template <int ACT, int TM, int TN, bool LB>
__device__ __forceinline__ void store_hidden_t(const GemmArgs& a, const f32x16 (&acc)[TM][TN], int row0, int col0,
                                               int wm, int wn, int lane, const float* bl) {
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int u0 = col0 + (wn * TN + j) * 32;
    float b[16];
    if constexpr (LB) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(bl + (wn * TN + j) * 32 + 8 * q + 4 * h);
        b[4 * q] = v.x, b[4 * q + 1] = v.y, b[4 * q + 2] = v.z, b[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) b[r] = a.bias[u0 + (r & 3) + 8 * (r >> 2) + 4 * h];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      uint32_t p[8];  // p[2q], p[2q + 1]: units 8q + 4h + 0..3 as bf16 pairs
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        const float v0 = act_of<ACT>(acc[i][j][2 * w] + b[2 * w], a.act, a.thr);
        const float v1 = act_of<ACT>(acc[i][j][2 * w + 1] + b[2 * w + 1], a.act, a.thr);
        p[w] = pack_bf16x2(v0, v1);
      }
      // swap(X, Y): X keeps the low half's own X and takes the low half's Y into the high half;
      // Y takes the high half's X into the low half — runs (q, q + 1) become the 16-byte run 2q + h
      uint4 c[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const auto x0 = __builtin_amdgcn_permlane32_swap(p[4 * s + 0], p[4 * s + 2], false, false);
        const auto x1 = __builtin_amdgcn_permlane32_swap(p[4 * s + 1], p[4 * s + 3], false, false);
        c[s] = make_uint4(x0[0], x1[0], x0[1], x1[1]);
      }
      const size_t row = (size_t)(row0 + (wm * TM + i) * 32 + l32);
      __bf16* dst = static_cast<__bf16*>(a.C) + row * a.ldc + u0 + 8 * h;
      *reinterpret_cast<uint4*>(dst) = c[0];
      *reinterpret_cast<uint4*>(dst + 16) = c[1];
    }
  }
}

// 128-byte ROW-SEGMENT stores of the transposed accumulators (K = 64 persistent kernel, VERDICT r4
// item 4). store_hidden_t leaves a 32 x 32 tile as 16-byte stores whose 64 lanes sit on 32 rows —
// every store instruction touches 32 cache lines, and the K = 64 layer, which writes 2 GB per 1M
// rows, is bound by the address unit (TA 78 % busy, profiles/r4ad). Here a pair of 32-unit tiles
// (one 128-byte segment of a row) is packed to bf16 per tile, the pair's rows pass through a
// 2 KiB wave-private LDS scratch 16 rows at a time (16-byte chunks XOR-swizzled by row & 7: both
// the staging writes and the segment reads are conflict free), and each global store instruction
// covers 8 whole 128-byte row segments (8 lines). Same store count (4 per tile pair and 32 rows),
// same values; only the wave's own lanes touch its scratch, so no barrier.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// NTS: non-temporal stores (the nt bit: streamed past the caches' retention; gemm_k64p_kernel)
// IB / IE: only the accumulator rows i in [IB, IE) (the persistent kernel stores a tile in halves)
template <int ACT, int TM, int TN, bool LB = true, bool NTS = false, int IB = 0, int IE = TM>
__device__ __forceinline__ void store_hidden_seg(const GemmArgs& a, const f32x16 (&acc)[TM][TN], int row0, int col0,
                                                 int wm, int wn, int lane, const float* bl, unsigned char* ws) {
  static_assert(TN % 2 == 0, "tile pairs");
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int i = IB; i < IE; ++i) {
#pragma unroll
    for (int jp = 0; jp < TN / 2; ++jp) {
      uint4 c[2][2];  // [tile of the pair][run]: runs at chunks h, 2 + h of the tile's 64 bytes
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * jp + jj;
        float b[16];
        if constexpr (LB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = *reinterpret_cast<const float4*>(bl + (wn * TN + j) * 32 + 8 * q + 4 * h);
            b[4 * q] = v.x, b[4 * q + 1] = v.y, b[4 * q + 2] = v.z, b[4 * q + 3] = v.w;
          }
        } else {
          const int ub = col0 + (wn * TN + j) * 32;
#pragma unroll
          for (int r = 0; r < 16; ++r) b[r] = a.bias[ub + (r & 3) + 8 * (r >> 2) + 4 * h];
        }
        uint32_t p[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
          const float v0 = act_of<ACT>(acc[i][j][2 * w] + b[2 * w], a.act, a.thr);
          const float v1 = act_of<ACT>(acc[i][j][2 * w + 1] + b[2 * w + 1], a.act, a.thr);
          p[w] = pack_bf16x2(v0, v1);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const auto x0 = __builtin_amdgcn_permlane32_swap(p[4 * s + 0], p[4 * s + 2], false, false);
          const auto x1 = __builtin_amdgcn_permlane32_swap(p[4 * s + 1], p[4 * s + 3], false, false);
          c[jj][s] = make_uint4(x0[0], x1[0], x0[1], x1[1]);
        }
      }
      const int u0 = col0 + (wn * TN + 2 * jp) * 32;  // first unit of the pair's 128-byte segment
      const size_t rb = (size_t)(row0 + (wm * TM + i) * 32);
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        if ((l32 >> 4) == ph) {  // rows 16 ph .. 16 ph + 15 stage their 4 x 16 bytes per lane
          const int r = l32 & 15;
          unsigned char* rowp = ws + r * 128;
          const int sw = r & 7;
          *reinterpret_cast<uint4*>(rowp + (((0 + h) ^ sw) << 4)) = c[0][0];
          *reinterpret_cast<uint4*>(rowp + (((2 + h) ^ sw) << 4)) = c[0][1];
          *reinterpret_cast<uint4*>(rowp + (((4 + h) ^ sw) << 4)) = c[1][0];
          *reinterpret_cast<uint4*>(rowp + (((6 + h) ^ sw) << 4)) = c[1][1];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // lane L: chunk L & 7 of rows L >> 3 and 8 + (L >> 3) (LDS hands a wave's ops back in order)
        const int rr = lane >> 3, k = lane & 7;
        const uint4 v0 = *reinterpret_cast<const uint4*>(ws + rr * 128 + ((k ^ (rr & 7)) << 4));
        const uint4 v1 = *reinterpret_cast<const uint4*>(ws + (rr + 8) * 128 + ((k ^ ((rr + 8) & 7)) << 4));
        __bf16* d0 = static_cast<__bf16*>(a.C) + (rb + 16 * ph + rr) * a.ldc + u0 + 8 * k;
        if constexpr (NTS) {
          __builtin_nontemporal_store(u32x4{v0.x, v0.y, v0.z, v0.w}, reinterpret_cast<u32x4*>(d0));
          __builtin_nontemporal_store(u32x4{v1.x, v1.y, v1.z, v1.w}, reinterpret_cast<u32x4*>(d0 + 8 * (size_t)a.ldc));
        } else {
          *reinterpret_cast<uint4*>(d0) = v0;
          *reinterpret_cast<uint4*>(d0 + 8 * (size_t)a.ldc) = v1;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
}

template <int TM, int TN, bool LB = true, bool NTS = false, int IB = 0, int IE = TM>
__device__ __forceinline__ void store_hidden_seg_any(const GemmArgs& a, const f32x16 (&acc)[TM][TN], int row0,
                                                     int col0, int wm, int wn, int lane, const float* bl,
                                                     unsigned char* ws) {
  switch (a.act) {
    case A_IDENTITY: store_hidden_seg<A_IDENTITY, TM, TN, LB, NTS, IB, IE>(a, acc, row0, col0, wm, wn, lane, bl, ws); break;
    case A_RELU: store_hidden_seg<A_RELU, TM, TN, LB, NTS, IB, IE>(a, acc, row0, col0, wm, wn, lane, bl, ws); break;
    case A_LOGISTIC: store_hidden_seg<A_LOGISTIC, TM, TN, LB, NTS, IB, IE>(a, acc, row0, col0, wm, wn, lane, bl, ws); break;
    case A_TANH: store_hidden_seg<A_TANH, TM, TN, LB, NTS, IB, IE>(a, acc, row0, col0, wm, wn, lane, bl, ws); break;
    default: store_hidden_seg<-1, TM, TN, LB, NTS, IB, IE>(a, acc, row0, col0, wm, wn, lane, bl, ws); break;
  }
}

template <int TM, int TN, bool LB = false>
__device__ __forceinline__ void store_hidden_t_any(const GemmArgs& a, const f32x16 (&acc)[TM][TN], int row0, int col0,
                                                   int wm, int wn, int lane, const float* bl = nullptr) {
  switch (a.act) {
    case A_IDENTITY: store_hidden_t<A_IDENTITY, TM, TN, LB>(a, acc, row0, col0, wm, wn, lane, bl); break;
    case A_RELU: store_hidden_t<A_RELU, TM, TN, LB>(a, acc, row0, col0, wm, wn, lane, bl); break;
    case A_LOGISTIC: store_hidden_t<A_LOGISTIC, TM, TN, LB>(a, acc, row0, col0, wm, wn, lane, bl); break;
    case A_TANH: store_hidden_t<A_TANH, TM, TN, LB>(a, acc, row0, col0, wm, wn, lane, bl); break;
    default: store_hidden_t<-1, TM, TN, LB>(a, acc, row0, col0, wm, wn, lane, bl); break;
  }
}

// Output-layer decode of one row from its n_out activated output units z[]: the regression
// affine + Target epilogue, or softmax / simplemax, probabilities, argmax and the label table.
__device__ __forceinline__ void decode_row(const GemmArgs& a, int row, const float* z) {
  const bool bad = !a.row_ok[row];
  if (a.final_norm == 0 && a.n_out == 1) {
    apply_epilogue(a.epi, [&](int) { return z[0]; }, !bad, row, a.rows, a.score, a.valid, a.probs);
    return;
  }
  float mx = -__builtin_inff();
  for (int u = 0; u < a.n_out; ++u) mx = fmaxf(mx, z[u]);
  float sum = 0.f;
  for (int u = 0; u < a.n_out; ++u) sum += (a.final_norm == 1) ? __expf(z[u] - mx) : z[u];
  float best = -__builtin_inff();
  int best_u = 1 << 30;
  for (int u = 0; u < a.n_out; ++u) {
    float p = (a.final_norm == 1) ? __expf(z[u] - mx) : z[u];
    if (a.final_norm != 0) p /= sum;
    if (p > best || (p == best && u < best_u)) { best = p; best_u = u; }
    if (a.probs) a.probs[(size_t)row * a.n_out + u] = p;
  }
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

// Hidden-layer epilogue through a wave-private LDS scratch (bf16; opt-in, flag bit 5 — measured
// slower than the direct stores: 2.70 vs 2.60 ms for a 1024 x 1024 layer, 0.99 vs 0.84 ms for the
// K = 64 layer, profiles/r4k). Each 32 x 32 accumulator tile
// (a unit per lane, 16 rows in the registers) is written to the wave's own 2.5 KiB of LDS as bf16
// pairs and read back as 16-byte row chunks, so the tile leaves in 2 full-width 16-byte global
// stores per lane instead of 16 two-unit stores by half the lanes — the store instruction count,
// not the bytes, bounds a store-heavy epilogue. No block barrier: a wave's LDS operations complete
// in order. Rows padded to 80 B so the two lane halves' rows (r, r + 4) use different banks.
constexpr int WEPI_RP = 80;                    // bytes per scratch row
constexpr int WEPI_BYTES = 32 * WEPI_RP;       // per wave

template <int ACT, int TM, int TN>
__device__ __forceinline__ void store_hidden_wave(const GemmArgs& a, const f32x16 (&acc)[TM][TN], int row0, int col0,
                                                  int wm, int wn, int lane, unsigned char* scratch) {
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int u0 = col0 + (wn * TN + j) * 32;
    const float b = a.bias[u0 + l32];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = row0 + (wm * TM + i) * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = act_of<ACT>(acc[i][j][r] + b, a.act, a.thr);
        const float o = __shfl_xor(v, 1);
        if ((lane & 1) == 0) {
          const uint32_t lo = __builtin_bit_cast(uint16_t, (__bf16)v);
          const uint32_t hi = __builtin_bit_cast(uint16_t, (__bf16)o);
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          *reinterpret_cast<uint32_t*>(scratch + row * WEPI_RP + 2 * l32) = lo | (hi << 16);
        }
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int q = 0; q < 2; ++q) {  // chunk c = lane + 64 q: row c >> 2, 16-byte part c & 3
        const int c = lane + 64 * q;
        const uint4 v = *reinterpret_cast<const uint4*>(scratch + (c >> 2) * WEPI_RP + 16 * (c & 3));
        *reinterpret_cast<uint4*>(static_cast<__bf16*>(a.C) + (size_t)(rb + (c >> 2)) * a.ldc + u0 + 8 * (c & 3)) = v;
      }
      asm volatile("" ::: "memory");
    }
  }
}

template <int TM, int TN>
__device__ __forceinline__ void store_hidden_wave_any(const GemmArgs& a, const f32x16 (&acc)[TM][TN], int row0,
                                                      int col0, int wm, int wn, int lane, unsigned char* scratch) {
  switch (a.act) {
    case A_IDENTITY: store_hidden_wave<A_IDENTITY, TM, TN>(a, acc, row0, col0, wm, wn, lane, scratch); break;
    case A_RELU: store_hidden_wave<A_RELU, TM, TN>(a, acc, row0, col0, wm, wn, lane, scratch); break;
    case A_LOGISTIC: store_hidden_wave<A_LOGISTIC, TM, TN>(a, acc, row0, col0, wm, wn, lane, scratch); break;
    case A_TANH: store_hidden_wave<A_TANH, TM, TN>(a, acc, row0, col0, wm, wn, lane, scratch); break;
    default: store_hidden_wave<-1, TM, TN>(a, acc, row0, col0, wm, wn, lane, scratch); break;
  }
}

template <int BN, bool HEAD, bool F32, bool TST = false>
__global__ __launch_bounds__(NT, 1) void gemm_kernel(GemmArgs a) {
  static_assert(!TST || (!HEAD && !F32), "transposed stores: bf16 hidden layers");
  constexpr int WM = BN == 256 ? 2 : 8;  // waves along rows
  constexpr int WN = 8 / WM;             // waves along units
  constexpr int TM = BM / WM / 32;       // 32-row accumulator tiles per wave
  constexpr int TN = BN / WN / 32;       // 32-unit accumulator tiles per wave
  constexpr int ES = F32 ? 4 : 2;          // element bytes
  constexpr int SK = SLICE_B / ES;          // k per slice
  constexpr int A_BYTES = BM * SLICE_B;
  constexpr int B_BYTES = BN * SLICE_B;
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned char* As = smem;
  unsigned char* Bs = smem + 2 * A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int n_ct = a.Mp / BN;
  const int total = (a.rows_p / BM) * n_ct;
  int t = blockIdx.x;
  if ((total & 7) == 0) t = (t & 7) * (total >> 3) + (t >> 3);  // XCD-contiguous tile ranges
  const int row0 = (t / n_ct) * BM;
  const int col0 = (t % n_ct) * BN;
  const int wm = wave / WN, wn = wave % WN;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const size_t lda_b = (size_t)a.lda * ES, ldw_b = (size_t)a.ldw * ES;
  const unsigned char* Ab = static_cast<const unsigned char*>(a.A) + (size_t)row0 * lda_b;
  const unsigned char* Bb = static_cast<const unsigned char*>(a.Wt) + (size_t)col0 * ldw_b;
  const int KT = a.K / SK;
  stage_slice<BM>(Ab, lda_b, 0, As, wave, lane);
  stage_slice<BN>(Bb, ldw_b, 0, Bs, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) {  // next slice in flight while this one computes
      stage_slice<BM>(Ab, lda_b, (size_t)(kt + 1) * SLICE_B, As + (cur ^ 1) * A_BYTES, wave, lane);
      stage_slice<BN>(Bb, ldw_b, (size_t)(kt + 1) * SLICE_B, Bs + (cur ^ 1) * B_BYTES, wave, lane);
    }
    const unsigned char* ai = As + cur * A_BYTES;
    const unsigned char* bi = Bs + cur * B_BYTES;
    if constexpr (F32) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // chunk 2g + h: 4 k per lane, one MFMA each
        f32x4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag<f32x4>(ai, (wm * TM + i) * 32 + l32, 2 * g + h);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag<f32x4>(bi, (wn * TN + j) * 32 + l32, 2 * g + h);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][e], bfr[j][e], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag(ai, (wm * TM + i) * 32 + l32, 2 * ks + h);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag(bi, (wn * TN + j) * 32 + l32, 2 * ks + h);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = TST ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_waitcnt(0);  // the slice in flight has landed (LDS-DMA retires on vmcnt)
    __syncthreads();                // ... for every wave before anyone reads / overwrites it
  }

  if constexpr (TST) {
    store_hidden_t_any<TM, TN>(a, acc, row0, col0, wm, wn, lane);
  } else if constexpr (!HEAD) {
    switch (a.act) {  // uniform: one unrolled epilogue per common activation
      case A_IDENTITY: store_hidden<A_IDENTITY, TM, TN, F32>(a, acc, row0, col0, wm, wn, lane); break;
      case A_RELU: store_hidden<A_RELU, TM, TN, F32>(a, acc, row0, col0, wm, wn, lane); break;
      case A_LOGISTIC: store_hidden<A_LOGISTIC, TM, TN, F32>(a, acc, row0, col0, wm, wn, lane); break;
      case A_TANH: store_hidden<A_TANH, TM, TN, F32>(a, acc, row0, col0, wm, wn, lane); break;
      default: store_hidden<-1, TM, TN, F32>(a, acc, row0, col0, wm, wn, lane); break;
    }
  } else {
    float* zt = reinterpret_cast<float*>(smem);  // [BM][HEAD_LD] (the staging buffers are drained)
    const int unit = l32;
    const float b = unit < a.n_out ? a.bias[unit] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = (wm * TM) * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
      zt[rl * HEAD_LD + unit] = activate(a.act, acc[0][0][r] + b, a.thr);
    }
    __syncthreads();
    if (tid < BM) {
      const int row = row0 + tid;
      if (row < a.rows) {
        if (a.C) {  // one 32-output group of a wider output layer: its activated outputs (fp32)
          float* zo = static_cast<float*>(a.C) + (size_t)row * a.ldc;
          for (int u = 0; u < a.n_out; ++u) zo[u] = zt[tid * HEAD_LD + u];
        } else {
          decode_row(a, row, zt + tid * HEAD_LD);
        }
      }
    }
  }
}

// Decode of an output layer wider than one 32-unit tile: Z holds every row's activated outputs
// (fp32, row pitch ldz), written group by group by the output-layer GEMM. Streaming passes (max,
// normaliser, probabilities + argmax) — no per-row array, any n_out.
__global__ __launch_bounds__(256) void nn_decode_wide_kernel(GemmArgs a, const float* __restrict__ Z, int ldz) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= a.rows) return;
  const float* z = Z + (size_t)row * ldz;
  const bool bad = !a.row_ok[row];
  float mx = -__builtin_inff();
  for (int u = 0; u < a.n_out; ++u) mx = fmaxf(mx, z[u]);
  float sum = 0.f;
  for (int u = 0; u < a.n_out; ++u) sum += (a.final_norm == 1) ? __expf(z[u] - mx) : z[u];
  float best = -__builtin_inff();
  int best_u = 1 << 30;
  for (int u = 0; u < a.n_out; ++u) {
    float p = (a.final_norm == 1) ? __expf(z[u] - mx) : z[u];
    if (a.final_norm != 0) p /= sum;
    if (p > best || (p == best && u < best_u)) { best = p; best_u = u; }
    if (a.probs) a.probs[(size_t)row * a.n_out + u] = p;
  }
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

// First hidden layer over a narrow input (bf16, K = 64: one slice). The layer is bound by its
// output (2 bytes per unit, ~2 GB for 1M rows x 1024 units), not by its 16 MFMAs per wave: the
// 256 x 256 / 8-wave tile of gemm_kernel holds a whole CU (128 KiB LDS), so every tile's load
// latency, MFMAs and stores run back to back. Here a 128 x 256 tile on 4 waves (48 KiB LDS,
// 2 x 4 accumulators per wave) lets three workgroups share a CU — one drains its stores while
// the others load and multiply.
// PREP: the input stage fused in (nn_prep_kernel's gather, NormContinuous, missing values, bf16 and
// row validity): the A tile is built from the raw records straight into the swizzled LDS image
// (no [rows, 64] bf16 round trip through HBM, no separate launch); column tile 0 writes row_ok.
constexpr int K64_BM = 128, K64_NT = 256;

template <bool PREP, bool TST>
__global__ __launch_bounds__(K64_NT, 2) void gemm_k64_kernel(GemmArgs a, PrepArgs p) {
  constexpr int TM = 2, TN = 4;  // 2 x 2 waves, 64 rows x 128 units each
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned char* As = smem;
  unsigned char* Bs = smem + K64_BM * SLICE_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int n_ct = a.Mp / 256;
  const int total = (a.rows_p / K64_BM) * n_ct;
  int t = blockIdx.x;
  if ((total & 7) == 0) t = (t & 7) * (total >> 3) + (t >> 3);  // XCD-contiguous tile ranges
  const int row0 = (t / n_ct) * K64_BM;
  const int col0 = (t % n_ct) * 256;
  const int wm = wave >> 1, wn = wave & 1;
  const size_t lda_b = (size_t)a.lda * 2, ldw_b = (size_t)a.ldw * 2;
  stage_slice<256, 4>(static_cast<const unsigned char*>(a.Wt) + (size_t)col0 * ldw_b, ldw_b, 0, Bs, wave, lane);
  if constexpr (PREP) {
    // item it = row r (of the tile) x 8-input chunk c; a row's 8 chunks are 8 consecutive lanes
#pragma unroll 1
    for (int q = 0; q < K64_BM * 8 / K64_NT; ++q) {
      const int it = tid + K64_NT * q;
      const int r = it >> 3, c = it & 7;
      const int row = row0 + r;
      const bool live = row < p.n_rows;
      const float* x = p.X + (size_t)(live ? row : 0) * p.ldx;
      bool bad = false;
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * c + j;
        float z = 0.f;
        if (live && k < p.n_in) {
          const float xv = x[p.in_index[k]];
          z = xv == xv ? fmaf(xv, p.in_scale[k], p.in_shift[k]) : p.in_missing[k];
          bad = bad || (z != z);
          z = z == z ? z : 0.f;
        }
        b[j] = (__bf16)z;
      }
      *reinterpret_cast<bf16x8*>(As + r * SLICE_B + (((c ^ swz(r)) & 7) << 4)) = b;
      const unsigned long long m = __ballot(bad);
      if (col0 == 0 && c == 0) p.row_ok[row] = (live && ((m >> (lane & ~7)) & 0xFFull) == 0) ? 1 : 0;
    }
  } else {
    stage_slice<K64_BM, 4>(static_cast<const unsigned char*>(a.A) + (size_t)row0 * lda_b, lda_b, 0, As, wave, lane);
  }
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
#pragma unroll
  for (int ks = 0; ks < BK / 16; ++ks) {
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = frag(As, (wm * TM + i) * 32 + l32, 2 * ks + h);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = frag(Bs, (wn * TN + j) * 32 + l32, 2 * ks + h);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = TST ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0)
                        : __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
  if constexpr (TST) {
    store_hidden_t_any<TM, TN>(a, acc, row0, col0, wm, wn, lane);
    return;
  }
  if ((a.f32 >> 5) & 1) {  // bit 5: the wave-private LDS epilogue (measured slower, profiles/r4k)
    __syncthreads();  // every wave is done reading the staged tiles: their LDS becomes scratch
    store_hidden_wave_any<TM, TN>(a, acc, row0, col0, wm, wn, lane, smem + wave * WEPI_BYTES);
    return;
  }
  switch (a.act) {
    case A_IDENTITY: store_hidden<A_IDENTITY, TM, TN, false>(a, acc, row0, col0, wm, wn, lane); break;
    case A_RELU: store_hidden<A_RELU, TM, TN, false>(a, acc, row0, col0, wm, wn, lane); break;
    case A_LOGISTIC: store_hidden<A_LOGISTIC, TM, TN, false>(a, acc, row0, col0, wm, wn, lane); break;
    case A_TANH: store_hidden<A_TANH, TM, TN, false>(a, acc, row0, col0, wm, wn, lane); break;
    default: store_hidden<-1, TM, TN, false>(a, acc, row0, col0, wm, wn, lane); break;
  }
}

// ---------------------------------------------------------------------------------------------
// Hidden layers, bf16, phase-interleaved (gemm8_kernel). Same 256 x 256 tile, BK = 64 slices, 8
// waves with a 128 x 64 sub-tile each (4 x 2 accumulators of 32x32x16), but:
//  * each slice is staged as four 16 KiB half-tiles — A0 / A1: the first / second 64 rows of
//    each wave row-group's 128, B0 / B1: the first / second 32 units of each wave column's 64 —
//    into two buffers of four slots;
//  * a slice is consumed in four phases, one output quadrant each: P1 A0 x B0 (reads A0, B0),
//    P2 A0 x B1 (reads B1), P3 A1 x B1 (reads A1), P4 A1 x B0 (no reads, B0 kept in registers);
//    a phase = its fragment reads + one half-tile LDS-DMA, lgkmcnt(0), raw barrier, 8 MFMAs,
//    raw barrier;
//  * a slot is restaged one phase after the barrier that ends its last read: P1 stages A1 of
//    slice t + 1 (into the other buffer), P2 / P3 / P4 stage A0 / B0 / B1 of slice t + 2 into
//    the slots P1 / P1 / P2 freed, and ONE counted vmcnt(6) per slice (at P4, after its issue)
//    retires everything of slice t + 1 while three half-tiles of t + 2 stay in flight across
//    the barriers (__syncthreads() would add vmcnt(0));
//  * the two wave row-groups run one barrier apart (group 1 passes one extra barrier first), so
//    on every SIMD one wave's MFMAs overlap the other wave's fragment reads and staging.
// Hazards, by barrier matching (group 1's n-th barrier is group 0's (n+1)-th): a wave reads a
// slice only after a barrier that every wave reached after its vmcnt for that slice; a wave
// restages a slot only after a barrier that every wave reached after lgkmcnt(0) on its reads of
// the slot's previous contents.
// ---------------------------------------------------------------------------------------------
constexpr int HALF_B = 128 * SLICE_B;  // one half-tile slot: 128 rows x 128 B

// Half-tile `half` of a slice: slot row j <- A row (j >> 6) * 128 + half * 64 + (j & 63), or
// weight row (unit) (j >> 5) * 64 + half * 32 + (j & 31). Two 1 KiB LDS-DMA instructions per wave.
template <bool IS_A>
__device__ __forceinline__ void stage_half(const unsigned char* src, size_t ldb, size_t kb0, unsigned char* slot,
                                           int half, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave * 2 + i;
    const int p = q * 64 + lane;
    const int j = p >> 3;
    const int c = (p & 7) ^ swz(j);
    const int r = IS_A ? ((j >> 6) * 128 + half * 64 + (j & 63)) : ((j >> 5) * 64 + half * 32 + (j & 31));
    glds16(src + (size_t)r * ldb + kb0 + 16 * c, slot + q * 1024);
  }
}

// stage_half as inline-asm LDS-DMA in the SADDR form: 64-bit wave-uniform base (the tile's first
// row + the slice's byte column) in SGPRs, a 32-bit per-lane offset in one VGPR, the LDS
// destination in M0. For the persistent kernel, whose register budget is exhausted: hipcc keeps
// the builtin's per-lane 64-bit addresses (16 VGPRs) loop-invariant and spilled them, with a
// vmcnt(0) per reload in the loop. Invisible to hipcc's wait-count pass, which is what the kernel
// wants: every wait on these loads is an explicit counted vmcnt already, and hipcc no longer
// drains them before the epilogue's LDS accesses. ldb * 256 rows must fit 32 bits (launcher).
// M0 is clobbered (hipcc notes it cannot preserve a reserved register): none of the gemm8p_kernel
// instantiations uses M0 outside these statements (checked in the generated .s).
__device__ __forceinline__ void glds16s(const unsigned char* sbase, uint32_t voff, const unsigned char* lds) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(m), "v"(voff), "s"(sbase)
               : "memory", "m0");
}
template <bool IS_A>
__device__ __forceinline__ void stage_half_s(const unsigned char* src, uint32_t ldb, unsigned char* slot, int half,
                                             int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave * 2 + i;
    const int p = q * 64 + lane;
    const int j = p >> 3;
    const int c = (p & 7) ^ swz(j);
    const int r = IS_A ? ((j >> 6) * 128 + half * 64 + (j & 63)) : ((j >> 5) * 64 + half * 32 + (j & 31));
    glds16s(src, (uint32_t)r * ldb + 16u * (uint32_t)c, slot + q * 1024);
  }
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// A phase: reads issued -> mma_begin (lgkmcnt(0), barrier, high priority) -> MFMAs -> mma_end.
__device__ __forceinline__ void mma_begin() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  __builtin_amdgcn_s_setprio(1);
}
__device__ __forceinline__ void mma_end() {
  __builtin_amdgcn_s_setprio(0);
  raw_barrier();
}

// acc[i0 + i][j] += a[i] . b over the slice's four k16 steps. The empty volatile asm on the
// accumulators pins the MFMAs between the phase's two barriers (register-only instructions are
// otherwise free to sink past them; sched_barrier alone did not keep them there).
// SWAP: the transposed product (weights as the A operand): the accumulator tile is [unit][row],
// a row per lane and the units in the registers — the layout a following MFMA takes as its B
// operand with no lane movement (the fused output layer of gemm8_kernel<true>).
template <bool SWAP = false>
__device__ __forceinline__ void mma_quad(f32x16& c0, f32x16& c1, const bf16x8 (&a)[2][4], const bf16x8 (&b)[4]) {
  asm volatile("" : "+v"(c0), "+v"(c1));
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    if constexpr (SWAP) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[ks], a[0][ks], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[ks], a[1][ks], c1, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][ks], b[ks], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][ks], b[ks], c1, 0, 0, 0);
    }
  }
  asm volatile("" : "+v"(c0), "+v"(c1));
}

struct HeadFuse {
  const __bf16* wh;  // [32][ldw] output-layer weights, k permuted within 32-unit groups (fuse_head_perm)
  float* part;       // [Mp / 256][rows_p][n_out] per-column-tile partial output sums
  int ldw, n_out;
};

// Fused output layer (gemm8_kernel<true>, the last hidden layer): the accumulators hold the
// transposed tile [unit][row] (mma_quad<true>), so bias + activation + bf16 of 8 consecutive
// registers IS an MFMA B fragment [k = unit][col = row] — with the output-layer weights' k order
// permuted the same way on the host (fuse_head_perm), Z[out][row] = Wh · H accumulates with no
// lane movement, no LDS round trip and no store of the hidden layer. The four column waves of a
// row group leave their Z in LDS and the block writes the in-order sum, its [256, n_out] partial,
// to hf.part[column tile] (deterministic); nn_head_decode_kernel sums the column tiles in order
// and decodes.
// LW (the persistent kernel): the output-layer weights' first n_out rows come from an LDS copy
// whl [n_out][Mp] (rows >= n_out are zero in hf.wh) and the partial-sum exchange uses a raw barrier
// — no global load and no fence in the epilogue, so nothing makes hipcc wait for vector memory
// (the next tile's LDS-DMA loads are in flight).
template <int ACT, bool LW = false>
__device__ __forceinline__ void head_partial(const GemmArgs& a, const HeadFuse& hf, const f32x16 (&acc)[4][2], int row0,
                                             int col0, int wr, int wc, int lane, int tid, unsigned char* smem,
                                             const float* btile, const __bf16* whl = nullptr) {
  const int h = lane >> 5, l32 = lane & 31;
  const int no = hf.n_out;
  float* zp = reinterpret_cast<float*>(smem);  // [4 column waves][BM][n_out] (staging buffers drained / scratch)
  bf16x8 wf[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if constexpr (LW)
        wf[j][s] = l32 < no ? *reinterpret_cast<const bf16x8*>(whl + l32 * a.Mp + col0 + wc * 64 + 32 * j + 16 * s + 8 * h)
                            : bf16x8{};
      else
        wf[j][s] = *reinterpret_cast<const bf16x8*>(hf.wh + (size_t)l32 * hf.ldw + col0 + wc * 64 + 32 * j + 16 * s + 8 * h);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x16 z = f32x16{};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float* bias = btile + wc * 64 + 32 * j + 4 * h;  // btile: the column tile's biases
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 hb;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int r = 8 * s + e;
          hb[e] = (__bf16)act_of<ACT>(acc[i][j][r] + bias[(r & 3) + 8 * (r >> 2)], a.act, a.thr);
        }
        z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[j][s], hb, z, 0, 0, 0);
      }
    }
    // z[r]: output unit o = (r & 3) + 8 (r >> 2) + 4 h of block row wr * 128 + 32 i + l32
    float* dst = zp + ((size_t)wc * BM + wr * 128 + 32 * i + l32) * no;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
      if (o < no) dst[o] = z[r];
    }
  }
  if constexpr (LW) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
  } else {
    __syncthreads();
  }
  float* out = hf.part + ((size_t)(col0 >> 8) * a.rows_p + row0) * no;
  const size_t plane = (size_t)BM * no;
  for (int e = tid; e < BM * no; e += NT) out[e] = ((zp[e] + zp[plane + e]) + zp[2 * plane + e]) + zp[3 * plane + e];
}

template <bool HEADF, bool TST>
__global__ __launch_bounds__(NT, 1) void gemm8_kernel(GemmArgs a, HeadFuse hf) {
  constexpr bool SWAP = HEADF || TST;  // transposed accumulator tiles
  constexpr int TM = 4, TN = 2;  // acc[2 * a_half + tile][b_half]
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int n_ct = a.Mp / 256;
  const int total = (a.rows_p / BM) * n_ct;
  int t = blockIdx.x;
  if ((total & 7) == 0) t = (t & 7) * (total >> 3) + (t >> 3);  // XCD-contiguous tile ranges
  const int row0 = (t / n_ct) * BM;
  const int col0 = (t % n_ct) * 256;
  const int wr = wave >> 2, wc = wave & 3;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const size_t lda_b = (size_t)a.lda * 2, ldw_b = (size_t)a.ldw * 2;
  const unsigned char* Ab = static_cast<const unsigned char*>(a.A) + (size_t)row0 * lda_b;
  const unsigned char* Bb = static_cast<const unsigned char*>(a.Wt) + (size_t)col0 * ldw_b;
  const int KT = a.K / BK;
  // slot s of buffer b: 0 A0, 1 A1, 2 B0, 3 B1
#define SLOT(b, s) (smem + (b) * 4 * HALF_B + (s) * HALF_B)
  stage_half<true>(Ab, lda_b, 0, SLOT(0, 0), 0, wave, lane);
  stage_half<false>(Bb, ldw_b, 0, SLOT(0, 2), 0, wave, lane);
  stage_half<false>(Bb, ldw_b, 0, SLOT(0, 3), 1, wave, lane);
  stage_half<true>(Ab, lda_b, 0, SLOT(0, 1), 1, wave, lane);
  if (KT > 1) {
    stage_half<true>(Ab, lda_b, SLICE_B, SLOT(1, 0), 0, wave, lane);
    stage_half<false>(Bb, ldw_b, SLICE_B, SLOT(1, 2), 0, wave, lane);
    stage_half<false>(Bb, ldw_b, SLICE_B, SLOT(1, 3), 1, wave, lane);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  if (wr == 1) raw_barrier();  // group 1 runs one barrier behind group 0

  const int ra = wr * 64 + l32, rb = wc * 32 + l32;  // slot rows of this lane's fragments
  for (int kt = 0; kt < KT; ++kt) {
    const int b = kt & 1;
    const size_t k1 = (size_t)(kt + 1) * SLICE_B, k2 = (size_t)(kt + 2) * SLICE_B;
    bf16x8 a0[2][4], a1[2][4], b0[4], b1[4];
    // P1: A0 x B0
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
      for (int i = 0; i < 2; ++i) a0[i][ks] = frag(SLOT(b, 0), ra + 32 * i, 2 * ks + h);
      b0[ks] = frag(SLOT(b, 2), rb, 2 * ks + h);
    }
    if (kt + 1 < KT) stage_half<true>(Ab, lda_b, k1, SLOT(b ^ 1, 1), 1, wave, lane);
    mma_begin();
    mma_quad<SWAP>(acc[0][0], acc[1][0], a0, b0);
    mma_end();
    // P2: A0 x B1
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) b1[ks] = frag(SLOT(b, 3), rb, 2 * ks + h);
    if (kt + 2 < KT) stage_half<true>(Ab, lda_b, k2, SLOT(b, 0), 0, wave, lane);
    mma_begin();
    mma_quad<SWAP>(acc[0][1], acc[1][1], a0, b1);
    mma_end();
    // P3: A1 x B1
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i) a1[i][ks] = frag(SLOT(b, 1), ra + 32 * i, 2 * ks + h);
    if (kt + 2 < KT) stage_half<false>(Bb, ldw_b, k2, SLOT(b, 2), 0, wave, lane);
    mma_begin();
    mma_quad<SWAP>(acc[2][1], acc[3][1], a1, b1);
    mma_end();
    // P4: A1 x B0; slice kt + 1 retired (three half-tiles of kt + 2 may stay in flight)
    if (kt + 2 < KT) stage_half<false>(Bb, ldw_b, k2, SLOT(b, 3), 1, wave, lane);
    if (kt + 2 < KT) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mma_begin();
    mma_quad<SWAP>(acc[2][0], acc[3][0], a1, b0);
    mma_end();
  }
#undef SLOT
  if (wr == 0) raw_barrier();  // balance group 1's extra barrier
  if constexpr (HEADF) {
    switch (a.act) {
      case A_IDENTITY: head_partial<A_IDENTITY>(a, hf, acc, row0, col0, wr, wc, lane, tid, smem, a.bias + col0); break;
      case A_RELU: head_partial<A_RELU>(a, hf, acc, row0, col0, wr, wc, lane, tid, smem, a.bias + col0); break;
      case A_LOGISTIC: head_partial<A_LOGISTIC>(a, hf, acc, row0, col0, wr, wc, lane, tid, smem, a.bias + col0); break;
      case A_TANH: head_partial<A_TANH>(a, hf, acc, row0, col0, wr, wc, lane, tid, smem, a.bias + col0); break;
      default: head_partial<-1>(a, hf, acc, row0, col0, wr, wc, lane, tid, smem, a.bias + col0); break;
    }
    return;
  } else if constexpr (TST) {
    if (!((a.f32 >> 11) & 1)) {
      // 128-byte row-segment stores through a 2 KiB wave scratch (the staging slots are drained:
      // every wave is past the balancing barrier above); bit 11: store_hidden_t
      store_hidden_seg_any<TM, TN, false>(a, acc, row0, col0, wr, wc, lane, nullptr, smem + wave * 2048);
    } else {
      store_hidden_t_any<TM, TN>(a, acc, row0, col0, wr, wc, lane);
    }
  } else {
    if ((a.f32 >> 5) & 1) {  // bit 5: the wave-private LDS epilogue (measured slower, profiles/r4k)
      // every wave is past its last LDS read of the staged slices (the balancing barrier above)
      store_hidden_wave_any<TM, TN>(a, acc, row0, col0, wr, wc, lane, smem + wave * WEPI_BYTES);
      return;
    }
    switch (a.act) {
      case A_IDENTITY: store_hidden<A_IDENTITY, TM, TN, false>(a, acc, row0, col0, wr, wc, lane); break;
      case A_RELU: store_hidden<A_RELU, TM, TN, false>(a, acc, row0, col0, wr, wc, lane); break;
      case A_LOGISTIC: store_hidden<A_LOGISTIC, TM, TN, false>(a, acc, row0, col0, wr, wc, lane); break;
      case A_TANH: store_hidden<A_TANH, TM, TN, false>(a, acc, row0, col0, wr, wc, lane); break;
      default: store_hidden<-1, TM, TN, false>(a, acc, row0, col0, wr, wc, lane); break;
    }
  }
}

// Persistent phase-interleaved hidden layer (gemm8p_kernel; bf16, K >= 128: the default of the
// transposed-store path and of the fused output layer; flag bit 12 selects gemm8_kernel / the
// 2-buffer loop).
// gemm8_kernel runs ONE 256 x 256 tile per workgroup; at one workgroup per CU the matrix cores
// idle while a fresh workgroup fills its first slices and while the last one drains its
// epilogue. Here a grid of one workgroup per CU walks a list of tiles and the slice stream of
// gemm8_kernel continues across tile boundaries: global slice g = j * KT + kt of the workgroup's
// j-th tile, buffer g & 1, the same four phases, restaging points and counted vmcnt(6) — the
// first slices of tile j + 1 are staged by the last phases of tile j, and tile j's epilogue runs
// between two phases while they are in flight:
//  * hidden layer: bias from LDS, activation, 128-byte row-segment stores through the wave's own
//    scratch (store_hidden_seg), no barrier. The stores are older than the next slices' loads, so
//    the counted wait of the next tile's first slice retires them too (vector-memory operations
//    retire in issue order);
//  * fused output layer (HEADF, n_out <= 4): head_partial with the biases from LDS and its
//    partial sums in the scratch region, the two wave groups re-aligned around its barrier.
// The LDS-DMA is issued as inline asm (stage_half_s): hipcc kept the builtin's 64-bit per-lane
// addresses live and spilled them (a vmcnt(0) per reload inside the loop) and drained the loads
// in flight before the epilogue's first LDS access; neither happens to loads it cannot see.
// LDS: the 128 KiB of staging slots, 16 KiB of wave scratch / head partials, the Mp biases.
// Tile list: the XCD-contiguous order of gemm8_kernel — XCD x (blockIdx & 7) owns tiles
// [x T / 8, (x + 1) T / 8) and its G / 8 workgroups take every (G / 8)-th of them, so the column
// tiles of a row block run together on one XCD and its A rows come from HBM once.
// Measured (profiles/r5n, r5t; 1M rows, one process, interleaved): 1024 x 1024 2.04 vs 2.23 ms for
// gemm8_kernel<false, true> (without any stores, bit 13, timing only: 1.63 ms); K = 4096 6.92 vs
// 7.42 ms; K = 256 0.25 / 0.47 vs 0.32 / 0.60 ms for the 2-buffer loop (256 / 512 units). (With the
// builtin LDS-DMA the K = 4096 layer was slower persistent, profiles/r5m: 7.71 vs 7.37 ms.)
// Measured and dropped (profiles/r5m, r5n): staging the next tile's A1 before the
// epilogue with the stores left in flight one slice longer (+9 %), half of the next slice's A0
// fragments read in the otherwise read-free P4 (12/4/8/0 -> 8/4/8/4 reads per phase: +8 %),
// XCDs 4-7 started half a tile late to split the chip-wide store burst (no change).
constexpr int P8_SCR = 8 * 2048;
constexpr int P8_MAX_MP = (160 * 1024 - 8 * HALF_B - P8_SCR) / 4;
constexpr int P8_HEAD_MAX_OUT = P8_SCR / (4 * BM * 4);  // head partials [4 column waves][BM][n_out] fp32
constexpr int P8_HEAD_MAX_MP = (160 * 1024 - 8 * HALF_B - P8_SCR) / (4 + 2 * P8_HEAD_MAX_OUT);  // biases + whl

// NOSTORE (flag bit 13, timing only): the hidden epilogue writes nothing — the cost of the stores.
// (Non-temporal stores, which take 10 % off gemm_k64p_kernel, measured no change here: profiles/r5p.)
// DEFER (flag bit 15, measured slower, profiles/r5r: 2.17-2.22 vs 2.10-2.14 ms): a tile is stored
// in two halves. Accumulator rows 0-1 are read by the next tile's P1 / P2, rows 2-3 only from its
// P3 on — so rows 0-1 leave at the tile boundary and rows 2-3 after the next tile's P2, half of the
// stores overlapping two phases of MFMAs. P4 of a tile's first slice then retires slice g + 1 with
// the 8 deferred stores still in flight: everything younger than A1 of g + 1 is A0 of g + 2, the
// 8 stores, B0 / B1 of g + 2 = 14 instructions.
constexpr int P8_HALF_STORES = 8;  // global stores of store_hidden_seg rows [2, 4) per lane (all lanes)
// (Also measured and dropped, profiles/r5z: the last slice of a tile staging A1 of slice g + 2 in
// its P4 so that the next tile's first slice can retire g + 2 with the epilogue's stores still in
// flight — 2.09-2.14 vs 1.99-2.08 ms with the asm staging, as it was with the builtin one.)
template <bool HEADF, bool NOSTORE, bool DEFER = false>
__global__ __launch_bounds__(NT, 1) void gemm8p_kernel(GemmArgs a, HeadFuse hf) {
  constexpr bool DF = DEFER && !HEADF && !NOSTORE;
  constexpr int TM = 4, TN = 2;
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int n_ct = a.Mp / 256;
  const int total = (a.rows_p / BM) * n_ct;
  const int G = gridDim.x;
  int base, step, n_my;
  if ((total & 7) == 0 && (G & 7) == 0) {
    const int T8 = total >> 3, G8 = G >> 3, s = blockIdx.x >> 3;
    base = (blockIdx.x & 7) * T8 + s;
    step = G8;
    n_my = s < T8 ? (T8 - s + G8 - 1) / G8 : 0;
  } else {
    base = blockIdx.x;
    step = G;
    n_my = (int)blockIdx.x < total ? (total - (int)blockIdx.x + G - 1) / G : 0;
  }
  if (n_my <= 0) return;  // workgroup-uniform, before any barrier
  unsigned char* scr = smem + 8 * HALF_B;  // wave scratch (hidden) / head partials (HEADF)
  float* bl = reinterpret_cast<float*>(smem + 8 * HALF_B + P8_SCR);
  __bf16* whl = reinterpret_cast<__bf16*>(bl + a.Mp);  // HEADF: [n_out][Mp] output-layer weights
  for (int u = tid; u < a.Mp; u += NT) bl[u] = a.bias[u];
  if constexpr (HEADF)
    for (int e = tid; e < hf.n_out * a.Mp; e += NT) whl[e] = hf.wh[(size_t)(e / a.Mp) * hf.ldw + e % a.Mp];
  __syncthreads();

  const int wr = wave >> 2, wc = wave & 3;
  const size_t lda_b = (size_t)a.lda * 2, ldw_b = (size_t)a.ldw * 2;
  const uint32_t lda32 = (uint32_t)lda_b, ldw32 = (uint32_t)ldw_b;
  const unsigned char* A0p = static_cast<const unsigned char*>(a.A);
  const unsigned char* B0p = static_cast<const unsigned char*>(a.Wt);
  const int KT = a.K / BK;
  const int NS = n_my * KT;
  // the sources of slices g + 1 (s1) and g + 2 (s2): tile pointers + slice offset
  struct Src {
    const unsigned char* A;
    const unsigned char* B;
    int j, k;
  };
  auto at_tile = [&](int j, int k) -> Src {
    const int t = base + j * step;
    return Src{A0p + (size_t)((t / n_ct) * BM) * lda_b, B0p + (size_t)((t % n_ct) * 256) * ldw_b, j, k};
  };
  auto advance = [&](const Src& s) -> Src {
    return s.k + 1 < KT ? Src{s.A, s.B, s.j, s.k + 1} : (s.j + 1 < n_my ? at_tile(s.j + 1, 0) : Src{s.A, s.B, s.j + 1, 0});
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

#define SLOT(b, s) (smem + (b) * 4 * HALF_B + (s) * HALF_B)
  const Src s0 = at_tile(0, 0);
  Src s1 = advance(s0);
  Src s2 = advance(s1);
  stage_half_s<true>(s0.A, lda32, SLOT(0, 0), 0, wave, lane);
  stage_half_s<false>(s0.B, ldw32, SLOT(0, 2), 0, wave, lane);
  stage_half_s<false>(s0.B, ldw32, SLOT(0, 3), 1, wave, lane);
  stage_half_s<true>(s0.A, lda32, SLOT(0, 1), 1, wave, lane);
  if (NS > 1) {
    const size_t kb = (size_t)s1.k * SLICE_B;
    stage_half_s<true>(s1.A + kb, lda32, SLOT(1, 0), 0, wave, lane);
    stage_half_s<false>(s1.B + kb, ldw32, SLOT(1, 2), 0, wave, lane);
    stage_half_s<false>(s1.B + kb, ldw32, SLOT(1, 3), 1, wave, lane);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  if (wr == 1) raw_barrier();  // group 1 runs one barrier behind group 0

  const int ra = wr * 64 + l32, rb = wc * 32 + l32;
  int row0 = (base / n_ct) * BM, col0 = (base % n_ct) * 256;
  int prow0 = 0, pcol0 = 0;  // DF: the previous tile, whose rows 2-3 are still in acc[2], acc[3]
  for (int g = 0, kt = 0, j = 0; g < NS; ++g) {
    const int b = g & 1;
    const bool n1 = g + 1 < NS, n2 = g + 2 < NS;
    const bool first = DF && kt == 0 && g > 0;
    const size_t k1 = (size_t)s1.k * SLICE_B, k2 = (size_t)s2.k * SLICE_B;
    bf16x8 a0[2][4], a1[2][4], b0[4], b1[4];
    // P1: A0 x B0
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
      for (int i = 0; i < 2; ++i) a0[i][ks] = frag(SLOT(b, 0), ra + 32 * i, 2 * ks + h);
      b0[ks] = frag(SLOT(b, 2), rb, 2 * ks + h);
    }
    if (n1) stage_half_s<true>(s1.A + k1, lda32, SLOT(b ^ 1, 1), 1, wave, lane);
    mma_begin();
    mma_quad<true>(acc[0][0], acc[1][0], a0, b0);
    mma_end();
    // P2: A0 x B1
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) b1[ks] = frag(SLOT(b, 3), rb, 2 * ks + h);
    if (n2) stage_half_s<true>(s2.A + k2, lda32, SLOT(b, 0), 0, wave, lane);
    mma_begin();
    mma_quad<true>(acc[0][1], acc[1][1], a0, b1);
    mma_end();
    if constexpr (DF) {
      if (first) {  // the previous tile's rows 2-3, before this tile's P3 accumulates into them
        store_hidden_seg_any<TM, TN, true, false, 2, 4>(a, acc, prow0, pcol0, wr, wc, lane, bl + pcol0, scr + wave * 2048);
#pragma unroll
        for (int i = 2; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < TN; ++q) acc[i][q] = f32x16{};
        // B1 re-read rather than held through the epilogue (its slot is restaged only in P4)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) b1[ks] = frag(SLOT(b, 3), rb, 2 * ks + h);
      }
    }
    // P3: A1 x B1
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i) a1[i][ks] = frag(SLOT(b, 1), ra + 32 * i, 2 * ks + h);
    if (n2) stage_half_s<false>(s2.B + k2, ldw32, SLOT(b, 2), 0, wave, lane);
    mma_begin();
    mma_quad<true>(acc[2][1], acc[3][1], a1, b1);
    mma_end();
    // P4: A1 x B0; slice g + 1 retired (three half-tiles of g + 2 may stay in flight — and, on a
    // tile's first slice, the previous epilogue's stores, which are older, retired with it)
    if (n2) stage_half_s<false>(s2.B + k2, ldw32, SLOT(b, 3), 1, wave, lane);
    if (n2) {
      if (first) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + P8_HALF_STORES) : "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (n1) {
      if (first) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P8_HALF_STORES) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mma_begin();
    mma_quad<true>(acc[2][0], acc[3][0], a1, b0);
    mma_end();
    s1 = s2;
    s2 = advance(s2);
    if (++kt == KT) {  // tile j done: epilogue between two phases, the next tile's slices in flight
      if constexpr (HEADF) {
        if (wr == 0) raw_barrier();  // align the groups for head_partial's barrier
        switch (a.act) {
          case A_IDENTITY: head_partial<A_IDENTITY, true>(a, hf, acc, row0, col0, wr, wc, lane, tid, scr, bl + col0, whl); break;
          case A_RELU: head_partial<A_RELU, true>(a, hf, acc, row0, col0, wr, wc, lane, tid, scr, bl + col0, whl); break;
          case A_LOGISTIC: head_partial<A_LOGISTIC, true>(a, hf, acc, row0, col0, wr, wc, lane, tid, scr, bl + col0, whl); break;
          case A_TANH: head_partial<A_TANH, true>(a, hf, acc, row0, col0, wr, wc, lane, tid, scr, bl + col0, whl); break;
          default: head_partial<-1, true>(a, hf, acc, row0, col0, wr, wc, lane, tid, scr, bl + col0, whl); break;
        }
        if (wr == 1) raw_barrier();  // group 1 one barrier behind again
      } else if constexpr (NOSTORE) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(acc[i][0]), "v"(acc[i][1]));
      } else if constexpr (DF) {
        store_hidden_seg_any<TM, TN, true, false, 0, 2>(a, acc, row0, col0, wr, wc, lane, bl + col0, scr + wave * 2048);
        prow0 = row0;
        pcol0 = col0;
      } else {
        store_hidden_seg_any<TM, TN, true>(a, acc, row0, col0, wr, wc, lane, bl + col0, scr + wave * 2048);
      }
#pragma unroll
      for (int i = 0; i < (DF ? 2 : TM); ++i)
#pragma unroll
        for (int q = 0; q < TN; ++q) acc[i][q] = f32x16{};
      kt = 0;
      if (++j < n_my) {
        const int t = base + j * step;
        row0 = (t / n_ct) * BM;
        col0 = (t % n_ct) * 256;
      }
    }
  }
#undef SLOT
  if constexpr (DF)  // the last tile's rows 2-3
    store_hidden_seg_any<TM, TN, true, false, 2, 4>(a, acc, prow0, pcol0, wr, wc, lane, bl + pcol0, scr + wave * 2048);
  if (wr == 0) raw_barrier();  // balance group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Persistent K = 64 hidden layer (bf16, the input stage separate): a workgroup owns one 256-unit
// column tile — its weight slice (32 KiB) and biases staged in LDS ONCE — and walks row tiles of
// 128 rows, the next tile's A slice (16 KiB, LDS-DMA) in flight while the current one multiplies
// and leaves through the transposed-accumulator stores (store_hidden_t). The wait for a tile's A is
// a COUNTED vmcnt: the only younger vector-memory operations are the previous tile's 16 stores
// (loads, stores and LDS-DMA retire in issue order), so the stores drain behind the next tile's
// work instead of at a workgroup exit. Workgroups are laid out XCD-major: blockIdx & 7 is the XCD,
// and the n_ct column-tile owners of a row group share it, so a row tile's A is fetched from HBM
// once and hit in that XCD's L2 by the other column tiles. Two workgroups per CU (65 KiB of LDS each).
constexpr int K64P_STORES = 16;  // store_hidden_t<2, 4>: 2 x 4 tiles x 2 stores per lane
template <bool SEG, bool NTS = false>
__global__ __launch_bounds__(K64_NT, 2) void gemm_k64p_kernel(GemmArgs a, int rg) {
  constexpr int TM = 2, TN = 4;
  constexpr int A_B = K64_BM * SLICE_B;
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned char* Bs = smem;                          // 256 units x 128 B
  unsigned char* As = smem + 256 * SLICE_B;          // two 128-row A buffers
  float* bl = reinterpret_cast<float*>(As + 2 * A_B);  // 256 biases
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned char* ws = reinterpret_cast<unsigned char*>(bl + 256) + wave * 2048;  // SEG: wave scratch
  const int h = lane >> 5, l32 = lane & 31;
  const int n_ct = a.Mp / 256, n_rt = a.rows_p / K64_BM;
  const int local = blockIdx.x >> 3;
  const int ct = local % n_ct;
  const int g = (local / n_ct) * 8 + (blockIdx.x & 7);  // row group: XCD-major
  const int stride = 8 * rg;
  if (g >= n_rt) return;
  const int col0 = ct * 256;
  const int wm = wave >> 1, wn = wave & 1;
  const size_t lda_b = (size_t)a.lda * 2, ldw_b = (size_t)a.ldw * 2;
  const unsigned char* A = static_cast<const unsigned char*>(a.A);
  stage_slice<256, 4>(static_cast<const unsigned char*>(a.Wt) + (size_t)col0 * ldw_b, ldw_b, 0, Bs, wave, lane);
  stage_slice<K64_BM, 4>(A + (size_t)g * K64_BM * lda_b, lda_b, 0, As, wave, lane);
  bl[tid] = a.bias[col0 + tid];  // K64_NT == 256
  int it = 0;
  for (int rt = g; rt < n_rt; rt += stride, ++it) {
    const unsigned char* Ac = As + (it & 1) * A_B;
    if (it == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K64P_STORES) : "memory");
    raw_barrier();  // every wave's part of A(rt) landed; every wave's reads of the other buffer done
    if (rt + stride < n_rt)
      stage_slice<K64_BM, 4>(A + (size_t)(rt + stride) * K64_BM * lda_b, lda_b, 0, As + ((it + 1) & 1) * A_B, wave,
                             lane);
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag(Ac, (wm * TM + i) * 32 + l32, 2 * ks + h);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = frag(Bs, (wn * TN + j) * 32 + l32, 2 * ks + h);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if constexpr (SEG) store_hidden_seg_any<TM, TN, true, NTS>(a, acc, rt * K64_BM, col0, wm, wn, lane, bl, ws);
    else store_hidden_t_any<TM, TN, true>(a, acc, rt * K64_BM, col0, wm, wn, lane, bl);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int cu_count() {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
  }
  return n_cu;
}

int launch_k64p(hipStream_t stream, const GemmArgs& a) {
  const int n_cu = cu_count();
  const int n_ct = a.Mp / 256;
  const int rg = std::max(1, (2 * n_cu / 8) / n_ct);  // row groups per XCD: ~2 workgroups per CU
  // 128-byte row-segment stores through a 2 KiB wave scratch (store_hidden_seg, default: 0.565 ->
  // 0.438 ms for 1M rows x 1024 units, TA busy 78 -> 52 %, profiles/r5f); bit 10: store_hidden_t
  const bool seg = !((a.f32 >> 10) & 1);
  const size_t lds = (size_t)(256 + 2 * K64_BM) * SLICE_B + 256 * 4 + (seg ? 4 * 2048 : 0);
  // non-temporal row-segment stores (the layer streams 2 GB of output per 1M rows and reads
  // little): 0.435 -> 0.391 ms, profiles/r5p; bit 14: ordinary stores
  const bool nts = seg && !((a.f32 >> 14) & 1);
  const void* kp = nts ? reinterpret_cast<const void*>(&gemm_k64p_kernel<true, true>)
                 : seg ? reinterpret_cast<const void*>(&gemm_k64p_kernel<true>)
                       : reinterpret_cast<const void*>(&gemm_k64p_kernel<false>);
  if (hipFuncSetAttribute(kp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -5;
  if (nts)
    hipLaunchKernelGGL((gemm_k64p_kernel<true, true>), dim3(8 * n_ct * rg), dim3(K64_NT), lds, stream, a, rg);
  else if (seg)
    hipLaunchKernelGGL(gemm_k64p_kernel<true>, dim3(8 * n_ct * rg), dim3(K64_NT), lds, stream, a, rg);
  else
    hipLaunchKernelGGL(gemm_k64p_kernel<false>, dim3(8 * n_ct * rg), dim3(K64_NT), lds, stream, a, rg);
  return 0;
}

template <bool HEADF, bool TST = false>
int launch8(hipStream_t stream, const GemmArgs& a, const HeadFuse& hf) {
  const size_t lds = 8 * (size_t)HALF_B;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm8_kernel<HEADF, TST>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -5;
  hipLaunchKernelGGL((gemm8_kernel<HEADF, TST>), dim3((a.rows_p / BM) * (a.Mp / 256)), dim3(NT), lds, stream, a, hf);
  return 0;
}

template <bool HEADF>
int launch8p(hipStream_t stream, const GemmArgs& a, const HeadFuse& hf) {
  const size_t lds = 8 * (size_t)HALF_B + P8_SCR + 4 * (size_t)a.Mp + (HEADF ? 2 * (size_t)hf.n_out * a.Mp : 0);
  const bool nostore = !HEADF && ((a.f32 >> 13) & 1), defer = !HEADF && !nostore && ((a.f32 >> 15) & 1);
  const void* kp = HEADF ? reinterpret_cast<const void*>(&gemm8p_kernel<true, false>)
                 : nostore ? reinterpret_cast<const void*>(&gemm8p_kernel<false, true>)
                 : defer ? reinterpret_cast<const void*>(&gemm8p_kernel<false, false, true>)
                         : reinterpret_cast<const void*>(&gemm8p_kernel<false, false>);
  if (hipFuncSetAttribute(kp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -5;
  const int total = (a.rows_p / BM) * (a.Mp / 256);
  const int grid = std::min(total, cu_count());
  if (HEADF) hipLaunchKernelGGL((gemm8p_kernel<true, false>), dim3(grid), dim3(NT), lds, stream, a, hf);
  else if (nostore) hipLaunchKernelGGL((gemm8p_kernel<false, true>), dim3(grid), dim3(NT), lds, stream, a, hf);
  else if (defer) hipLaunchKernelGGL((gemm8p_kernel<false, false, true>), dim3(grid), dim3(NT), lds, stream, a, hf);
  else hipLaunchKernelGGL((gemm8p_kernel<false, false>), dim3(grid), dim3(NT), lds, stream, a, hf);
  return 0;
}

// whether the persistent kernel takes a layer (a: the hidden layer's args; flag bit 12 opts out)
bool use8p(const GemmArgs& a) {
  return !((a.f32 >> 12) & 1) && a.Mp <= P8_MAX_MP && (size_t)a.lda * 2 * BM < (1ull << 31) &&
         (size_t)a.ldw * 2 * 256 < (1ull << 31);
}

// The fused output layer's second half: one thread per row sums the column tiles' partials in
// order, + bias, output activation, decode.
__global__ __launch_bounds__(256) void nn_head_decode_kernel(GemmArgs a, const float* __restrict__ part, int n_ct) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= a.rows) return;
  float z[32];
  for (int o = 0; o < a.n_out; ++o) {
    float s = 0.f;
    for (int c = 0; c < n_ct; ++c) s += part[((size_t)c * a.rows_p + row) * a.n_out + o];
    z[o] = activate(a.act, s + a.bias[o], a.thr);
  }
  decode_row(a, row, z);
}

template <int BN, bool HEAD, bool F32, bool TST = false>
int launch(hipStream_t stream, const GemmArgs& a) {
  const size_t stage = 2 * (size_t)BM * SLICE_B + 2 * (size_t)BN * SLICE_B;
  const size_t head = HEAD ? (size_t)BM * HEAD_LD * 4 : 0;
  const size_t lds = stage > head ? stage : head;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<BN, HEAD, F32, TST>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -5;
  dim3 grid((a.rows_p / BM) * (a.Mp / BN));
  hipLaunchKernelGGL((gemm_kernel<BN, HEAD, F32, TST>), grid, dim3(NT), lds, stream, a);
  return 0;
}

}  // namespace

PMML_API int pmml_gemm_args_size() { return (int)sizeof(GemmArgs); }
PMML_API int pmml_nn_prep_args_size() { return (int)sizeof(PrepArgs); }

PMML_API int pmml_nn_prep_launch(hipStream_t stream, const PrepArgs* args) {
  PrepArgs a = *args;
  if (a.rows_p <= 0) return 0;
  if ((a.k0 & 7) || a.k0 < a.n_in || a.k0 > NN_MAX_INPUTS || (a.ldh & 7) || (reinterpret_cast<uintptr_t>(a.H) & 15))
    return -4;
  if (a.f32 != 0 && a.f32 != 1) return -4;
  // the vector path needs every row's first input 16-byte aligned
  if (a.contig && ((reinterpret_cast<uintptr_t>(a.X) & 15) || (a.ldx & 3))) a.contig = 0;
  int g = 0;
  while ((1 << g) < (a.k0 >> 3) && g < 6) ++g;  // lanes per row: chunks rounded up to a power of two, <= 64
  const long long threads = (long long)a.rows_p << g;
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (a.f32) hipLaunchKernelGGL(nn_prep_kernel<true>, grid, dim3(256), 0, stream, a, g);
  else hipLaunchKernelGGL(nn_prep_kernel<false>, grid, dim3(256), 0, stream, a, g);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

// head = 0: hidden layer (BN 256, output C in the operand type); head = 1: output layer (BN 32,
// n_out <= 32, decode). args->f32 selects bf16 (0) or fp32 (1) operands.
PMML_API int pmml_gemm_launch(hipStream_t stream, const GemmArgs* args, int head) {
  const GemmArgs a = *args;
  if (a.rows <= 0) return 0;
  const int BN = head ? 32 : 256;
  if (a.f32 & ~0x1FFE1) return -4;
  // bf16 hidden layers with K >= 512 run the phase-interleaved kernel (profiles/r3ao: 2048 x 2048
  // 8.73 -> 8.36 ms, 1024 x 1024 2.62 -> 2.48 ms over 1M rows); below that the layer is bound by
  // its output writes and the 2-buffer loop is faster (K = 64: 0.83 vs 0.92 ms). Bit 7 forces it.
  const int f32 = a.f32 & 1, ph8 = !f32 && (((a.f32 >> 7) & 1) || a.K >= 512);
  const int sk = f32 ? SLICE_B / 4 : SLICE_B / 2;
  if (a.rows_p % BM || a.rows_p < a.rows || a.K % sk || a.K <= 0 || a.Mp % BN || a.Mp <= 0) return -4;
  if ((a.lda & 7) || (a.ldw & 7) || a.lda < a.K || a.ldw < a.K) return -4;
  if ((reinterpret_cast<uintptr_t>(a.A) & 15) || (reinterpret_cast<uintptr_t>(a.Wt) & 15)) return -4;
  if (head && (a.n_out < 1 || a.n_out > 32 || a.Mp != 32 || (!a.C && (!a.row_ok || !a.score || !a.valid)))) return -4;
  if (head && a.C && (a.ldc < a.n_out || (reinterpret_cast<uintptr_t>(a.C) & 3))) return -4;
  if (!head && ((a.ldc & 7) || a.ldc < a.Mp || !a.C || (reinterpret_cast<uintptr_t>(a.C) & 15))) return -4;
  // transposed-accumulator stores (store_hidden_t) unless bit 8 or the bit-5 LDS epilogue asks otherwise
  const bool tst = !((a.f32 >> 8) & 1) && !((a.f32 >> 5) & 1);
  if (!head && !f32 && a.K == 64 && !((a.f32 >> 6) & 1)) {  // bit 6 forces the 256 x 256 tile
    const dim3 grid((a.rows_p / K64_BM) * (a.Mp / 256));
    const size_t lds = (size_t)(K64_BM + 256) * SLICE_B;
    if (tst && !((a.f32 >> 9) & 1)) {  // bit 9: the one-tile-per-workgroup kernel
      const int rc = launch_k64p(stream, a);
      if (rc) return rc;
    } else if (tst) {
      hipLaunchKernelGGL((gemm_k64_kernel<false, true>), grid, dim3(K64_NT), lds, stream, a, PrepArgs{});
    } else {
      hipLaunchKernelGGL((gemm_k64_kernel<false, false>), grid, dim3(K64_NT), lds, stream, a, PrepArgs{});
    }
    return hipGetLastError() == hipSuccess ? 0 : -7;
  }
  // persistent tile walk (gemm8p_kernel) for the transposed-store phase-interleaved layers with the
  // row-segment stores and K <= 1024, unless bit 12 (one tile per workgroup) or bit 11
  // (store_hidden_t) is set
  // bf16 hidden layers with K >= 128 (bit 7: also K = 64) on the transposed-store path run the
  // persistent kernel (profiles/r5t: K = 256 layers 0.25 / 0.47 vs 0.32 / 0.60 ms on the 2-buffer
  // loop, K = 4096 6.92 vs 7.42 ms on gemm8_kernel)
  const bool p8 = !f32 && tst && !head && !((a.f32 >> 11) & 1) && (a.K >= 128 || ((a.f32 >> 7) & 1)) &&
                  (use8p(a) || ((a.f32 >> 13) & 1) || ((a.f32 >> 16) & 1));
  const int rc = f32 ? (head ? launch<32, true, true>(stream, a) : launch<256, false, true>(stream, a))
                     : (head ? launch<32, true, false>(stream, a)
                             : (p8 ? launch8p<false>(stream, a, HeadFuse{})
                                   : ph8 ? (tst ? launch8<false, true>(stream, a, HeadFuse{}) : launch8<false, false>(stream, a, HeadFuse{}))
                                   : (tst ? launch<256, false, false, true>(stream, a) : launch<256, false, false>(stream, a))));
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

// The last hidden layer and the output layer in one GEMM launch + one decode launch
// (gemm8_kernel<true>): the hidden activations never reach HBM. hidden: a bf16 hidden layer (K a
// multiple of 64, Mp of 256); head: the output layer's args (Wt unused: wh_perm holds its weights
// [32][hidden.Mp], k permuted by fuse_head_perm); part: (hidden.Mp / 256) * rows_p * n_out floats.
PMML_API int pmml_gemm_fused_head_launch(hipStream_t stream, const GemmArgs* hidden, const GemmArgs* head,
                                         const void* wh_perm, float* part) {
  const GemmArgs a = *hidden;
  const GemmArgs o = *head;
  if (a.rows <= 0) return 0;
  if ((a.f32 & 1) || (o.f32 & 1)) return -4;  // bf16 only (bit 7, the gemm8 force flag, is moot here)
  if (a.rows_p % BM || a.rows_p < a.rows || a.K % BK || a.K <= 0 || a.Mp % 256 || a.Mp <= 0) return -4;
  if ((a.lda & 7) || (a.ldw & 7) || a.lda < a.K || a.ldw < a.K) return -4;
  if ((reinterpret_cast<uintptr_t>(a.A) & 15) || (reinterpret_cast<uintptr_t>(a.Wt) & 15)) return -4;
  if (o.n_out < 1 || o.n_out > 32 || o.K != a.Mp || o.rows != a.rows || o.rows_p != a.rows_p) return -4;
  if (!o.row_ok || !o.score || !o.valid || !part || !wh_perm || (reinterpret_cast<uintptr_t>(wh_perm) & 15)) return -4;
  HeadFuse hf{static_cast<const __bf16*>(wh_perm), part, a.Mp, o.n_out};
  const bool p8 = use8p(a) && o.n_out <= P8_HEAD_MAX_OUT && a.Mp <= P8_HEAD_MAX_MP;
  int rc = p8 ? launch8p<true>(stream, a, hf) : launch8<true, false>(stream, a, hf);
  if (rc) return rc;
  hipLaunchKernelGGL(nn_head_decode_kernel, dim3((a.rows + 255) / 256), dim3(256), 0, stream, o, part, a.Mp / 256);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

// Input stage + first hidden layer in one launch (gemm_k64_kernel<true>): bf16, K = k0 = 64 (at
// most 64 network inputs), hidden-layer output C; p->row_ok receives the row validity as
// pmml_nn_prep_launch would (p->H is not written).
PMML_API int pmml_nn_first_layer_launch(hipStream_t stream, const GemmArgs* args, const PrepArgs* prep) {
  const GemmArgs a = *args;
  const PrepArgs p = *prep;
  if (a.rows <= 0) return 0;
  if ((a.f32 & 1) || p.f32 != 0 || a.K != 64 || p.k0 != 64 || p.n_in > 64 || p.n_in < 0) return -4;
  if (a.rows_p % 256 || a.rows_p < a.rows || p.rows_p != a.rows_p || p.n_rows != a.rows) return -4;
  if (a.Mp % 256 || a.Mp <= 0 || (a.ldw & 7) || a.ldw < a.K || (reinterpret_cast<uintptr_t>(a.Wt) & 15)) return -4;
  if ((a.ldc & 7) || a.ldc < a.Mp || !a.C || (reinterpret_cast<uintptr_t>(a.C) & 15) || !p.row_ok || !p.X) return -4;
  const dim3 grid((a.rows_p / K64_BM) * (a.Mp / 256));
  const size_t lds = (size_t)(K64_BM + 256) * SLICE_B;
  if (!((a.f32 >> 8) & 1) && !((a.f32 >> 5) & 1))
    hipLaunchKernelGGL((gemm_k64_kernel<true, true>), grid, dim3(K64_NT), lds, stream, a, p);
  else
    hipLaunchKernelGGL((gemm_k64_kernel<true, false>), grid, dim3(K64_NT), lds, stream, a, p);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

// Decode of a wide output layer (n_out > 32) from its activated outputs Z [rows][ldz] fp32.
PMML_API int pmml_nn_decode_wide(hipStream_t stream, const GemmArgs* args, const float* Z, int ldz) {
  const GemmArgs a = *args;
  if (a.rows <= 0) return 0;
  if (a.n_out < 1 || ldz < a.n_out || !Z || !a.row_ok || !a.score || !a.valid) return -4;
  hipLaunchKernelGGL(nn_decode_wide_kernel, dim3((a.rows + 255) / 256), dim3(256), 0, stream, a, Z, ldz);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
