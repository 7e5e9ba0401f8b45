// NeuralNetwork (MLP) scoring on the matrix cores: all layers fused in one persistent kernel.
//
// Orientation (unchanged from the first version): data rows on the MFMA N dimension (lanes),
// neurons on M (registers): each layer computes Zᵀ[units, 32 rows] = Wᵀ[units, K] · Hᵀ[K, 32 rows].
// The 32x32 accumulator of one output tile (units on registers, rows on lanes) is directly the B
// operand of the next layer's MFMA (cdna_hip_programming.md §3, "An accumulator tile as the next
// MFMA's operand"), so activations never leave the register file between layers.
//
// What changed (round 2): the weights (A operands) are no longer fetched from L2 by every wave
// for every MFMA. They stream through an LDS ring of PANELS — one panel = all k-step fragments of
// one 32-unit output tile of one layer, pre-permuted on the host into exactly the k order the
// registers provide. One 512-thread workgroup (8 waves x 32 rows = 256 rows) shares every panel,
// so each weight byte read from L2 serves 256 rows (was 32), and the A-fragment read is a
// conflict-free ds_read_b128 per MFMA with LDS latency instead of L2 latency. The panel for
// step p+2 is loaded into registers while step p computes and stored after it (one barrier per
// panel). Each output tile is ONE accumulation chain (16 MFMAs back to back on one accumulator,
// which the 32x32x16 pipe sustains at full rate), so only 16 accumulator registers are live and
// the activations of the current and the next layer fit in 2 x 64 VGPRs (bf16) — two waves per
// SIMD. The grid is persistent (one workgroup per CU walks row tiles), so the panel pipeline
// runs across tile boundaries without draining.
//
// Two precisions (one template):
//   BF16 = true : v_mfma_f32_32x32x16_bf16 (bf16 in, fp32 accumulate) — the throughput path;
//   BF16 = false: v_mfma_f32_32x32x2_f32  (exact fp32 FMA chain)     — the parity path (default).
// Input normalisation (NormContinuous as scale/shift), missing handling, activations, output-layer
// normalisation (softmax / simplemax) and the target decode are fused.
#include "epilogue.h"
#include "nn_act.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MT = 8;          // max 32-unit output tiles per layer -> 256 units per layer
constexpr int MAXL = 8;        // max layers (biases staged in LDS)
constexpr int KMAX = 256;      // max inputs per layer
constexpr int NSLOT = 4;       // LDS panel ring slots


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
  const int2* panels;       // [n_panels] {offset, size} in 16-byte units, consumption order
  int n_panels, contiguous; // contiguous: in_index[k] == k (vector input loads)
  unsigned long long* prof; // optional phase timers of workgroup 0 / wave 0 (s_memtime ticks):
                            // [stage, chain, barrier, epilogue, tiles, steps]
  int reg_kernel;           // bf16: 1 = register-weight kernel (host checked the shape), 0 = panel kernel
  int pad_;
};


// row (unit) index inside a 32x32 accumulator tile held by register r of lane half h
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <bool BF16> struct Cfg;
template <> struct Cfg<true> {
  static constexpr int WAVES = 8, KS = KMAX / 16, Q = 2;   // Q: uint4 per thread per 16 KiB panel
  static constexpr int PANEL = 16 * 1024;
  typedef bf16x8 B;
};
template <> struct Cfg<false> {
  static constexpr int WAVES = 4, KS = KMAX / 2, Q = 8;    // 32 KiB panels (128 k-steps x 256 B)
  static constexpr int PANEL = 32 * 1024;
  typedef float B;
};

// Input normalisation tables in LDS are padded to KMAX with neutral entries (index 0, scale 0,
// shift 0, replacement 0): padded k read column 0 and contribute exactly 0. `contiguous` (identity
// index) is only set by the host when n_in == k0, so no record load leaves the row.

// Panel p -> LDS ring slot p % NSLOT with direct global->LDS loads (global_load_lds_dwordx4, no
// VGPR staging): thread t copies 16-byte elements t, t+T, ... The LDS destination of one
// wave-instruction is its wave-uniform base + 16*lane, i.e. elements [64w + jT, 64w + jT + 63]
// land contiguously, exactly the panel image. Elements past the panel's size re-read its last
// element into the slot's unused tail (the slot holds a full PANEL).
//
// Issued as inline asm rather than __builtin_amdgcn_global_load_lds: the compiler treats the
// builtin as an LDS write that may alias every later ds_read and drains it (vmcnt(0)) before the
// chain's first A-fragment read, which serialises the copy with the MFMAs it should overlap.
// Here the kernel owns the ordering: panel_barrier() retires a panel before any wave reads it,
// and a slot is rewritten only two steps after its last read (NSLOT = 4). The compiler's own
// vmcnt waits stay correct: loads retire in order, so an unseen younger load only makes them
// wait longer.
__device__ __forceinline__ void glds16(const void* g, uint32_t lds_byte_addr) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_byte_addr) : "memory");
}

template <bool BF16>
__device__ __forceinline__ void issue_panel(const MlpArgs& a, const int2* s_pan, int p, int tid, uint4* ring) {
  constexpr int T = 64 * Cfg<BF16>::WAVES;
  const uint4* W4 = reinterpret_cast<const uint4*>(a.weights);
  const int2 d = s_pan[p % a.n_panels];
  const int last = d.y > 0 ? d.y - 1 : 0;
  // LDS byte address of this wave's destination: the dynamic LDS (ring = its start) begins right
  // after the kernel's static LDS
  const uint32_t off = 16u * (uint32_t)((p % NSLOT) * (Cfg<BF16>::PANEL / 16) + (tid & ~63));
  const uint32_t base = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_groupstaticsize() + off);
  (void)ring;
#pragma unroll
  for (int i = 0; i < Cfg<BF16>::Q; ++i) glds16(W4 + d.x + min(tid + i * T, last), base + 16u * i * T);
}

// Retire this thread's loads of the panel issued one step earlier (the one just issued may stay
// in flight: Q glds per panel), then a raw barrier: every thread's share has landed. A raw
// s_barrier, not __syncthreads(), whose fence would also drain the panel still in flight.
template <bool BF16>
__device__ __forceinline__ void panel_barrier() {
  if constexpr (Cfg<BF16>::Q == 2) {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
}

// The accumulation chain of one output tile over STEPS k-steps, fully unrolled with no per-step
// predicate: the A fragments come from the LDS panel (the compiler can issue the ds_reads ahead
// of the MFMAs), B from registers (compile-time indices keep them in VGPRs).
template <bool BF16, int STEPS>
__device__ __forceinline__ void mfma_chain(const uint4* slot, int lane, const typename Cfg<BF16>::B (&pb)[Cfg<BF16>::KS],
                                           f32x16& acc) {
  // A fragments run W steps ahead of the MFMA that consumes them (a rolling register window), so
  // the LDS latency of step s+W overlaps the MFMAs of steps s..s+W-1 instead of stalling each one
  constexpr int W = STEPS < (BF16 ? 4 : 8) ? STEPS : (BF16 ? 4 : 8);
  if constexpr (BF16) {
    uint4 win[W];
#pragma unroll
    for (int i = 0; i < W; ++i) win[i] = slot[i * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);  // keep the window: the scheduler would sink each read to its use
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const uint4 w = win[s % W];
      if (s + W < STEPS) win[s % W] = slot[(s + W) * 64 + lane];
      bf16x8 A;
      __builtin_memcpy(&A, &w, 16);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, pb[s], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    const float* fs = reinterpret_cast<const float*>(slot);
    float win[W];
#pragma unroll
    for (int i = 0; i < W; ++i) win[i] = fs[i * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const float A = win[s % W];
      if (s + W < STEPS) win[s % W] = fs[(s + W) * 64 + lane];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A, pb[s], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// k-step groups: bf16 one k-step (K = 16) per group, fp32 eight (K = 16); the host pads every
// layer's K to a multiple of 16, so a layer has 1..16 groups and each count is its own chain.
template <bool BF16>
__device__ __forceinline__ void mfma_chain_n(int groups, const uint4* slot, int lane,
                                             const typename Cfg<BF16>::B (&pb)[Cfg<BF16>::KS], f32x16& acc) {
  constexpr int G = BF16 ? 1 : 8;
  switch (groups) {
#define PMML_CHAIN(N) \
    case N: mfma_chain<BF16, N * G>(slot, lane, pb, acc); break;
    PMML_CHAIN(1) PMML_CHAIN(2) PMML_CHAIN(3) PMML_CHAIN(4) PMML_CHAIN(5) PMML_CHAIN(6) PMML_CHAIN(7)
    PMML_CHAIN(8) PMML_CHAIN(9) PMML_CHAIN(10) PMML_CHAIN(11) PMML_CHAIN(12) PMML_CHAIN(13) PMML_CHAIN(14)
    PMML_CHAIN(15) PMML_CHAIN(16)
#undef PMML_CHAIN
    default: break;
  }
}

// Write the activated accumulator of output tile TI into the next layer's B registers. TI is a
// compile-time index so nb stays in VGPRs; this is the only per-tile code copy (the MFMA chain is
// shared by all tiles, keeping the hot loop small enough for the instruction cache).
template <bool BF16, int TI>
__device__ __forceinline__ void store_nb(const f32x16& acc, typename Cfg<BF16>::B (&nb)[Cfg<BF16>::KS]) {
  if constexpr (BF16) {
    bf16x8 lo, hi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lo[j] = (__bf16)acc[j];
      hi[j] = (__bf16)acc[8 + j];
    }
    nb[2 * TI] = lo;
    nb[2 * TI + 1] = hi;
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) nb[16 * TI + r] = acc[r];
  }
}

// One 32-unit output tile ti of one layer: a single accumulation chain over the layer's k-steps
// (A from the LDS panel, B from registers), activation, and the result written into the next
// layer's B-operand registers.
template <bool BF16>
__device__ __forceinline__ void tile_step(const MlpArgs& a, const LayerMeta& m, int ti, int groups, bool last,
                                          int h, int lane, int tid, const float* s_b, const int2* s_pan,
                                          uint4* ring, const typename Cfg<BF16>::B (&pb)[Cfg<BF16>::KS],
                                          typename Cfg<BF16>::B (&nb)[Cfg<BF16>::KS], f32x16& out, int& p,
                                          bool prof_on, unsigned long long* prof_acc) {
  using C = Cfg<BF16>;
  // panel p+2 streams into slot (p+2) % NSLOT while this one is multiplied; that slot was last
  // read at step p-2, before the previous barrier
  const unsigned long long t0 = prof_on ? __builtin_amdgcn_s_memtime() : 0ull;
  issue_panel<BF16>(a, s_pan, p + 2, tid, ring);
  const uint4* slot = ring + (p % NSLOT) * (C::PANEL / 16);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = s_b[m.b_off + 32 * ti + acc_row(r, h)];
  mfma_chain_n<BF16>(groups, slot, lane, pb, acc);
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = activate(m.act, acc[r], m.thr);
  if (last) {
    if (ti == 0) out = acc;
  } else {
    switch (ti) {
      case 0: store_nb<BF16, 0>(acc, nb); break;
      case 1: store_nb<BF16, 1>(acc, nb); break;
      case 2: store_nb<BF16, 2>(acc, nb); break;
      case 3: store_nb<BF16, 3>(acc, nb); break;
      case 4: store_nb<BF16, 4>(acc, nb); break;
      case 5: store_nb<BF16, 5>(acc, nb); break;
      case 6: store_nb<BF16, 6>(acc, nb); break;
      default: store_nb<BF16, 7>(acc, nb); break;
    }
  }
  const unsigned long long t1 = prof_on ? __builtin_amdgcn_s_memtime() : 0ull;
  panel_barrier<BF16>();  // panel p+1 resident for the next step
  if (prof_on && lane == 0) {
    prof_acc[1] += t1 - t0;
    prof_acc[2] += __builtin_amdgcn_s_memtime() - t1;
    prof_acc[5] += 1;
  }
  ++p;
}

template <bool BF16>
__global__ __launch_bounds__(64 * Cfg<BF16>::WAVES, 1) void mlp_kernel(MlpArgs a) {
  using C = Cfg<BF16>;
  typedef typename C::B BT;
  constexpr int T = 64 * C::WAVES;
  constexpr int KS = C::KS;
  extern __shared__ __align__(16) uint4 smem4[];
  uint4* ring = smem4;                                             // [NSLOT][PANEL/16]
  float* s_sc = reinterpret_cast<float*>(ring + NSLOT * (C::PANEL / 16));
  float* s_sh = s_sc + KMAX;
  float* s_ms = s_sh + KMAX;
  int* s_ix = reinterpret_cast<int*>(s_ms + KMAX);
  float* s_b = reinterpret_cast<float*>(s_ix + KMAX);              // [MAXL * MT * 32]
  int2* s_pan = reinterpret_cast<int2*>(s_b + MAXL * MT * 32);      // [MAXL * MT] panel schedule
  int* s_rowbad = reinterpret_cast<int*>(s_pan + MAXL * MT);          // [WAVES * 32][2] NaN-operand counts

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int h = lane >> 5;
  const int col = lane & 31;

  // ---- once per workgroup: preparation tables + biases into LDS
  for (int k = tid; k < KMAX; k += T) {
    const bool u = k < a.n_in;
    s_sc[k] = u ? a.in_scale[k] : 0.f;
    s_sh[k] = u ? a.in_shift[k] : 0.f;
    s_ms[k] = u ? a.in_missing[k] : 0.f;
    s_ix[k] = u ? a.in_index[k] : 0;
  }
  int nbias = 0;
  for (int L = 0; L < a.n_layers; ++L) nbias = max(nbias, a.layers[L].b_off + a.layers[L].mp);
  for (int i = tid; i < nbias; i += T) s_b[i] = a.biases[i];
  for (int i = tid; i < a.n_panels; i += T) s_pan[i] = a.panels[i];
  __syncthreads();

  // ---- panel ring prologue: panels 0 and 1 (panel 1 may stay in flight into step 0)
  issue_panel<BF16>(a, s_pan, 0, tid, ring);
  issue_panel<BF16>(a, s_pan, 1, tid, ring);
  panel_barrier<BF16>();

  const int n_tiles = (a.n_rows + 32 * C::WAVES - 1) / (32 * C::WAVES);
  int p = 0;  // panel counter (runs across row tiles)
  const bool prof_on = a.prof != nullptr && blockIdx.x == 0 && wave == 0;
  unsigned long long* prof_acc = reinterpret_cast<unsigned long long*>(s_rowbad + C::WAVES * 64);  // [6] in LDS
  if (prof_on && lane == 0) {
    for (int i = 0; i < 6; ++i) prof_acc[i] = 0ull;
  }
  for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const unsigned long long ts0 = prof_on ? __builtin_amdgcn_s_memtime() : 0ull;
    const int row = (tile * C::WAVES + wave) * 32 + col;
    const bool in_range = row < a.n_rows;
    const float* xrow = a.X + (size_t)(in_range ? row : 0) * a.ldx;

    // ---- layer-0 B operands straight from the record (normalised), into pb. The lane's table
    // offset goes through an opaque register each tile, so the per-k LDS addresses stay
    // base + immediate (hoisting them out of the tile loop would cost hundreds of VGPRs).
    BT pb[KS], nb[KS];
    int nbad = 0;
    {
      uint32_t kb = BF16 ? 8u * h : (uint32_t)h;  // first k of this lane half
      __asm__ volatile("" : "+v"(kb));
      const float* tsc = s_sc + kb;
      const float* tsh = s_sh + kb;
      const float* tms = s_ms + kb;
      const int* tix = s_ix + kb;
      const float* xr = xrow + (a.contiguous ? kb : 0u);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if constexpr (BF16) {
          if (16 * s < a.k0) {
            bf16x8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int o = 16 * s + j;
              const float x = a.contiguous ? xr[o] : xrow[tix[o]];
              const float y = (x != x) ? tms[o] : fmaf(x, tsc[o], tsh[o]);
              nbad += (y != y) ? 1 : 0;
              v[j] = (__bf16)y;
            }
            pb[s] = v;
          }
          if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        } else {
          if (16 * (s >> 3) < a.k0) {  // whole K=16 groups (k0 is a multiple of 16)
            const int o = 2 * s;
            const float x = a.contiguous ? xr[o] : xrow[tix[o]];
            const float y = (x != x) ? tms[o] : fmaf(x, tsc[o], tsh[o]);
            nbad += (y != y) ? 1 : 0;
            pb[s] = y;
          }
          if ((s & 15) == 15) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    // Row validity: a missing input without a replacement value invalidates the row (PMML NN
    // rule). Each lane half counts its NaN operands (an integer in a VGPR, not a boolean: a flag
    // kept as an SGPR lane mask across the whole layer loop came back wrong on the GPU) and parks
    // the count in LDS for the epilogue.
    int* rbad = s_rowbad + 2 * (wave * 32 + col);  // read back after the layer loop (barriers between)
    rbad[h] = nbad;
    if (prof_on && lane == 0) {
      prof_acc[0] += __builtin_amdgcn_s_memtime() - ts0;
      prof_acc[4] += 1;
    }

    f32x16 out = {};
    for (int L = 0; L < a.n_layers; ++L) {
      const LayerMeta m = a.layers[L];
      const int mtiles = m.mp >> 5;
      const int groups = m.kp >> 4;  // k-step groups of K = 16 (the host pads K to a multiple of 16)
      const bool last = L == a.n_layers - 1;
#pragma unroll 1
      for (int ti = 0; ti < mtiles; ++ti)
        tile_step<BF16>(a, m, ti, groups, last, h, lane, tid, s_b, s_pan, ring, pb, nb, out, p, prof_on, prof_acc);
      if (!last) {
#pragma unroll
        for (int s = 0; s < KS; ++s) pb[s] = nb[s];
      }
    }

    // ---- output layer: units 0..n_out-1 live in tile 0; lanes l and l^32 hold the two halves
    const unsigned long long te0 = prof_on ? __builtin_amdgcn_s_memtime() : 0ull;
    if (prof_on && lane == 0) prof_acc[3] -= te0;  // closed at the loop end (both epilogue paths)
    if (a.final_norm == 0 && a.n_out == 1) {
      if (h == 0 && in_range) {
        const bool bad = (rbad[0] | rbad[1]) != 0;
        apply_epilogue(a.epi, [&](int) { return out[0]; }, !bad, row, a.n_rows, a.score, a.valid, a.probs);
      }
      if (prof_on && lane == 0) prof_acc[3] += __builtin_amdgcn_s_memtime();
      continue;
    }
    float mx = -__builtin_inff();
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (acc_row(r, h) < a.n_out) mx = fmaxf(mx, out[r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float pr[16];
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool u = acc_row(r, h) < a.n_out;
      float v = out[r];
      if (a.final_norm == 1) v = __expf(v - mx);
      pr[r] = u ? v : 0.f;
      sum += pr[r];
    }
    sum += __shfl_xor(sum, 32);
    float best = -__builtin_inff();
    int best_u = 1 << 30;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u = acc_row(r, h);
      if (u < a.n_out) {
        if (a.final_norm != 0) pr[r] /= sum;
        if (pr[r] > best || (pr[r] == best && u < best_u)) { best = pr[r]; best_u = u; }
        if (a.probs && in_range) a.probs[(size_t)row * a.n_out + u] = pr[r];
      }
    }
    const float ob = __shfl_xor(best, 32);
    const int ou = __shfl_xor(best_u, 32);
    if (ob > best || (ob == best && ou < best_u)) { best = ob; best_u = ou; }
    if (h == 0 && in_range) {
      bool ok = (rbad[0] | rbad[1]) == 0 && best == best && best_u < a.n_out;
      float sc = ok ? (a.epi.has_table ? a.epi.table[best_u] : (float)best_u) : __builtin_nanf("");
      ok = ok && (sc == sc);
      a.score[row] = ok ? sc : __builtin_nanf("");
      a.valid[row] = ok ? 1 : 0;
      if (a.epi.score2) {
        a.epi.score2[row] = ok ? sc : __builtin_nanf("");
        a.epi.valid2[row] = ok ? 1 : 0;
      }
    }
    if (prof_on && lane == 0) prof_acc[3] += __builtin_amdgcn_s_memtime();
  }
  if (prof_on && lane == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) a.prof[i] = prof_acc[i];
  }
}

template <bool BF16>
size_t lds_bytes() {
  return (size_t)NSLOT * Cfg<BF16>::PANEL + 4 * KMAX * 4 + (size_t)MAXL * MT * 32 * 4 + (size_t)MAXL * MT * 8 +
         (size_t)Cfg<BF16>::WAVES * 32 * 2 * 4 + 6 * 8;
}

int n_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}


// ================================================================================================
// Register-weight kernel (bf16; 1 or 2 hidden layers of <= 256 units over <= 256 inputs, then an
// output layer of <= 32 units) — the shape of almost every exported PMML NeuralNetwork.
//
// The panel kernel above keeps each wave's ROWS stationary (activations in registers) and streams
// every weight through LDS, one barrier per 32-unit output tile. Here the WEIGHTS are stationary:
// wave w of the 8 owns output tile t = w % T of every hidden layer and holds that tile's A
// fragments (all k-steps) in VGPRs for the whole persistent kernel — loaded once per workgroup,
// never re-read. Activations move through LDS instead: a 128-row block is staged once (fp32 ->
// normalised bf16, already in B-operand layout), each hidden layer reads its B fragments from one
// LDS buffer (conflict-free ds_read_b128, issued ahead) and writes its activated tile into the
// other (two ds_write_b128 per 32 rows: with the host's k permutation an accumulator register IS
// the next layer's B element, so no lane exchange). Two 32-row column blocks run as interleaved
// accumulation chains on the same A registers, so each wave keeps two independent MFMA chains and
// their LDS reads in flight.
//
// FOLD (output layer of <= 4 units, the regression / binary case): the output layer is folded into
// the last hidden layer — each wave dots its fp32 activated tile with the output weights (VALU,
// 16 units per lane + one lane-half exchange) and parks the partial sum per (tile, row) in LDS;
// the epilogue adds the tiles' partials in a fixed order (deterministic), the output bias and
// activation. The software pipeline is then two phases / two barriers per 128-row block:
//   NH = 2:  [hidden 0: buf0 -> buf1 | epilogue of the previous block]  barrier
//            [hidden 1: buf1 -> partials | stage next block -> buf0]     barrier
//   NH = 1:  [hidden 0: buf0 -> partials]  barrier  [epilogue | stage next -> buf0]  barrier
// Without FOLD (more outputs) the output layer is a 1-tile MFMA layer with A fragments staged in
// LDS once, and its fp32 result reaches the epilogue through LDS (four barriers per block).
//
// LDS (<= 156 KiB): 2 activation buffers [4 column blocks][16 k-steps][64 lanes] x 16 B
// (2 x 64 KiB); FOLD: partials [8][128][4] fp32 + output weights [4][256] fp32; else output-layer
// fragments (<= 16 KiB); normalisation tables, biases, per-row flags -> one 512-thread workgroup
// per CU, two waves per SIMD.
constexpr int RR = 128;        // rows per block
constexpr int RCB = RR / 32;   // 32-row column blocks (MFMA N)
constexpr int RKS = 16;        // k-steps per column block in a buffer (K <= 256)
constexpr int RWV = 8;         // waves
constexpr int RT = RWV * 64;   // threads
constexpr int RBUF = RCB * RKS * 64;  // uint4 per activation buffer
constexpr int RFO = 4;         // max outputs of the folded output layer

// ---- accumulation chains: A from registers (compile-time indices after inlining), B from LDS
template <int N>
__device__ __forceinline__ void rchain1_n(const bf16x8* A, const uint4* b, f32x16& acc) {
  constexpr int W = N < 4 ? N : 4;
  uint4 win[W];
#pragma unroll
  for (int i = 0; i < W; ++i) win[i] = b[i * 64];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const uint4 x = win[s % W];
    if (s + W < N) win[s % W] = b[(s + W) * 64];
    bf16x8 B;
    __builtin_memcpy(&B, &x, 16);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[s], B, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// two column blocks on the same A fragments: two independent chains, interleaved MFMA by MFMA
template <int N>
__device__ __forceinline__ void rchain2_n(const bf16x8* A, const uint4* b0, const uint4* b1, f32x16& c0,
                                          f32x16& c1) {
  constexpr int W = N < 2 ? N : 2;
  uint4 w0[W], w1[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
    w0[i] = b0[i * 64];
    w1[i] = b1[i * 64];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const uint4 x0 = w0[s % W], x1 = w1[s % W];
    if (s + W < N) {
      w0[s % W] = b0[(s + W) * 64];
      w1[s % W] = b1[(s + W) * 64];
    }
    bf16x8 B0, B1;
    __builtin_memcpy(&B0, &x0, 16);
    __builtin_memcpy(&B1, &x1, 16);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[s], B0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[s], B1, c1, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int KA, int N = 1>
__device__ __forceinline__ void rchain1(int ks, const bf16x8 (&A)[KA], const uint4* b, f32x16& acc) {
  if (ks == N) {
    rchain1_n<N>(A, b, acc);
  } else if constexpr (N < KA) {
    rchain1<KA, N + 1>(ks, A, b, acc);
  }
}

template <int KA, int N = 1>
__device__ __forceinline__ void rchain2(int ks, const bf16x8 (&A)[KA], const uint4* b0, const uint4* b1,
                                        f32x16& c0, f32x16& c1) {
  if (ks == N) {
    rchain2_n<N>(A, b0, b1, c0, c1);
  } else if constexpr (N < KA) {
    rchain2<KA, N + 1>(ks, A, b0, b1, c0, c1);
  }
}

// output layer without FOLD: both operands from LDS
template <int N>
__device__ __forceinline__ void rchain_ll_n(const uint4* a, const uint4* b, f32x16& acc) {
  constexpr int W = N < 4 ? N : 4;
  uint4 wa[W], wb[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
    wa[i] = a[i * 64];
    wb[i] = b[i * 64];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const uint4 x = wa[s % W], y = wb[s % W];
    if (s + W < N) {
      wa[s % W] = a[(s + W) * 64];
      wb[s % W] = b[(s + W) * 64];
    }
    bf16x8 A, B;
    __builtin_memcpy(&A, &x, 16);
    __builtin_memcpy(&B, &y, 16);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int N = 1>
__device__ __forceinline__ void rchain_ll(int ks, const uint4* a, const uint4* b, f32x16& acc) {
  if (ks == N) {
    rchain_ll_n<N>(a, b, acc);
  } else if constexpr (N < RKS) {
    rchain_ll<N + 1>(ks, a, b, acc);
  }
}

__device__ __forceinline__ void activate16(int act, float thr, f32x16& acc) {
  switch (act) {  // uniform
    case A_IDENTITY: break;
    case A_RELU:
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = fmaxf(acc[r], 0.0f);
      break;
    case A_LOGISTIC:
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 1.0f / (1.0f + __expf(-acc[r]));
      break;
    default:
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = activate(act, acc[r], thr);
      break;
  }
}

__device__ __forceinline__ void bias16(const float* s_b, int t, int h, f32x16& acc) {
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = s_b[32 * t + acc_row(r, h)];
}

struct RLayer {  // one hidden layer as wave w sees it
  int ks, t, q, nq, mreal, act;
  float thr;
};
__device__ __forceinline__ RLayer rlayer(const LayerMeta& m, int w) {
  const int T = m.mp >> 5;
  const int t = w % T;
  return RLayer{m.kp >> 4, t, w / T, (RWV - 1 - t) / T + 1, m.mreal, m.act, m.thr};
}

// activation, zeroed padded units (a padded unit's 0 must stay 0 through e.g. reciprocal), then
// either the bf16 B fragments of the next layer or (FOLD) the partial output dot products
template <bool LAST_FOLD>
__device__ __forceinline__ void rfinish(const RLayer& L, f32x16& acc, int cb, int lane, int h, uint4* bout,
                                        float* s_part, const float* s_wo, int n_out) {
  activate16(L.act, L.thr, acc);
  if (32 * L.t + 32 > L.mreal) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (32 * L.t + acc_row(r, h) >= L.mreal) acc[r] = 0.0f;
  }
  if constexpr (LAST_FOLD) {
    const int col = lane & 31;
    for (int o = 0; o < n_out; ++o) {  // uniform, <= 4
      const float* wo = s_wo + o * 256 + 32 * L.t;
      float p = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) p = fmaf(acc[r], wo[acc_row(r, h)], p);
      // lane-half sum without an LDS round trip: v_permlane32_swap (CDNA4)
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(p), __float_as_uint(p), false, false);
      p = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
      if (h == 0) s_part[(L.t * RR + 32 * cb + col) * RFO + o] = p;
    }
  } else {
    bf16x8 lo, hi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lo[j] = (__bf16)acc[j];
      hi[j] = (__bf16)acc[8 + j];
    }
    uint4 ulo, uhi;
    __builtin_memcpy(&ulo, &lo, 16);
    __builtin_memcpy(&uhi, &hi, 16);
    bout[(cb * RKS + 2 * L.t) * 64 + lane] = ulo;
    bout[(cb * RKS + 2 * L.t + 1) * 64 + lane] = uhi;
  }
}

// One hidden layer for wave w: its tile over the column blocks it owns, two at a time.
template <int KA, bool LAST_FOLD>
__device__ __forceinline__ void rhidden(const RLayer& L, const bf16x8 (&A)[KA], int lane, int h, const uint4* bin,
                                        uint4* bout, const float* s_b, float* s_part, const float* s_wo,
                                        int n_out) {
  int cb = L.q;
  for (; cb + L.nq < RCB; cb += 2 * L.nq) {
    const int cb1 = cb + L.nq;
    f32x16 c0;
    bias16(s_b, L.t, h, c0);
    f32x16 c1 = c0;
    rchain2<KA>(L.ks, A, bin + cb * RKS * 64 + lane, bin + cb1 * RKS * 64 + lane, c0, c1);
    rfinish<LAST_FOLD>(L, c0, cb, lane, h, bout, s_part, s_wo, n_out);
    rfinish<LAST_FOLD>(L, c1, cb1, lane, h, bout, s_part, s_wo, n_out);
  }
  if (cb < RCB) {
    f32x16 c0;
    bias16(s_b, L.t, h, c0);
    rchain1<KA>(L.ks, A, bin + cb * RKS * 64 + lane, c0);
    rfinish<LAST_FOLD>(L, c0, cb, lane, h, bout, s_part, s_wo, n_out);
  }
}

// Staging item i of a block: 8 consecutive inputs (k-group kg) of one row; 8 consecutive items are
// 8 consecutive rows of one k-group (coalesced row segments, conflict-free 16-B LDS stores).
struct RItem {
  int row, kg;
};
__device__ __forceinline__ RItem ritem(int i, int KG) {
  const int c_lo = i & 7;
  const int rest = i >> 3;
  return RItem{8 * (rest / KG) + c_lo, rest % KG};
}

__device__ __forceinline__ void rload(const MlpArgs& a, const int* s_ix, int row, int kg, bool vec, float (&v)[8]) {
  if (row >= a.n_rows) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    return;
  }
  const float* xr = a.X + (size_t)row * a.ldx;
  if (vec) {
    const float4 p = *reinterpret_cast<const float4*>(xr + 8 * kg);
    const float4 q = *reinterpret_cast<const float4*>(xr + 8 * kg + 4);
    v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w;
    v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * kg + j;
      v[j] = k < a.n_in ? xr[s_ix[k]] : 0.f;
    }
  }
}

__device__ __forceinline__ void rstore(const MlpArgs& a, const float* s_sc, const float* s_sh, const float* s_ms,
                                       int row, int row0, int kg, const float (&v)[8], uint4* buf, int* s_bad) {
  bf16x8 o;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kg + j;
    const float x = v[j];
    float y = (x != x) ? s_ms[k] : fmaf(x, s_sc[k], s_sh[k]);
    if (k >= a.n_in || row0 + row >= a.n_rows) y = 0.f;
    bad = bad || (y != y);
    o[j] = (__bf16)y;
  }
  if (bad && row0 + row < a.n_rows) s_bad[row] = 1;
  uint4 u;
  __builtin_memcpy(&u, &o, 16);
  const int s = kg >> 1, hh = kg & 1, cb = row >> 5, col = row & 31;
  buf[(cb * RKS + s) * 64 + hh * 32 + col] = u;
}

// Output values of one row (accessor out(u), u < n_out) -> final normalisation, label / target
// decode, score / valid / probability stores.
template <typename Out>
__device__ __forceinline__ void repilogue(const MlpArgs& a, Out out, bool bad, int row) {
  if (a.final_norm == 0 && a.n_out == 1) {
    apply_epilogue(a.epi, [&](int) { return out(0); }, !bad, row, a.n_rows, a.score, a.valid, a.probs);
    return;
  }
  float mx = -__builtin_inff();
  for (int u = 0; u < a.n_out; ++u) mx = fmaxf(mx, out(u));
  float sum = 0.f;
  for (int u = 0; u < a.n_out; ++u) sum += (a.final_norm == 1) ? __expf(out(u) - mx) : out(u);
  float best = -__builtin_inff();
  int best_u = 1 << 30;
  for (int u = 0; u < a.n_out; ++u) {
    float p = (a.final_norm == 1) ? __expf(out(u) - mx) : out(u);
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

// NH hidden layers (A in registers: KA0 k-steps for layer 0, 16 for layer 1) + output layer.
// PF: staging items prefetched per thread (vector-loadable rows, k0 <= 64: 2 items = 16 VGPRs);
// 0 = load at staging. FOLD: output layer (<= 4 units) folded into the last hidden layer.
template <int NH, int KA0, int PF, bool FOLD>
__global__ __launch_bounds__(RT, 1) void mlp_reg_kernel(MlpArgs a) {
  extern __shared__ __align__(16) uint4 rsm[];
  uint4* buf0 = rsm;
  uint4* buf1 = rsm + RBUF;
  uint4* s_oa = rsm + 2 * RBUF;                                    // !FOLD: output-layer A [RKS][64]
  float* s_part = reinterpret_cast<float*>(rsm + 2 * RBUF);        // FOLD: [8 tiles][RR][RFO]
  float* s_wo = s_part + RWV * RR * RFO;                           // FOLD: [RFO][256] output weights
  float* s_sc = FOLD ? s_wo + RFO * 256 : reinterpret_cast<float*>(s_oa + RKS * 64);
  float* s_sh = s_sc + KMAX;
  float* s_ms = s_sh + KMAX;
  int* s_ix = reinterpret_cast<int*>(s_ms + KMAX);
  float* s_b = reinterpret_cast<float*>(s_ix + KMAX);              // [3][256]
  int* s_bad = reinterpret_cast<int*>(s_b + 3 * 256);              // [2][RR] per block parity

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int col = lane & 31;
  const LayerMeta m0 = a.layers[0];
  const LayerMeta m1 = a.layers[NH >= 2 ? 1 : 0];
  const LayerMeta mo = a.layers[NH];
  const int KG = a.k0 >> 3;  // k-groups of 8 inputs (k0 is a multiple of 16)
  const bool vec = a.contiguous && (a.ldx & 3) == 0 && ((uintptr_t)a.X & 15) == 0;
  const int n_out = a.n_out;

  // ---- once per workgroup: tables, biases, output layer, this wave's A fragments
  for (int k = tid; k < KMAX; k += RT) {
    const bool u = k < a.n_in;
    s_sc[k] = u ? a.in_scale[k] : 0.f;
    s_sh[k] = u ? a.in_shift[k] : 0.f;
    s_ms[k] = u ? a.in_missing[k] : 0.f;
    s_ix[k] = u ? a.in_index[k] : 0;
  }
  for (int i = tid; i < (NH + 1) * 256; i += RT) {
    const int L = i >> 8, u = i & 255;
    const LayerMeta& m = L == 0 ? m0 : (L == NH ? mo : m1);
    s_b[i] = u < m.mp ? a.biases[m.b_off + u] : 0.f;
  }
  for (int i = tid; i < 2 * RR; i += RT) s_bad[i] = 0;
  const uint4* W4 = reinterpret_cast<const uint4*>(a.weights);
  const int kso = mo.kp >> 4;
  if constexpr (FOLD) {
    // the output layer's weights W[o][k] back from its A fragments (one 32-unit tile):
    // fragment (s, lane = (h', r)) element j = W[unit r][B-k index 16 s + 8 h' + j]
    const __bf16* Wb = reinterpret_cast<const __bf16*>(a.weights) + mo.w_off;
    for (int i = tid; i < RFO * 256; i += RT) {
      const int o = i >> 8, k = i & 255;
      float v = 0.f;
      if (o < n_out && k < mo.kp) {
        const int s = k >> 4, hh = (k >> 3) & 1, j = k & 7;
        v = (float)Wb[((size_t)s * 64 + hh * 32 + o) * 8 + j];
      }
      // B-k index k of the last hidden layer's output = unit acc_row(r, h) of tile k / 32 with
      // r = 8 * ((k >> 4) & 1) + (k & 7), h = (k >> 3) & 1 (the host permutation, inverted)
      const int t = k >> 5, rr = 8 * ((k >> 4) & 1) + (k & 7), hh2 = (k >> 3) & 1;
      s_wo[o * 256 + 32 * t + acc_row(rr, hh2)] = v;
    }
  } else {
    for (int i = tid; i < kso * 64; i += RT) s_oa[i] = W4[mo.w_off / 8 + i];
  }
  bf16x8 A0[KA0];
  bf16x8 A1[NH >= 2 ? RKS : 1];
  const RLayer L0 = rlayer(m0, w);
  const RLayer L1 = rlayer(m1, w);
#pragma unroll
  for (int s = 0; s < KA0; ++s) {
    if (s < L0.ks) {
      const uint4 u = W4[m0.w_off / 8 + (L0.t * L0.ks + s) * 64 + lane];
      __builtin_memcpy(&A0[s], &u, 16);
    }
  }
  if constexpr (NH >= 2) {
#pragma unroll
    for (int s = 0; s < RKS; ++s) {
      if (s < L1.ks) {
        const uint4 u = W4[m1.w_off / 8 + (L1.t * L1.ks + s) * 64 + lane];
        __builtin_memcpy(&A1[s], &u, 16);
      }
    }
  }
  const int T_last = ((NH == 2 ? m1.mp : m0.mp) >> 5);
  float* s_out = reinterpret_cast<float*>(NH == 2 ? buf1 : buf0);  // !FOLD: [RR][33] fp32 output layer
  // Retire the A-fragment loads here, explicitly: otherwise the compiler's wait for them sits at
  // their first use INSIDE the block loop as a vmcnt(0), which every block would then also spend
  // waiting for the record prefetch of the next block (issued just before).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  const int n_blk = (a.n_rows + RR - 1) / RR;
  const int n_items = RR * KG;
  // PF > 0: this thread's staging items are the same in every block (i = tid + it * RT), so only
  // their row pointers advance between blocks
  float4 pf[PF > 0 ? PF : 1][2];
  auto prefetch = [&](int b) {
    if constexpr (PF > 0) {
      if (b < n_blk) {
#pragma unroll
        for (int it = 0; it < PF; ++it) {
          const int i = tid + it * RT;
          const RItem ri = ritem(i, KG);
          const int row = min(b * RR + ri.row, a.n_rows - 1);
          const float4* src = reinterpret_cast<const float4*>(a.X + (size_t)row * a.ldx + 8 * ri.kg);
          if (i < n_items) {
            pf[it][0] = src[0];
            pf[it][1] = src[1];
          }
        }
      }
    }
  };
  auto stage = [&](int b, int par) {  // block b -> buf0 (normalised bf16, B layout of layer 0)
    const int row0 = b * RR;
    int* bad = s_bad + par * RR;
    if constexpr (PF > 0) {
#pragma unroll
      for (int it = 0; it < PF; ++it) {
        const int i = tid + it * RT;
        if (i < n_items) {
          const RItem ri = ritem(i, KG);
          const float v[8] = {pf[it][0].x, pf[it][0].y, pf[it][0].z, pf[it][0].w,
                              pf[it][1].x, pf[it][1].y, pf[it][1].z, pf[it][1].w};
          rstore(a, s_sc, s_sh, s_ms, ri.row, row0, ri.kg, v, buf0, bad);
        }
      }
      prefetch(b + gridDim.x);  // the next block's records load while this one computes
    } else {
      for (int i = tid; i < n_items; i += RT) {
        const RItem ri = ritem(i, KG);
        float v[8];
        rload(a, s_ix, row0 + ri.row, ri.kg, vec, v);
        rstore(a, s_sc, s_sh, s_ms, ri.row, row0, ri.kg, v, buf0, bad);
      }
    }
  };
  auto epilogue_fold = [&](int b, int par) {  // block b's rows from the partials (fixed tile order)
    if (tid < RR) {
      const int row = b * RR + tid;
      const bool bad = s_bad[par * RR + tid] != 0;
      s_bad[par * RR + tid] = 0;
      if (row < a.n_rows) {
        float z[RFO];
#pragma unroll
        for (int o = 0; o < RFO; ++o) {
          if (o < n_out) {
            float acc = s_b[NH * 256 + o];
            for (int t = 0; t < T_last; ++t) acc += s_part[(t * RR + tid) * RFO + o];
            z[o] = activate(mo.act, acc, mo.thr);
          }
        }
        repilogue(a, [&](int u) {
          float r = z[0];
#pragma unroll
          for (int o = 1; o < RFO; ++o) r = (u == o) ? z[o] : r;
          return r;
        }, bad, row);
      }
    }
  };

  const bool prof_on = a.prof != nullptr && blockIdx.x == 0 && w == 0;
  unsigned long long pacc[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
  unsigned long long tp = prof_on ? __builtin_amdgcn_s_memtime() : 0ull;
  auto stamp = [&](int i) {  // optional phase timers (kbench --mlp-prof): wave 0 of workgroup 0
    if (prof_on) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      pacc[i] += t - tp;
      tp = t;
    }
  };

  int blk = blockIdx.x;
  int par = 0;  // block parity: s_bad half of the current block
  prefetch(blk);
  if (blk < n_blk) stage(blk, 0);
  __syncthreads();
  stamp(4);

  if constexpr (FOLD) {
    int prev = -1;
    for (; blk < n_blk; blk += gridDim.x, par ^= 1) {
      const int nxt = blk + gridDim.x;
      if constexpr (NH == 2) {
        rhidden<KA0, false>(L0, A0, lane, h, buf0, buf1, s_b, s_part, s_wo, n_out);
        stamp(0);
        if (prev >= 0) epilogue_fold(prev, par ^ 1);
        __syncthreads();
        stamp(1);
        rhidden<RKS, true>(L1, A1, lane, h, buf1, nullptr, s_b + 256, s_part, s_wo, n_out);
        stamp(2);
        if (nxt < n_blk) stage(nxt, par ^ 1);
        __syncthreads();
        stamp(3);
        prev = blk;
      } else {
        rhidden<KA0, true>(L0, A0, lane, h, buf0, nullptr, s_b, s_part, s_wo, n_out);
        __syncthreads();
        stamp(1);
        epilogue_fold(blk, par);
        if (nxt < n_blk) stage(nxt, par ^ 1);
        __syncthreads();
        stamp(2);
      }
      pacc[5] += 1;
    }
    if (NH == 2 && prev >= 0) epilogue_fold(prev, par ^ 1);
  } else {
    for (; blk < n_blk; blk += gridDim.x, par ^= 1) {
      const int row0 = blk * RR;
      rhidden<KA0, false>(L0, A0, lane, h, buf0, buf1, s_b, nullptr, nullptr, 0);
      __syncthreads();
      stamp(1);
      if constexpr (NH >= 2) {
        rhidden<RKS, false>(L1, A1, lane, h, buf1, buf0, s_b + 256, nullptr, nullptr, 0);
        __syncthreads();
      }
      stamp(2);
      // output layer: one tile, waves 0..3 take one column block each
      const uint4* bo = NH == 2 ? buf0 : buf1;
      if (w < RCB) {
        const int cb = w;
        f32x16 acc;
        bias16(s_b + NH * 256, 0, h, acc);
        rchain_ll(kso, s_oa + lane, bo + cb * RKS * 64 + lane, acc);
        activate16(mo.act, mo.thr, acc);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int u = acc_row(r, h);
          if (u < n_out) s_out[(32 * cb + col) * 33 + u] = acc[r];
        }
      }
      __syncthreads();
      stamp(3);
      if (tid < RR) {
        const int row = row0 + tid;
        const bool bad = s_bad[par * RR + tid] != 0;
        s_bad[par * RR + tid] = 0;
        const float* o = s_out + tid * 33;
        if (row < a.n_rows) repilogue(a, [&](int u) { return o[u]; }, bad, row);
      }
      __syncthreads();  // s_out / buf0 are read above and restaged below
      const int nxt = blk + gridDim.x;
      if (nxt < n_blk) stage(nxt, par ^ 1);
      __syncthreads();
      stamp(4);
      pacc[5] += 1;
    }
  }
  if (prof_on && lane == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) a.prof[i] = pacc[i];
  }
}

template <bool FOLD>
constexpr size_t reg_lds_bytes() {
  return (size_t)2 * RBUF * 16 + (FOLD ? (size_t)(RWV * RR * RFO + RFO * 256) * 4 : (size_t)RKS * 64 * 16) +
         4 * KMAX * 4 + 3 * 256 * 4 + 2 * RR * 4;
}

template <int NH, int KA0, int PF, bool FOLD>
int launch_reg(hipStream_t stream, const MlpArgs& a) {
  const int n_blk = (a.n_rows + RR - 1) / RR;
  dim3 grid(min(n_blk, n_cus()));
  const size_t lds = reg_lds_bytes<FOLD>();
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(mlp_reg_kernel<NH, KA0, PF, FOLD>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -5;
  hipLaunchKernelGGL((mlp_reg_kernel<NH, KA0, PF, FOLD>), grid, dim3(RT), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

template <int NH, bool FOLD>
int launch_reg_nh(hipStream_t stream, const MlpArgs& a, bool narrow) {
  return narrow ? launch_reg<NH, 4, 2, FOLD>(stream, a) : launch_reg<NH, 16, 0, FOLD>(stream, a);
}

}  // namespace

PMML_API int pmml_mlp_args_size() { return (int)sizeof(MlpArgs); }
PMML_API int pmml_mlp_layer_meta_size() { return (int)sizeof(LayerMeta); }

PMML_API int pmml_mlp_launch(hipStream_t stream, const MlpArgs* args, int bf16) {
  const MlpArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_layers < 1 || a.n_layers > MAXL || a.n_out > 32 || a.k0 > KMAX || a.n_in > KMAX || a.n_panels < 1 ||
      a.n_panels > MAXL * MT)
    return -4;
  if (bf16 && a.reg_kernel) {
    // register-weight kernel: the host (runtime/nn_plans.py::reg_kernel_ok) checked every layer's
    // shape (hidden K, M <= 256, output layer one 32-unit tile)
    if (a.n_layers < 2 || a.n_layers > 3) return -4;
    const bool vec = a.contiguous && (a.ldx & 3) == 0 && ((uintptr_t)a.X & 15) == 0;
    const bool narrow = a.k0 <= 64 && vec;  // prefetching variant: vector row loads
    const bool fold = a.n_out <= RFO;
    if (a.n_layers == 2)
      return fold ? launch_reg_nh<1, true>(stream, a, narrow) : launch_reg_nh<1, false>(stream, a, narrow);
    return fold ? launch_reg_nh<2, true>(stream, a, narrow) : launch_reg_nh<2, false>(stream, a, narrow);
  }
  const int waves = bf16 ? Cfg<true>::WAVES : Cfg<false>::WAVES;
  const int n_tiles = (a.n_rows + 32 * waves - 1) / (32 * waves);
  dim3 grid(min(n_tiles, n_cus()));
  if (bf16) {
    const size_t lds = lds_bytes<true>();
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(mlp_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -5;
    hipLaunchKernelGGL(mlp_kernel<true>, grid, dim3(64 * waves), lds, stream, a);
  } else {
    const size_t lds = lds_bytes<false>();
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(mlp_kernel<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -5;
    hipLaunchKernelGGL(mlp_kernel<false>, grid, dim3(64 * waves), lds, stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
