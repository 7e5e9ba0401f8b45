// Tree-ensemble scoring (PMML TreeModel / MiningModel GBDT, random forest, model chains).
//
// Design (MI355X / CDNA4):
//  * rows-stationary: one 256-thread workgroup (4 wave64s) owns 256 rows, one row per lane, for
//    the whole ensemble; the prepared feature tile lives in LDS transposed as [F][256] so that a
//    lane's feature read `feat[f][lane]` is bank-conflict free whatever feature each lane needs;
//  * trees stream through an LDS chunk buffer shared by the 4 waves (the ensemble is L2/MALL
//    resident, so every workgroup re-reads it at L2 bandwidth, not HBM);
//  * PERFECT layout for depth <= 10: every tree is padded to a perfect binary tree of depth D,
//    nodes are 8 bytes {threshold, meta} in level order, traversal is branch-free
//    `idx = 2*idx + 1 + (x >= T)` for exactly D steps — no divergence, one ds_read_b64 + one
//    ds_read_b32 per level, ILP trees interleaved per lane to hide LDS latency;
//    split operators are canonicalised on the host to "go right iff x >= T" with T rounded so the
//    fp32 comparison is exact for fp32 inputs (see runtime/plans.py);
//  * POINTER layout for deeper / wider ensembles: {T, meta, left, right} nodes read from global
//    memory (L2-resident), divergent walk;
//  * the per-row epilogue (sum / average / vote / link function / label table) is fused;
//  * WIDE kernel (the default for P = 1 ensembles, tree_perfect_wide_kernel): 1024 threads per CU
//    own 256 / 128 / 64 rows x G tree groups; sum ensembles on 256-row tiles claim 8-tree batches
//    dynamically (deterministic slot sums); fp8 leaf pairs / VOTE8 class codes live in the
//    last-level node words. Its walk is LDS-port bound (profiles/r2_tree_variants.md).
//
// Missing values: a per-node default-direction bit routes NaN (XGBoost / LightGBM `defaultChild`).
// PMML `missingValueStrategy="nullPrediction"` (scikit-learn exports) and `none` with complement
// predicates + `returnNullPrediction` make the tree's prediction null when a visited split sees a
// missing value: flag bit NI of the perfect record's default-right words (node index NI does not
// exist), bit 30 of the pointer node's meta. A null tree poisons the row's sum with NaN
// (-> EmptyScore, the MiningModel `returnMissing`/`continue` rule), or marks the row invalid for
// multi-slot accumulators.
//
// fp8 leaves (variant 2, BASELINE config 5): the two leaves below every last-level node are
// stored as OCP e4m3 bytes in the upper half of that node's meta word (the lower half is the
// feature byte offset, < 64 KiB); one global scale is folded into the epilogue. Thresholds and
// decisions stay fp32 — only the leaf values are quantised. The record shrinks by the whole leaf
// array (768 -> 512 B at depth 6) and the last level needs no separate leaf read.
//
// This header holds the PERFECT-layout kernels (narrow + wide) and their launcher template; every
// depth is instantiated in its own translation unit (tree_d<D>.hip) so the build parallelises.
#pragma once
#include "epilogue.h"

namespace pmml_tree {

constexpr int TB = 256;   // rows per workgroup (= threads)

struct TreeArgs {
  const float* X;
  int n_rows, n_feat, ldx;
  int pad0;
  const FieldPrep* prep;        // nullable
  const uint8_t* row_valid_in;  // nullable
  const uint32_t* blob;         // perfect: [n_trees][rec_words]; pointer: nodes uint4[]
  const int* roots;             // pointer layout: per-tree root code (>=0 node, <0 ~leaf)
  const float* leaves;          // pointer layout: [n_leaves][P]
  const int* tree_slot;         // general accumulation: slot per tree
  int n_trees, rec_words, chunk_trees, P;
  int C, trees_per_split, general, variant;  // variant & 3: 1 wide perfect kernel, 2 wide + fp8 leaves;
                                             // | VAR_NAN_FAST | VAR_NAN_PLANES (wide kernel only)
  Epilogue epi;
  float* score;
  uint8_t* valid;
  float* probs;
  float* partial;               // split mode: [splits][C+1][n_rows]
  const uint32_t* blob_nan;     // wide kernel, nullable: the records re-pointed at the NaN plane
  int chunk_trees_nan;          // (tiles with missing values; own chunk size, LDS holds 2 planes)
  int xcd_split;                // pointer / hybrid layouts: > 0 = XCD-aware tree splits (tree_block)
  const float* tree_w;          // wide MODE_CLASS: per-tree vote weight (nullable = 1)
  const float* acc_init;        // wide multi-class: per-class initial accumulator (nullable = 0)
  const int* feat_map;          // wide kernel: staged column j -> X column (nullable = identity)
  int rows_wide, mode;          // wide kernel: rows per workgroup (256/128/64), accumulation mode
  int n_stage, pilp;            // wide kernel: staged feature columns; pointer kernel: walks per lane (4/8/16)
  unsigned long long* prof;     // nullable: per-wave phase ticks of one workgroup ([16][4], s_memtime)
  const float* rank_thr;        // RANK3 pointer layout: per feature, its sorted unique split thresholds
  const int* rank_cnt;          // ... and their count (<= 254); row f of rank_thr starts at f * rank_stride
  int rank_stride;
  int leaf_onehot;               // pointer_walk GENERAL: leaves are {class, weight bits} int pairs (one-hot votes)
};
// One grouped launch of the wide kernel over a mixed-model slice (tree_grouped_wide_kernel).
struct GroupedTreeArgs {
  const TreeArgs* models;   // [n_models] device copies of the entries' launch args (row fields unset)
  const int* model_code;    // [n_models] the entry's model code (index into row_start)
  const int* row_start;     // [K + 1] grouped-row range of every code in this slice (device)
  const int* tile_start;    // [n_models + 1] first tile of every entry, prefix over all entries (device)
  const float* Xg;          // grouped rows [m][F]
  const int* perm;          // grouped row -> arrival-order row of the slice
  float* out_s;             // arrival-order outputs of the slice
  uint8_t* out_v;
  int n_models, F;
};
constexpr int VAR_NAN_FAST = 4;    // wide kernel: take the fast path even on tiles with missing values
constexpr int VAR_NAN_PLANES = 8;  // ... via blob_nan + a second feature plane (NaN -> +inf)
constexpr int VAR_POINTER_REFILL = 16;  // pointer layout: refill schedule (tree.hip)
constexpr int VAR_POINTER_COMPACT = 32; // pointer layout: 8-byte BFS slots (tree.hip::tree_compact_kernel)
constexpr int VAR_POINTER_MASKED = 64;  // pointer layout, lock-step sums: exec-masked loads of finished walks
constexpr int VAR_POINTER_SUPER = 128;  // pointer layout: two levels per 16-byte slot (tree.hip::tree_super_kernel)
constexpr int VAR_POINTER_USKIP = 256;  // pointer layout, lock-step: wave-uniform skip of finished walk slots
constexpr int VAR_POINTER_PEEL = 512;   // pointer layout, lock-step: top two levels from uniform (scalar) loads
constexpr int VAR_POINTER_RANK3 = 1024; // pointer layout: three levels per 16-byte record on threshold ranks (tree.hip)
constexpr int VAR_POINTER_INLINE = 4096; // pointer layout, lock-step: leaf payloads inline in the parent (tree.hip)
constexpr int VAR_POINTER_LTOP = 8192;   // pointer layout, lock-step, BFS: top levels of each group's trees from LDS

// per-depth launchers (tree_d<D>.hip)
#define PMML_TREE_DECL(D) int launch_perfect_d##D(hipStream_t st, const TreeArgs& a, dim3 grid, size_t lds); \
  int launch_grouped_d##D(hipStream_t st, const TreeArgs& a, const GroupedTreeArgs& g, int tiles, size_t lds);
PMML_TREE_DECL(1) PMML_TREE_DECL(2) PMML_TREE_DECL(3) PMML_TREE_DECL(4) PMML_TREE_DECL(5)
PMML_TREE_DECL(6) PMML_TREE_DECL(7) PMML_TREE_DECL(8) PMML_TREE_DECL(9) PMML_TREE_DECL(10)
#undef PMML_TREE_DECL

namespace {

// Workgroup -> (row block, tree split). Default: grid (row blocks, splits). XCD-aware mode
// (a.xcd_split = S > 0): a 1-D grid of row_blocks * S workgroups where workgroup L scores tree
// split L % S of row block L / S. The dispatcher deals workgroups to the 8 XCDs round-robin
// (L % 8), so with S = 8 every XCD only ever walks ONE eighth of the forest: a deep forest too big
// for one 4 MiB L2 (300 trees x depth 14 = 14 MB of nodes) is split into 8 slices that each stay
// L2-resident, instead of every XCD gathering the whole forest from the Infinity Cache. The 8
// workgroups of one row block run side by side, so the row tile they each stage is one HBM read.
// Placement is a speed hint only; correctness never depends on it.
__device__ __forceinline__ int2 tree_block(const TreeArgs& a) {
  if (a.xcd_split > 0) {
    const int L = blockIdx.x;
    return make_int2(L / a.xcd_split, L % a.xcd_split);
  }
  return make_int2(blockIdx.x, blockIdx.y);
}

__device__ __forceinline__ void finish_row(const TreeArgs& a, float acc0, const float* accl, int split,
                                           bool general, int row, bool row_ok) {
  if (row >= a.n_rows) return;
  if (a.partial) {
    const size_t stride = (size_t)a.n_rows;
    float* base = a.partial + (size_t)split * (a.C + 1) * stride;
    if (general) {
      for (int c = 0; c < a.C; ++c) base[c * stride + row] = accl[c * TB + threadIdx.x];
    } else {
      base[row] = acc0;
    }
    base[a.C * stride + row] = row_ok ? 0.f : 1.f;
    return;
  }
  if (general) {
    apply_epilogue(a.epi, [&](int c) { return accl[c * TB + threadIdx.x]; }, row_ok, row, a.n_rows, a.score,
                   a.valid, a.probs);
  } else {
    apply_epilogue(a.epi, [&](int) { return acc0; }, row_ok, row, a.n_rows, a.score, a.valid, a.probs);
  }
}

// Tree-level "null prediction on a missing value" flag of a perfect record (bit NI of the
// default-right words, which start at word dr_off).
template <int DEPTH>
__device__ __forceinline__ bool null_flag(const char* rec, int dr_off) {
  constexpr int NI = (1 << DEPTH) - 1;
  return ((reinterpret_cast<const uint32_t*>(rec)[dr_off + (NI >> 5)] >> (NI & 31)) & 1u) != 0u;
}

// Next-chunk prefetch through registers: the global loads are issued before the traversal of the
// current chunk and written to the other LDS buffer after it, so L2 latency hides under compute.
// (An LDS-DMA variant was slower: hipcc drains in-flight LDS-DMA before the first ds_read it cannot
// prove disjoint from the DMA target, which serialised the copy with the traversal.)
constexpr int PREFETCH_Q = 8;  // uint4 per lane -> up to 32 KiB per chunk

// Loads are unconditional (index clamped into the valid range) so the values stay in VGPRs; only
// the LDS store is predicated. Written as macros over named registers: an array passed between
// helpers was demoted to scratch by hipcc.
#define PF_DECL uint4 pf0, pf1, pf2, pf3, pf4, pf5, pf6, pf7;
#define PF_LOAD1(R, I, S4, LAST) R = (S4)[min((int)threadIdx.x + (I) * TB, (LAST))];
#define PF_LOAD(SRC, N16)                                                              \
  {                                                                                    \
    const uint4* s4_ = reinterpret_cast<const uint4*>(SRC);                            \
    const int last_ = (N16) > 0 ? (N16) - 1 : 0;                                      \
    PF_LOAD1(pf0, 0, s4_, last_) PF_LOAD1(pf1, 1, s4_, last_) PF_LOAD1(pf2, 2, s4_, last_) \
    PF_LOAD1(pf3, 3, s4_, last_) PF_LOAD1(pf4, 4, s4_, last_) PF_LOAD1(pf5, 5, s4_, last_) \
    PF_LOAD1(pf6, 6, s4_, last_) PF_LOAD1(pf7, 7, s4_, last_)                          \
  }
#define PF_STORE1(R, I, D4, N)                      \
  {                                                  \
    const int idx_ = (int)threadIdx.x + (I) * TB;   \
    if (idx_ < (N)) (D4)[idx_] = R;                  \
  }
#define PF_STORE(DST, N16)                                                              \
  {                                                                                     \
    uint4* d4_ = reinterpret_cast<uint4*>(DST);                                         \
    PF_STORE1(pf0, 0, d4_, N16) PF_STORE1(pf1, 1, d4_, N16) PF_STORE1(pf2, 2, d4_, N16) \
    PF_STORE1(pf3, 3, d4_, N16) PF_STORE1(pf4, 4, d4_, N16) PF_STORE1(pf5, 5, d4_, N16) \
    PF_STORE1(pf6, 6, d4_, N16) PF_STORE1(pf7, 7, d4_, N16)                             \
  }

// Traverse `nt` perfect trees of one LDS chunk for this lane's row.
// Heap index j (root = 1): node j at byte (j-1)*8, children 2j / 2j+1, leaf j - 2^D.
// Fast path (MISSING=false): one ds_read_b64 node, one ds_read_b32 feature, one v_cmp, index update.
template <int DEPTH, bool GENERAL, bool MISSING, int ILP>
__device__ __forceinline__ void traverse_chunk(const TreeArgs& a, const uint32_t* buf, int nt, int t0,
                                               const char* feat_lane, float& acc, float* accl, bool& poisoned) {
  constexpr int NI = (1 << DEPTH) - 1;
  constexpr int NL = 1 << DEPTH;
  const int rw = a.rec_words;
  const int dr_off = 2 * NI + NL * a.P;  // words
  const int tid = threadIdx.x;
  int k = 0;
  for (; k + ILP <= nt; k += ILP) {
    uint32_t j[ILP];
    uint32_t pz[ILP];
    const char* base[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      j[i] = 1u;
      pz[i] = 0u;
      base[i] = reinterpret_cast<const char*>(buf + (k + i) * rw);
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        const uint2 nd = *reinterpret_cast<const uint2*>(base[i] - 8 + (j[i] << 3));
        const float x = *reinterpret_cast<const float*>(feat_lane + nd.y);
        uint32_t right = (x >= __uint_as_float(nd.x)) ? 1u : 0u;
        if (MISSING) {  // branch-free: NaN takes the node's default direction bit
          const uint32_t n = j[i] - 1u;
          const uint32_t w = reinterpret_cast<const uint32_t*>(base[i])[dr_off + (n >> 5)];
          const uint32_t isn = (x != x) ? 1u : 0u;
          right |= isn & (w >> (n & 31u));
          pz[i] |= isn;
        }
        j[i] = j[i] + j[i] + right;
      }
    }
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      const float* lv = reinterpret_cast<const float*>(base[i] + NI * 8) - NL * a.P;
      const bool pzn = MISSING && pz[i] && null_flag<DEPTH>(base[i], dr_off);
      if (GENERAL) {
        poisoned = poisoned || pzn;
        const int slot = a.tree_slot[t0 + k + i];
        for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += lv[j[i] * a.P + p];
      } else {
        acc += pzn ? __builtin_nanf("") : lv[j[i]];
      }
    }
  }
  for (; k < nt; ++k) {
    uint32_t j = 1u, pz = 0u;
    const char* base = reinterpret_cast<const char*>(buf + k * rw);
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const uint2 nd = *reinterpret_cast<const uint2*>(base - 8 + (j << 3));
      const float x = *reinterpret_cast<const float*>(feat_lane + nd.y);
      uint32_t right = (x >= __uint_as_float(nd.x)) ? 1u : 0u;
      if (MISSING) {
        const uint32_t n = j - 1u;
        const uint32_t w = reinterpret_cast<const uint32_t*>(base)[dr_off + (n >> 5)];
        const uint32_t isn = (x != x) ? 1u : 0u;
        right |= isn & (w >> (n & 31u));
        pz |= isn;
      }
      j = j + j + right;
    }
    const float* lv = reinterpret_cast<const float*>(base + NI * 8) - NL * a.P;
    const bool pzn = MISSING && pz && null_flag<DEPTH>(base, dr_off);
    if (GENERAL) {
      poisoned = poisoned || pzn;
      const int slot = a.tree_slot[t0 + k];
      for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += lv[j * a.P + p];
    } else {
      acc += pzn ? __builtin_nanf("") : lv[j];
    }
  }
}

template <int DEPTH, bool GENERAL, int ILP>
__global__ __launch_bounds__(TB, 2) void tree_perfect_kernel(TreeArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  const int rw = a.rec_words;
  const int chunk_words = a.chunk_trees * rw;
  float* feat = reinterpret_cast<float*>(smem);
  uint32_t* tbuf0 = smem + a.n_feat * TB;
  uint32_t* tbuf1 = tbuf0 + chunk_words;
  int* bad = reinterpret_cast<int*>(tbuf1 + chunk_words);
  int* any_missing = bad + TB;
  float* accl = reinterpret_cast<float*>(bad + TB + 4);

  const int tid = threadIdx.x;
  const int row0 = blockIdx.x * TB;
  const int split = blockIdx.y;
  const int tb = split * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);

  // chunk 0: issue its loads before the row staging so the two overlap
  PF_DECL
  int n16 = (tb < te) ? (min(a.chunk_trees, te - tb) * rw) >> 2 : 0;
  PF_LOAD(n16 > 0 ? a.blob + (size_t)tb * rw : a.blob, n16)

  // stage rows [F][TB] with field preparation; rows past the end are zero (never "missing")
  if (tid == 0) *any_missing = 0;
  bad[tid] = 0;
  __syncthreads();
  {
    const int F = a.n_feat;
    const int total = TB * F;
    bool miss = false;
    for (int e = tid; e < total; e += TB) {
      const int r = e / F;
      const int f = e - r * F;
      const int row = row0 + r;
      float x = 0.f;
      bool b = false;
      if (row < a.n_rows) {
        x = a.X[(size_t)row * a.ldx + f];
        if (a.prep) x = prep_value(x, a.prep[f], &b);
        miss = miss || (x != x);
      }
      feat[f * TB + r] = x;
      if (b) bad[r] = 1;
    }
    if (__any(miss) && (tid & 63) == 0) *any_missing = 1;
  }
  PF_STORE(tbuf0, n16)
  __syncthreads();

  const int row = row0 + tid;
  bool row_ok = bad[tid] == 0;
  if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
  const bool missing = *any_missing != 0;
  if (GENERAL) {
    for (int c = 0; c < a.C; ++c) accl[c * TB + tid] = 0.f;
  }
  float acc = 0.f;
  bool poisoned = false;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);

  int c = 0;
  for (int t0 = tb; t0 < te; t0 += a.chunk_trees, ++c) {
    const int nt = min(a.chunk_trees, te - t0);
    const uint32_t* cur = (c & 1) ? tbuf1 : tbuf0;
    uint32_t* nxt = (c & 1) ? tbuf0 : tbuf1;
    const int t1 = t0 + a.chunk_trees;
    n16 = (t1 < te) ? (min(a.chunk_trees, te - t1) * rw) >> 2 : 0;
    PF_LOAD(n16 > 0 ? a.blob + (size_t)t1 * rw : a.blob, n16)  // never form an OOB address
    if (missing) {
      traverse_chunk<DEPTH, GENERAL, true, ILP>(a, cur, nt, t0, feat_lane, acc, accl, poisoned);
    } else {
      traverse_chunk<DEPTH, GENERAL, false, ILP>(a, cur, nt, t0, feat_lane, acc, accl, poisoned);
    }
    // `nxt` was last read in the previous iteration, before that iteration's barrier
    PF_STORE(nxt, n16)
    __syncthreads();
  }
  finish_row(a, acc, accl, split, GENERAL, row, row_ok && !poisoned);
}

// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// Wide kernel (v4): one 1024-thread workgroup (16 waves) per ROWS-row tile, tree-group parallel.
// Half-wave hw = 2*wave + (lane >= 32) owns row set hw % RS (32 rows, RS = ROWS/32) and tree
// group g = hw / RS (G = 32/RS groups: 4 / 8 / 16 for ROWS = 256 / 128 / 64). Each 32-lane LDS
// access group reads 32 distinct rows of one feature plane (conflict free); both halves of a wave
// walk the same trees (g is wave-uniform). Group g takes trees k ≡ g (mod G) of every chunk; the
// G partial results of a row are combined in fixed order (deterministic).
//  * ROWS shrinks as the staged feature count grows (<= 64 / 128 / 256 columns): the feature
//    planes stay <= 64 KiB and 16 waves stay resident; beyond that the POINTER layout takes over;
//  * feature planes are [F][ROWS]: a traversal read by 32 consecutive rows hits bank r mod 32
//    whatever feature each lane's node tests (measured: a +1 pad per plane made that bank
//    (f + r) mod 32 and cost 35 % extra LDS cycles, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
//    The staging store keeps the same property: each 32-lane group writes 32 consecutive rows
//    of one feature (its global reads are row-strided; staging is once per tile, traversal once
//    per tree and level);
//  * `feat_map` stages only the columns the trees use (compaction of wide records);
//  * accumulation modes: SUM (regression / binary chain), SLOT (multi-class GBDT: each tree adds
//    its leaf to one class slot — wave-uniform, contiguous runs), CLASS (majority vote: the leaf is
//    a class index, the tree adds its weight to that class), VOTE8 (unweighted vote with <= 4
//    classes: the leaf is a packed increment `1 << 8*class`, one integer add per tree).
enum : int { MODE_SUM = 0, MODE_SLOT = 1, MODE_CLASS = 2, MODE_VOTE8 = 3 };
constexpr int WIDE_T = 1024;
constexpr int DYN_B = 8;       // MODE_SUM: trees per dynamically claimed batch
constexpr int DYN_SLOTS = 16;  // MODE_SUM: per-chunk batch slots (chunk <= DYN_B * DYN_SLOTS trees)
constexpr int CMAX = 8;  // class slots of the multi-class wide modes

template <int ROWS>
struct WideGeom {
  static constexpr int RS = ROWS / 32;  // row sets
  static constexpr int G = 32 / RS;     // tree groups
  static constexpr int PS = ROWS;       // feature plane stride (floats)
};

#define PF4_DECL uint4 pq0, pq1, pq2, pq3;
#define PF4_LOAD(SRC, N16, T)                                                          \
  {                                                                                    \
    const uint4* s4_ = reinterpret_cast<const uint4*>(SRC);                            \
    const int last_ = (N16) > 0 ? (N16) - 1 : 0;                                      \
    pq0 = s4_[min((int)threadIdx.x + 0 * (T), last_)];                                 \
    pq1 = s4_[min((int)threadIdx.x + 1 * (T), last_)];                                 \
    pq2 = s4_[min((int)threadIdx.x + 2 * (T), last_)];                                 \
    pq3 = s4_[min((int)threadIdx.x + 3 * (T), last_)];                                 \
  }
#define PF4_STORE(DST, N16, T)                                                         \
  {                                                                                    \
    uint4* d4_ = reinterpret_cast<uint4*>(DST);                                        \
    const int i0_ = (int)threadIdx.x;                                                  \
    if (i0_ < (N16)) d4_[i0_] = pq0;                                                   \
    if (i0_ + (T) < (N16)) d4_[i0_ + (T)] = pq1;                                       \
    if (i0_ + 2 * (T) < (N16)) d4_[i0_ + 2 * (T)] = pq2;                               \
    if (i0_ + 3 * (T) < (N16)) d4_[i0_ + 3 * (T)] = pq3;                               \
  }

__host__ __device__ constexpr int perfect_rec_words(int depth, int P) {
  return ((2 * ((1 << depth) - 1) + (1 << depth) * P + ((1 << depth) - 1 + 31) / 32) + 3) & ~3;
}
// fp8-leaf record: nodes + default-right words only (leaf pairs live in the last-level metas)
__host__ __device__ constexpr int perfect_rec_words8(int depth) {
  return ((2 * ((1 << depth) - 1) + ((1 << depth) - 1 + 31) / 32) + 3) & ~3;
}

// OCP e4m3 leaf pair in bits [31:16] of a last-level node's meta -> (left, right) as fp32
// VOTE8 forests with class codes (VC): bits [23:16] / [31:24] of a last-level meta are the left /
// right leaf's class index; the walk returns the packed-vote increment 1 << 8*class (as float bits)
template <bool VC>
__device__ __forceinline__ float leaf_pair_select(uint32_t meta, bool right) {
  if constexpr (VC) return __uint_as_float(1u << (8u * ((meta >> (right ? 24 : 16)) & 3u)));
  const auto pr = __builtin_amdgcn_cvt_pk_f32_fp8((int)meta, true);
  return right ? pr[1] : pr[0];
}

// Per-thread accumulator of one accumulation mode. `t` is the (wave-uniform) global tree index.
template <int MODE>
struct WAcc;
template <>
struct WAcc<MODE_SUM> {
  float s = 0.f;
  __device__ __forceinline__ void add(const TreeArgs&, int, float v) { s += v; }
  __device__ __forceinline__ void poison() { s = __builtin_nanf(""); }  // NaN sum -> EmptyScore
  __device__ __forceinline__ bool poisoned() const { return false; }
  __device__ __forceinline__ void finish() {}
};
template <>
struct WAcc<MODE_VOTE8> {
  uint32_t packed = 0u;
  bool pz = false;
  __device__ __forceinline__ void add(const TreeArgs&, int, float v) { packed += __float_as_uint(v); }
  __device__ __forceinline__ void poison() { pz = true; }
  __device__ __forceinline__ bool poisoned() const { return pz; }
  __device__ __forceinline__ void finish() {}
};
template <>
struct WAcc<MODE_CLASS> {
  float c[CMAX];
  bool pz = false;
  __device__ __forceinline__ WAcc() {
#pragma unroll
    for (int k = 0; k < CMAX; ++k) c[k] = 0.f;
  }
  __device__ __forceinline__ void add(const TreeArgs& a, int t, float v) {
    const float w = a.tree_w ? a.tree_w[t] : 1.f;
#pragma unroll
    for (int k = 0; k < CMAX; ++k) c[k] += (v == (float)k) ? w : 0.f;
    pz = pz || (v != v);  // a leaf without a class: the segment's prediction is missing
  }
  __device__ __forceinline__ void poison() { pz = true; }
  __device__ __forceinline__ bool poisoned() const { return pz; }
  __device__ __forceinline__ void finish() {}
};
template <>
struct WAcc<MODE_SLOT> {
  float c[CMAX];
  float run = 0.f;
  int cur = 0;
  bool pz = false;
  __device__ __forceinline__ WAcc() {
#pragma unroll
    for (int k = 0; k < CMAX; ++k) c[k] = 0.f;
  }
  __device__ __forceinline__ void flush() {
#pragma unroll
    for (int k = 0; k < CMAX; ++k) c[k] += (k == cur) ? run : 0.f;
    run = 0.f;
  }
  __device__ __forceinline__ void add(const TreeArgs& a, int t, float v) {
    const int sl = __builtin_amdgcn_readfirstlane(a.tree_slot[t]);  // runs of equal slots
    if (sl != cur) {
      flush();
      cur = sl;
    }
    run += v;
  }
  __device__ __forceinline__ void poison() { pz = true; }
  __device__ __forceinline__ bool poisoned() const { return pz; }
  __device__ __forceinline__ void finish() { flush(); }
};

// Missing-aware walk of one tree record (per-node default-direction bits): the leaf value, or
// NaN when the tree's prediction is null (a visited split saw a missing value and the tree is
// flagged null-on-missing).
template <int DEPTH, bool LEAF8, bool VC = false>
__device__ __forceinline__ float walk_missing(const TreeArgs& a, const char* base, const char* feat_lane,
                                              bool& null_pred) {
  constexpr int NI = (1 << DEPTH) - 1;
  constexpr int NL = 1 << DEPTH;
  const int dr_off = LEAF8 ? 2 * NI : 2 * NI + NL;
  uint32_t j = 1u, pz = 0u;
  float lf = 0.f;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const uint2 nd = *reinterpret_cast<const uint2*>(base - 8 + (j << 3));
    const uint32_t fo = (LEAF8 && d == DEPTH - 1) ? (nd.y & 0xFFFFu) : nd.y;
    const float x = *reinterpret_cast<const float*>(feat_lane + fo);
    uint32_t right = (x >= __uint_as_float(nd.x)) ? 1u : 0u;
    const uint32_t n = j - 1u;
    const uint32_t w = reinterpret_cast<const uint32_t*>(base)[dr_off + (n >> 5)];
    const uint32_t isn = (x != x) ? 1u : 0u;
    right |= isn & (w >> (n & 31u));
    pz |= isn;
    if (LEAF8 && d == DEPTH - 1) {
      lf = leaf_pair_select<VC>(nd.y, right != 0u);
    } else {
      j = j + j + right;
    }
  }
  null_pred = pz && null_flag<DEPTH>(base, dr_off);
  return LEAF8 ? lf : (reinterpret_cast<const float*>(base + NI * 8) - NL)[j];
}

// Missing-aware traversal of group g's trees of one chunk.
template <int DEPTH, int ILP, int G, bool LEAF8, int MODE>
__device__ __forceinline__ void traverse_chunk_g(const TreeArgs& a, const uint32_t* buf, int nt, int g, int t0,
                                                 const char* feat_lane, WAcc<MODE>& acc) {
  const int rw = a.rec_words;
  const int mt = (nt - g + G - 1) / G;
  for (int m = 0; m < mt; ++m) {
    bool nul;
    const float v = walk_missing<DEPTH, LEAF8, LEAF8 && MODE == MODE_VOTE8>(
        a, reinterpret_cast<const char*>(buf + (g + G * m) * rw), feat_lane, nul);
    if (nul) acc.poison();
    else acc.add(a, t0 + g + G * m, v);
  }
}

// Fast path (tile without missing values, or missing values routed by the NaN plane), written
// against explicit LDS byte addresses so the per-level work is: node ds_read_b64, feature address
// add, feature ds_read_b32, v_cmp, v_cndmask, v_lshl_add.
//  * u = LDS address of the current node of tree i minus i*TS (TS = compile-time tree stride of a
//    tree group, folded into the ds_read immediate offset); children: u' = 2u + (8 - b0) + 8r.
//  * last level, fp32 leaves: the two leaves under a node are adjacent, so the leaf PAIR (one
//    ds_read_b64 at u + C, C folded into the offset) is fetched together with the feature and the
//    final compare only selects between them;
//  * last level, fp8 leaves: the pair is already in the node's meta word (no leaf read at all).
// `__asm__("" : "+v"(...))` pins values in VGPRs so the compiler cannot re-derive them.
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const u32x2_t lds_u2_t;
typedef __attribute__((address_space(3))) const float lds_f_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}
__device__ __forceinline__ uint2 lds_ld2(uint32_t a) {
  const u32x2_t v = *(lds_u2_t*)(uintptr_t)a;
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ float lds_ldf(uint32_t a) { return *(lds_f_t*)(uintptr_t)a; }
// s_waitcnt lgkmcnt(0) between scheduling barriers: the traversal's issue slots are its bound
// (every instruction of a wave, s_waitcnt and s_nop included, takes one), so a phase of N
// independent LDS reads is drained by ONE wait rather than one lgkmcnt(k) per consumer.
__device__ __forceinline__ void lds_wait_all() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
}

// N trees of group g starting at its m-th tree, N independent walks interleaved (ILP).
template <int DEPTH, int N, int G, bool LEAF8, bool VC = false>
__device__ __forceinline__ void fast_batch(uint32_t lds0, int g, int m, uint32_t feat_lane, float (&v)[N]) {
  constexpr int NI = (1 << DEPTH) - 1;
  constexpr int NL = 1 << DEPTH;
  constexpr uint32_t RB = 4u * (LEAF8 ? perfect_rec_words8(DEPTH) : perfect_rec_words(DEPTH, 1));  // record bytes
  constexpr uint32_t TS = G * RB;                            // tree stride within a group
  constexpr uint32_t C = 8u + 8u * NI - 4u * NL;             // last-level node -> its leaf pair
  const uint32_t b0 = lds0 + (uint32_t)(g + G * m) * RB;
  uint32_t k0 = 8u - b0, k1 = 16u - b0;
  __asm__("" : "+v"(k0), "+v"(k1));
  uint32_t u[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    u[i] = b0;
    __asm__ volatile("" : "+v"(u[i]));  // separate root reads: ds_read2_b64 pairing costs 8 LDS
                                        // cycles vs 2 x 2 for two ds_read_b64
  }
  // Each level in three phases — N node reads, N feature reads, N child updates — with scheduling
  // barriers between them, so the N walks stay interleaved (the scheduler otherwise may serialise
  // them tree by tree, one LDS round trip at a time: it did so for the fp8-leaf variant).
#pragma unroll
  for (int d = 0; d + 1 < DEPTH; ++d) {
    uint2 nd[N];
#pragma unroll
    for (int i = 0; i < N; ++i) nd[i] = lds_ld2(u[i] + i * TS);
    lds_wait_all();  // one wait for the N node reads instead of one per consumer
    float x[N];
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = lds_ldf(feat_lane + nd[i].y);
    lds_wait_all();
    // compares into N separate lane masks (v_cmp_e64 -> SGPR pairs), then the child updates: no
    // VCC reuse, so no hazard s_nop between a compare and the select that reads it
    uint64_t r[N];
#pragma unroll
    for (int i = 0; i < N; ++i) r[i] = __builtin_amdgcn_ballot_w64(x[i] >= __uint_as_float(nd[i].x));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      u[i] = 2u * u[i] + (__builtin_amdgcn_inverse_ballot_w64(r[i]) ? k1 : k0);
      __asm__("" : "+v"(u[i]));
    }
  }
  uint2 nd[N], lv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    nd[i] = lds_ld2(u[i] + i * TS);
    if (!LEAF8) {
      uint32_t ul = u[i] + C;
      __asm__ volatile("" : "+v"(ul));  // keep the pair read out of a ds_read2_b64 with the node
      lv[i] = lds_ld2(ul + i * TS);
    }
  }
  lds_wait_all();
  float x[N];
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = lds_ldf(feat_lane + (LEAF8 ? (nd[i].y & 0xFFFFu) : nd[i].y));
  lds_wait_all();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (LEAF8) {
      v[i] = leaf_pair_select<VC>(nd[i].y, x[i] >= __uint_as_float(nd[i].x));
    } else {
      v[i] = (x[i] >= __uint_as_float(nd[i].x)) ? __uint_as_float(lv[i].y) : __uint_as_float(lv[i].x);
    }
  }
}

template <int DEPTH, int N, int G, bool LEAF8, int MODE>
__device__ __forceinline__ void fast_batch_acc(const TreeArgs& a, uint32_t lds0, int g, int m, int t0,
                                               uint32_t feat_lane, WAcc<MODE>& acc) {
  float v[N];
  fast_batch<DEPTH, N, G, LEAF8, LEAF8 && MODE == MODE_VOTE8>(lds0, g, m, feat_lane, v);
#pragma unroll
  for (int i = 0; i < N; ++i) acc.add(a, t0 + g + G * (m + i), v[i]);
}

// The group's trees in ILP-wide batches; the remainder in 4/2/1-wide batches (a plain serial
// tail is latency bound: one dependent LDS round trip per level and tree).
template <int DEPTH, int ILP, int G, bool LEAF8, int MODE>
__device__ __forceinline__ void traverse_fast_g(const TreeArgs& a, const uint32_t* buf, int nt, int g, int t0,
                                                uint32_t feat_lane, WAcc<MODE>& acc) {
  const uint32_t lds0 = lds_addr(buf);
  const int mt = (nt - g + G - 1) / G;
  int m = 0;
  for (; m + ILP <= mt; m += ILP) fast_batch_acc<DEPTH, ILP, G, LEAF8, MODE>(a, lds0, g, m, t0, feat_lane, acc);
  if (ILP > 8 && m + 8 <= mt) {
    fast_batch_acc<DEPTH, 8, G, LEAF8, MODE>(a, lds0, g, m, t0, feat_lane, acc);
    m += 8;
  }
  if (ILP > 4 && m + 4 <= mt) {
    fast_batch_acc<DEPTH, 4, G, LEAF8, MODE>(a, lds0, g, m, t0, feat_lane, acc);
    m += 4;
  }
  if (m + 2 <= mt) {
    fast_batch_acc<DEPTH, 2, G, LEAF8, MODE>(a, lds0, g, m, t0, feat_lane, acc);
    m += 2;
  }
  if (m < mt) fast_batch_acc<DEPTH, 1, G, LEAF8, MODE>(a, lds0, g, m, t0, feat_lane, acc);
}

// The wide kernel's work on one ROWS-row tile starting at row0 of a (tree split `split`).
// out_row (nullable): the epilogue writes row r's outputs at out_row[r] instead of r (the grouped
// mixed-model launch scatters its model-contiguous rows back to arrival order, grouped.hip).
template <int DEPTH, int ILP, int ROWS, bool LEAF8, int MODE>
__device__ __forceinline__ void wide_tile(const TreeArgs& a, const int row0, const int split,
                                          const int* __restrict__ out_row, const bool prof_on) {
  using WG = WideGeom<ROWS>;
  constexpr int G = WG::G, RS = WG::RS, PS = WG::PS, T = WIDE_T;
  extern __shared__ __align__(16) uint32_t smem[];
  const int rw = a.rec_words;
  // LDS: [bad ROWS][flag 4][claim counters 2 x 4][part P x ROWS][feature plane(s) F x PS][two chunk
  // buffers], P = max(G, DYN_SLOTS) for MODE_SUM, else G. A tile with missing values and a NaN
  // blob gets two planes (the second NaN -> +inf) and that blob's chunk size; any other tile one
  // plane and the main blob — chosen per workgroup.
  // dynamic batches (MODE_SUM, 256-row tiles: 4 waves per row-set pair; with 8 or 16 waves per
  // pair a chunk has too few batches to keep them busy — measured 6 % slower at 128 rows)
  constexpr bool DYN = MODE == MODE_SUM && ROWS == 256;
  constexpr int NPART = DYN ? DYN_SLOTS : G;
  int* bad = reinterpret_cast<int*>(smem);
  int* any_missing = bad + ROWS;
  int* claim = bad + ROWS + 4;                              // [2][4] per rowset pair, per chunk parity
  float* part = reinterpret_cast<float*>(claim + 8);        // [NPART][ROWS]
  float* feat = part + NPART * ROWS;
  const int F = a.n_stage;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int hw = (tid >> 6) * 2 + (lane >> 5);
  const int r_local = 32 * (hw % RS) + (lane & 31);
  const int g = __builtin_amdgcn_readfirstlane(hw / RS);  // both halves of a wave: same group
  const int tb = split * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);

  // optional per-wave phase timers of one workgroup (kbench --tree-prof): staging, traversal,
  // chunk store + barrier, total
  const unsigned long long tstart = prof_on ? __builtin_amdgcn_s_memtime() : 0ull;
  PF4_DECL
  int n16 = (tb < te) ? (min(a.chunk_trees, te - tb) * rw) >> 2 : 0;
  PF4_LOAD(n16 > 0 ? a.blob + (size_t)tb * rw : a.blob, n16, T)  // speculative: main blob

  if (tid == 0) *any_missing = 0;
  if (tid < ROWS) bad[tid] = 0;
  if (tid < 8) claim[tid] = 0;
  if constexpr (DYN) {
    for (int e = tid; e < NPART * ROWS; e += T) part[e] = 0.f;
  }
  __syncthreads();
  {
    bool miss = false;
    // identity column map, 16-byte aligned rows: each lane loads 4 consecutive columns of its row
    // (one 16-byte load instead of four 4-byte ones — the per-lane row stride makes every lane of
    // a load touch its own cache line) and stores them to 4 planes (still 32 consecutive rows per
    // store: conflict-free)
    const bool vec4 = a.feat_map == nullptr && (a.ldx & 3) == 0 && (reinterpret_cast<uintptr_t>(a.X) & 15) == 0;
    const int F4 = (F + 3) >> 2;
    for (int e = tid; vec4 && e < ROWS * F4; e += T) {
      const int q = e >> 5;
      const int rh = q / F4;
      const int fq = q - rh * F4;
      const int r = 32 * rh + (e & 31);
      const int row = row0 + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < a.n_rows) v = *reinterpret_cast<const float4*>(a.X + (size_t)row * a.ldx + 4 * fq);
      const float vv[4] = {v.x, v.y, v.z, v.w};
      bool b = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int f = 4 * fq + k;
        if (f < F) {
          float x = vv[k];
          if (row < a.n_rows) {
            if (a.prep) x = prep_value(x, a.prep[f], &b);
            miss = miss || (x != x);
          }
          feat[f * PS + r] = x;
        }
      }
      if (b) bad[r] = 1;
    }
    const int total = vec4 ? 0 : ROWS * F;
    for (int e = tid; e < total; e += T) {
      // item e: row (e & 31) + 32 * ((e >> 5) / F) of feature (e >> 5) % F — the 32 lanes of a
      // group store 32 consecutive rows of one plane (distinct banks)
      const int q = e >> 5;
      const int rh = q / F;
      const int f = q - rh * F;
      const int r = 32 * rh + (e & 31);
      const int row = row0 + r;
      float x = 0.f;
      bool b = false;
      if (row < a.n_rows) {
        const int col = a.feat_map ? a.feat_map[f] : f;
        x = a.X[(size_t)row * a.ldx + col];
        if (a.prep) x = prep_value(x, a.prep[col], &b);
        miss = miss || (x != x);
      }
      feat[f * PS + r] = x;
      if (b) bad[r] = 1;
    }
    if (__any(miss) && lane == 0) *any_missing = 1;
  }
  __syncthreads();
  const bool has_missing = *any_missing != 0;
  const bool use_nan = has_missing && a.blob_nan != nullptr;
  const uint32_t* blob = use_nan ? a.blob_nan : a.blob;
  const int chunk = use_nan ? a.chunk_trees_nan : a.chunk_trees;
  uint32_t* tbuf0 = reinterpret_cast<uint32_t*>(feat + (use_nan ? 2 : 1) * F * PS);
  uint32_t* tbuf1 = tbuf0 + chunk * rw;
  if (use_nan) {
    const int total = PS * F;
    for (int e = tid; e < total; e += T) {  // NaN-goes-right plane (pads copied along)
      const float x = feat[e];
      feat[total + e] = (x != x) ? __builtin_inff() : x;
    }
    n16 = (tb < te) ? (min(chunk, te - tb) * rw) >> 2 : 0;
    PF4_LOAD(n16 > 0 ? blob + (size_t)tb * rw : blob, n16, T)
  }
  PF4_STORE(tbuf0, n16, T)
  __syncthreads();

  // VAR_NAN_FAST: missing values need no per-node work — either no node sends NaN right (a NaN
  // compare is false: left), or the node's feature offset points into the NaN -> +inf plane
  const bool missing = has_missing && (a.variant & VAR_NAN_FAST) == 0;
  WAcc<MODE> acc;
  const char* feat_lane = reinterpret_cast<const char*>(feat + r_local);
  unsigned long long tp0 = 0, tp1 = 0, tp2 = 0, tq = 0;
  if (prof_on) tq = __builtin_amdgcn_s_memtime(), tp0 = tq - tstart;
  int c = 0;
  for (int t0 = tb; t0 < te; t0 += chunk, ++c) {
    const int nt = min(chunk, te - t0);
    const uint32_t* cur = (c & 1) ? tbuf1 : tbuf0;
    uint32_t* nxt = (c & 1) ? tbuf0 : tbuf1;
    const int t1 = t0 + chunk;
    n16 = (t1 < te) ? (min(chunk, te - t1) * rw) >> 2 : 0;
    PF4_LOAD(n16 > 0 ? blob + (size_t)t1 * rw : blob, n16, T)
    if constexpr (DYN) {
      // Dynamic batches. The waves that share a row-set pair (one per tree group, all on one
      // SIMD) claim DYN_B-tree batches of the chunk from an LDS counter instead of walking a fixed
      // share each: the SIMD's issue arbitration favours older waves, so with a static split the
      // youngest wave's trees were the critical path and the others idled at the chunk barrier
      // (profiles/r2_tree_variants.md). A batch's sum (its trees added in order, from 0) goes to
      // its slot, which only its claimer touches in this chunk and which accumulates over chunks
      // in chunk order: the row sum (slots added in slot order) is deterministic whichever wave
      // walked a batch, and the same on the per-node missing path and the fast paths. Slots are
      // indexed by the batch's position in the split (mod DYN_SLOTS, chunks are whole batches),
      // so the NaN blob's smaller chunks group the trees exactly as the main blob's.
      int* ctr = claim + (c & 1) * 4 + ((tid >> 6) % (RS / 2 > 0 ? RS / 2 : 1));
      if (tid < 4) claim[((c + 1) & 1) * 4 + tid] = 0;  // next chunk's counters (free since the last barrier)
      const uint32_t lds0 = lds_addr(cur);
      const uint32_t fl = lds_addr(feat + r_local);
      const int nb = (nt + DYN_B - 1) / DYN_B;
      for (;;) {
        int b = 0;
        if (lane == 0) b = atomicAdd(ctr, 1);
        b = __builtin_amdgcn_readfirstlane(b);
        if (b >= nb) break;
        const int m = b * DYN_B;
        float sum = 0.f;
        if (missing) {
          const int me = min(m + DYN_B, nt);
          for (int t = m; t < me; ++t) {
            bool nul;
            const float v = walk_missing<DEPTH, LEAF8>(a, reinterpret_cast<const char*>(cur + t * rw), feat_lane, nul);
            sum += nul ? __builtin_nanf("") : v;
          }
        } else if (m + DYN_B <= nt) {
          float v[DYN_B];
          fast_batch<DEPTH, DYN_B, 1, LEAF8>(lds0, 0, m, fl, v);
#pragma unroll
          for (int i = 0; i < DYN_B; ++i) sum += v[i];
        } else {
          int mm = m;
          if (mm + 4 <= nt) {
            float v[4];
            fast_batch<DEPTH, 4, 1, LEAF8>(lds0, 0, mm, fl, v);
#pragma unroll
            for (int i = 0; i < 4; ++i) sum += v[i];
            mm += 4;
          }
          if (mm + 2 <= nt) {
            float v[2];
            fast_batch<DEPTH, 2, 1, LEAF8>(lds0, 0, mm, fl, v);
            sum += v[0];
            sum += v[1];
            mm += 2;
          }
          if (mm < nt) {
            float v[1];
            fast_batch<DEPTH, 1, 1, LEAF8>(lds0, 0, mm, fl, v);
            sum += v[0];
          }
        }
        part[(((t0 - tb) / DYN_B + b) % DYN_SLOTS) * ROWS + r_local] += sum;
      }
    } else if (missing) {
      traverse_chunk_g<DEPTH, ILP, G, LEAF8, MODE>(a, cur, nt, g, t0, feat_lane, acc);
    } else {
      traverse_fast_g<DEPTH, ILP, G, LEAF8, MODE>(a, cur, nt, g, t0, lds_addr(feat + r_local), acc);
    }
    unsigned long long tm = 0;
    if (prof_on) tm = __builtin_amdgcn_s_memtime(), tp1 += tm - tq;
    PF4_STORE(nxt, n16, T)
    __syncthreads();
    if (prof_on) tq = __builtin_amdgcn_s_memtime(), tp2 += tq - tm;
  }
  acc.finish();
  if (prof_on && lane == 0) {
    unsigned long long* pw = a.prof + (tid >> 6) * 4;
    pw[0] = tp0;
    pw[1] = tp1;
    pw[2] = tp2;
    pw[3] = __builtin_amdgcn_s_memtime() - tstart;
  }
  if (acc.poisoned()) bad[r_local] = 1;  // a null tree invalidates a multi-class row
  const int row = row0 + r_local;
  if constexpr (MODE == MODE_SUM) {
    if constexpr (!DYN) {
      part[g * ROWS + r_local] = acc.s;
      __syncthreads();
    }  // DYN: the batch slots are complete since the last chunk barrier
    if (g == 0) {
      float sum = part[r_local];
#pragma unroll
      for (int q = 1; q < NPART; ++q) sum += part[q * ROWS + r_local];
      bool row_ok = bad[r_local] == 0;
      if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
      if (row < a.n_rows) {
        if (a.partial) {
          const size_t stride = (size_t)a.n_rows;
          float* pbase = a.partial + (size_t)split * 2 * stride;
          pbase[row] = sum;
          pbase[stride + row] = row_ok ? 0.f : 1.f;
        } else {
          const int orow = out_row ? out_row[row] : row;
          apply_epilogue(a.epi, [&](int) { return sum; }, row_ok, orow, a.n_rows, a.score, a.valid, a.probs);
        }
      }
    }
  } else {
    float tot[CMAX];
#pragma unroll
    for (int k = 0; k < CMAX; ++k) tot[k] = 0.f;
    if constexpr (MODE == MODE_VOTE8) {
      reinterpret_cast<uint32_t*>(part)[g * ROWS + r_local] = acc.packed;
      __syncthreads();
      if (g == 0) {
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const uint32_t pk = reinterpret_cast<const uint32_t*>(part)[q * ROWS + r_local];
#pragma unroll
          for (int k = 0; k < 4; ++k) tot[k] += (float)((pk >> (8 * k)) & 0xFFu);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < CMAX; ++k) {
        if (k < a.C) {  // uniform
          part[g * ROWS + r_local] = acc.c[k];
          __syncthreads();
          if (g == 0) {
#pragma unroll
            for (int q = 0; q < G; ++q) tot[k] += part[q * ROWS + r_local];
          }
          __syncthreads();
        }
      }
    }
    if (g == 0 && row < a.n_rows) {
      if (a.acc_init) {
#pragma unroll
        for (int k = 0; k < CMAX; ++k)
          if (k < a.C) tot[k] += a.acc_init[k];
      }
      bool row_ok = bad[r_local] == 0;
      if (a.row_valid_in) row_ok = row_ok && a.row_valid_in[row];
      auto sel = [&](int cls) {
        float r = tot[0];
#pragma unroll
        for (int k = 1; k < CMAX; ++k) r = (cls == k) ? tot[k] : r;
        return r;
      };
      apply_epilogue(a.epi, sel, row_ok, out_row ? out_row[row] : row, a.n_rows, a.score, a.valid, a.probs);
    }
  }
}

template <int DEPTH, int ILP, int ROWS, bool LEAF8, int MODE>
__global__ __launch_bounds__(WIDE_T, 1) void tree_perfect_wide_kernel(TreeArgs a) {
  const bool prof_on = a.prof != nullptr && blockIdx.x == gridDim.x / 2 && blockIdx.y == 0;
  wide_tile<DEPTH, ILP, ROWS, LEAF8, MODE>(a, blockIdx.x * ROWS, blockIdx.y, nullptr, prof_on);
}

// ONE launch over the model-contiguous rows of a mixed-model slice (runtime/grouped.py): the
// entries' tiles are numbered model after model (tile_start, computed on the device by
// grouped.hip::group_count_kernel), workgroup L takes tile tile_start[0] + L, finds its entry by
// binary search, and runs that model's wide tile with its own forest, prepare and epilogue; the
// epilogue scatters each row back to arrival order (perm). Workgroups past the slice's last tile
// (the grid is sized from the row count before the counts exist) exit at once.
template <int DEPTH, int ILP, int ROWS, bool LEAF8, int MODE>
__global__ __launch_bounds__(WIDE_T, 1) void tree_grouped_wide_kernel(GroupedTreeArgs ga) {
  const int t = ga.tile_start[0] + (int)blockIdx.x;
  if (t >= ga.tile_start[ga.n_models]) return;
  int lo = 0, hi = ga.n_models - 1;  // the last entry whose first tile is <= t (empty ones skipped)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ga.tile_start[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int e = __builtin_amdgcn_readfirstlane(lo);
  TreeArgs a = ga.models[e];
  const int code = ga.model_code[e];
  const int rs = ga.row_start[code];
  a.X = ga.Xg + (size_t)rs * ga.F;
  a.ldx = ga.F;
  a.n_feat = ga.F;
  a.n_rows = ga.row_start[code + 1] - rs;
  a.score = ga.out_s;
  a.valid = ga.out_v;
  a.row_valid_in = nullptr;
  a.partial = nullptr;
  a.prof = nullptr;
  a.trees_per_split = a.n_trees;
  wide_tile<DEPTH, ILP, ROWS, LEAF8, MODE>(a, (t - ga.tile_start[e]) * ROWS, 0, ga.perm + rs, false);
}

template <typename K>
int prepare_launch(K kernel, size_t lds) {
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

template <int D, int ROWS, bool LEAF8, int MODE>
int launch_wide(hipStream_t st, const TreeArgs& a, size_t lds_w) {
  using WG = WideGeom<ROWS>;
  dim3 grid((a.n_rows + ROWS - 1) / ROWS, (a.n_trees + a.trees_per_split - 1) / a.trees_per_split);
  (void)WG::G;
  // 8 independent tree walks per batch (measured: 16 was 1.42x slower at depth 6, 1000 trees —
  // profiles/r2_tree_kernel.md)
  auto k = tree_perfect_wide_kernel<D, 8, ROWS, LEAF8, MODE>;
  int err = prepare_launch(k, lds_w);
  if (!err) hipLaunchKernelGGL(k, grid, dim3(WIDE_T), lds_w, st, a);
  return err;
}

// Validation + dynamic LDS bytes of one wide-kernel launch (0 or a negative error code).
template <int D>
int wide_check(const TreeArgs& a, size_t& lds_w) {
  const bool leaf8 = (a.variant & 3) == 2;
  const int rows = a.rows_wide;
  if (!(rows == 256 || rows == 128 || rows == 64)) return -12;
  const int G = WIDE_T / rows;
  const bool dyn = a.mode == MODE_SUM && rows == 256;  // kernel's DYN / NPART
  const int npart = dyn ? DYN_SLOTS : G;
  const size_t head = (size_t)(rows + 4 + 8) * 4 + (size_t)npart * rows * 4;
  if (dyn && (a.chunk_trees > DYN_B * DYN_SLOTS || (a.blob_nan && a.chunk_trees_nan > DYN_B * DYN_SLOTS)))
    return -14;  // more batches per chunk than slots
  const size_t plane = (size_t)a.n_stage * rows * 4;
  lds_w = head + plane + 2 * (size_t)a.chunk_trees * a.rec_words * 4;
  if ((size_t)a.chunk_trees * a.rec_words > (size_t)WIDE_T * 4 * 4) return -9;
  if (a.blob_nan) {
    if (a.chunk_trees_nan < 1 || (size_t)a.chunk_trees_nan * a.rec_words > (size_t)WIDE_T * 4 * 4) return -9;
    lds_w = max(lds_w, head + 2 * plane + 2 * (size_t)a.chunk_trees_nan * a.rec_words * 4);
  }
  if (lds_w > 160 * 1024) return -5;
  if (a.P != 1 || a.rec_words != (leaf8 ? perfect_rec_words8(D) : perfect_rec_words(D, 1))) return -10;
  if (a.mode != MODE_SUM && (a.partial || a.C > CMAX || (a.mode == MODE_VOTE8 && a.C > 4) ||
                             (leaf8 && a.mode != MODE_VOTE8)))
    return -11;  // leaf pairs in the metas: fp8 sums or VOTE8 class codes
  if (a.mode == MODE_SLOT && !a.tree_slot) return -11;
  return 0;
}

// Grouped launch: `a` is a representative entry (kernel selection), lds the largest entry's need.
template <int D>
int launch_grouped(hipStream_t st, const TreeArgs& a, const GroupedTreeArgs& g, int tiles, size_t lds) {
  const bool leaf8 = (a.variant & 3) == 2;
#define PMML_GROUPED(R, L8, M)                                                       \
  {                                                                                  \
    auto k = tree_grouped_wide_kernel<D, 8, R, L8, M>;                               \
    int err = prepare_launch(k, lds);                                                \
    if (!err) hipLaunchKernelGGL(k, dim3(tiles), dim3(WIDE_T), lds, st, g);          \
    return err;                                                                      \
  }
#define PMML_GROUPED_ROWS(R)                                                         \
  if (a.rows_wide == R) {                                                            \
    switch (a.mode) {                                                                \
      case MODE_SUM:                                                                 \
        if (leaf8) PMML_GROUPED(R, true, MODE_SUM) else PMML_GROUPED(R, false, MODE_SUM)       \
      case MODE_SLOT: PMML_GROUPED(R, false, MODE_SLOT)                              \
      case MODE_CLASS: PMML_GROUPED(R, false, MODE_CLASS)                            \
      case MODE_VOTE8:                                                               \
        if (leaf8) PMML_GROUPED(R, true, MODE_VOTE8) else PMML_GROUPED(R, false, MODE_VOTE8)   \
      default: return -11;                                                           \
    }                                                                                \
  }
  PMML_GROUPED_ROWS(256)
  PMML_GROUPED_ROWS(128)
  PMML_GROUPED_ROWS(64)
#undef PMML_GROUPED_ROWS
#undef PMML_GROUPED
  return -12;
}

template <int D>
int launch_perfect(hipStream_t st, const TreeArgs& a, dim3 grid, size_t lds) {
  int err = 0;
  const int base = a.variant & 3;
  if (base == 1 || base == 2) {
    const bool leaf8 = base == 2;
    const int rows = a.rows_wide;
    size_t lds_w = 0;
    const int chk = wide_check<D>(a, lds_w);
    if (chk) return chk;
    (void)grid;
    (void)lds;
#define PMML_WIDE_ROWS(R)                                                                     \
    if (rows == R) {                                                                          \
      switch (a.mode) {                                                                       \
        case MODE_SUM: return leaf8 ? launch_wide<D, R, true, MODE_SUM>(st, a, lds_w)         \
                                    : launch_wide<D, R, false, MODE_SUM>(st, a, lds_w);       \
        case MODE_SLOT: return launch_wide<D, R, false, MODE_SLOT>(st, a, lds_w);             \
        case MODE_CLASS: return launch_wide<D, R, false, MODE_CLASS>(st, a, lds_w);           \
        case MODE_VOTE8: return leaf8 ? launch_wide<D, R, true, MODE_VOTE8>(st, a, lds_w)     \
                                      : launch_wide<D, R, false, MODE_VOTE8>(st, a, lds_w);   \
        default: return -11;                                                                  \
      }                                                                                       \
    }
    PMML_WIDE_ROWS(256)
    PMML_WIDE_ROWS(128)
    PMML_WIDE_ROWS(64)
#undef PMML_WIDE_ROWS
    return -12;
  }
  if (base == 2 || (a.variant & ~3)) return -10;  // fp8 leaves / NaN planes: wide kernel only
  if (a.general) {
    err = prepare_launch(tree_perfect_kernel<D, true, 4>, lds);
    if (!err) hipLaunchKernelGGL((tree_perfect_kernel<D, true, 4>), grid, dim3(TB), lds, st, a);
  } else {
    err = prepare_launch(tree_perfect_kernel<D, false, 8>, lds);
    if (!err) hipLaunchKernelGGL((tree_perfect_kernel<D, false, 8>), grid, dim3(TB), lds, st, a);
  }
  return err;
}

}  // namespace
}  // namespace pmml_tree
