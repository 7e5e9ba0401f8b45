// Tree-ensemble scoring: POINTER / GENERAL layouts, split reduction and the C entry points.
// The PERFECT-layout kernels live in tree_common.h (one translation unit per depth: tree_d<D>.hip).
#include "tree_common.h"

namespace pmml_tree {
namespace {
// Pointer layout: nodes uint4 {T bits, meta, left, right}; child < 0 => leaf ~child.
// meta: feature byte offset (or index when features stay in global memory) | bit 30 null-on-
// missing | bit 31 default right.
// MASKED: finished walks skip their load (exec-masked) instead of re-loading node 0 — the vector
// memory pipe then only processes the lanes still walking.
// USKIP: a walk slot whose walks have ended in EVERY lane of the wave issues no load and no
// compare (wave-uniform branch on a ballot): a lock-step group then costs the sum of its trees'
// wave-level depths in gather instructions instead of PILP x the deepest one.
// PEEL: the top two levels of every walk come from wave-uniform node loads (every lane of the
// wave starts on the same root, and a root's two children are adjacent BFS nodes): scalar loads
// through the constant cache plus a per-lane select, instead of two 64-lane vector gathers of
// the same one or two nodes (the walk is bound by the vector memory pipe's per-instruction cost,
// profiles/r3w).
// INL (VAR_POINTER_INLINE): a leaf child's payload sits in its parent's child field (meta bit 29:
// the left child is a leaf, bit 28: the right one) -- the leaf value's fp32 bits for a sum
// ensemble, the class index for an unweighted vote (GENERAL, one increment). The walk ends at the
// parent with the payload in hand: no leaf gather (one per tree and row; P of them for votes).
// LTOP (VAR_POINTER_LTOP, BFS node order): the first 2^LTOP - 1 nodes of the PILP trees of a
// lock-step group -- every internal node of their levels 0 .. LTOP-1 -- are staged in LDS (the
// next group's nodes are loaded into registers while this group walks and written after it:
// NBUF 1 = one buffer, two barriers per group; NBUF 2 = double buffered, one barrier), and the walk
// reads those levels with ds_read_b128 instead of 64-lane global gathers (each ~20 TA cycles
// whatever the lanes hit, profiles/r3w). The host pads the blob with 2^LTOP - 1 zero nodes so the
// staging reads stay in bounds.
template <bool GENERAL, bool FEAT_LDS, int PILP = 8, bool MASKED = false, bool USKIP = false, bool PEEL = false,
          bool INL = false, int LTOP = 0, int NBUF = 2>
__device__ __forceinline__ void pointer_walk(const TreeArgs& a) {
  // LDS: the feature planes, then (GENERAL) the class accumulators — no bad[] array: each thread
  // stages its own row and keeps the row's verdict in a register (POINTER_LDS_BYTES)
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  float* accl = reinterpret_cast<float*>(smem + (FEAT_LDS ? a.n_feat * TB : 0));
  const int tid = threadIdx.x;
  const int2 blk = tree_block(a);
  const int row0 = blk.x * TB;
  const int split = blk.y;
  const int row = row0 + tid;
  bool row_ok = true;
  if (FEAT_LDS) row_ok = !stage_rows_own<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, row0);
  // global-feature mode: apply preparation lazily per read
  const float* xrow = a.X + (size_t)min(row, a.n_rows - 1) * a.ldx;
  if (!FEAT_LDS && a.prep && row < a.n_rows) {
    for (int f = 0; f < a.n_feat; ++f) {
      bool b = false;
      (void)prep_value(xrow[f], a.prep[f], &b);
      if (b) row_ok = false;
    }
  }
  if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
  const uint4* nodes = reinterpret_cast<const uint4*>(a.blob);
  const int tb = split * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);
  if (GENERAL) {
    for (int c = 0; c < a.C; ++c) accl[c * TB + tid] = 0.f;
  }
  float acc = 0.f;
  bool poisoned = false;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);
  constexpr int NTOP = LTOP ? (1 << LTOP) - 1 : 1;
  constexpr int TOPN = PILP * NTOP;          // staged nodes per group
  constexpr int TOPK = (TOPN + TB - 1) / TB;  // ... per thread
  uint4* topl = reinterpret_cast<uint4*>(accl + (GENERAL ? a.C * TB : 0));  // [NBUF][PILP][NTOP]
  auto top_node = [&](int t0s, int e) -> uint4 {  // staged node e of the group at t0s
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (e < TOPN) {
      const int t = t0s + e / NTOP;
      const int r = t < te ? a.roots[t] : -1;
      if (r >= 0) v = nodes[r + e % NTOP];
    }
    return v;
  };
  if (LTOP) {
#pragma unroll
    for (int k = 0; k < TOPK; ++k)
      if (tid + k * TB < TOPN) topl[tid + k * TB] = top_node(tb, tid + k * TB);
    __syncthreads();
  }
  int grp = 0;
  // PILP trees walked in lock-step per lane: every level issues the PILP node loads (L2 gathers)
  // together, so one L2 round trip serves PILP walks instead of one — the walk is latency-bound
  // (dependent loads, divergent depths). Finished walks keep re-loading node 0 (clamped index,
  // no branch around the loads) and are masked out; leaves are accumulated in tree order, so the
  // sums are bit-identical to a serial walk.
  for (int t0 = tb; t0 < te; t0 += PILP, ++grp) {
    const int nt = min(PILP, te - t0);
    const uint4* topg = topl + (NBUF == 2 ? (grp & 1) * TOPN : 0);
    uint4 pre[TOPK];  // the next group's staged nodes, in flight during this group's walk
#pragma unroll
    for (int k = 0; k < TOPK; ++k)
      pre[k] = (LTOP && t0 + PILP < te) ? top_node(t0 + PILP, tid + k * TB) : make_uint4(0u, 0u, 0u, 0u);
    int rootc[PILP];
    int code[PILP];
    bool pz[PILP];
    bool inl[PILP];       // INL: the walk ended on an inline leaf payload (lpay)
    uint32_t lpay[PILP];
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      code[i] = i < nt ? a.roots[t0 + i] : -1;
      rootc[i] = code[i];
      pz[i] = false;
      inl[i] = false;
      lpay[i] = 0u;
    }
    if (PEEL) {
      // level 0: the root (uniform)
      int rc[PILP];
      uint4 n0[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        rc[i] = __builtin_amdgcn_readfirstlane(code[i]);
        n0[i] = nodes[max(rc[i], 0)];
      }
      bool r0[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const float x = *reinterpret_cast<const float*>(feat_lane + (n0[i].y & 0xFFFFu));
        const bool isn = (x != x);
        const bool nulled = rc[i] >= 0 && isn && ((n0[i].y >> 30) & 1u);
        r0[i] = (x >= __uint_as_float(n0[i].x)) || (isn && (n0[i].y >> 31));
        pz[i] = nulled;
        code[i] = rc[i] < 0 ? rc[i] : (nulled ? -1 : (r0[i] ? (int)n0[i].w : (int)n0[i].z));
      }
      // level 1: both children of the root (uniform), selected per lane
      uint4 nl[PILP], nr[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        nl[i] = nodes[max(__builtin_amdgcn_readfirstlane((int)n0[i].z), 0)];
        nr[i] = nodes[max(__builtin_amdgcn_readfirstlane((int)n0[i].w), 0)];
      }
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const uint4 nd = r0[i] ? nr[i] : nl[i];
        const bool act = code[i] >= 0;
        const float x = *reinterpret_cast<const float*>(feat_lane + (nd.y & 0xFFFFu));
        const bool isn = (x != x);
        const bool nulled = act && isn && ((nd.y >> 30) & 1u);
        const bool right = (x >= __uint_as_float(nd.x)) || (isn && (nd.y >> 31));
        pz[i] = pz[i] || nulled;
        code[i] = act ? (nulled ? -1 : (right ? (int)nd.w : (int)nd.z)) : code[i];
      }
    }
    bool live = true;
    int lvl = 0;
    while (live) {
      uint4 nd[PILP];
      bool any[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) any[i] = !USKIP || __builtin_amdgcn_ballot_w64(code[i] >= 0) != 0ull;
      const bool from_lds = LTOP && lvl < LTOP;  // wave-uniform: every walk of the group is on level lvl
      ++lvl;
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        if (from_lds) {
          // a live walk's level-lvl node is one of its tree's first NTOP (BFS); finished -> entry 0
          nd[i] = topg[i * NTOP + min(max(code[i] - rootc[i], 0), NTOP - 1)];
        } else if (USKIP) {
          nd[i] = make_uint4(0u, 0u, 0u, 0u);
          if (any[i]) nd[i] = nodes[max(code[i], 0)];
        } else if (MASKED) {
          nd[i] = make_uint4(0u, 0u, 0u, 0u);
          if (code[i] >= 0) nd[i] = nodes[code[i]];
        } else {
          nd[i] = nodes[max(code[i], 0)];
        }
      }
      live = false;
#pragma unroll
      for (int i = 0; i < PILP; ++i) {  // branch-free: finished walks compute on node 0 and keep their leaf
        if (USKIP && !any[i]) continue;
        const bool act = code[i] >= 0;
        float x;
        if (FEAT_LDS) {
          x = *reinterpret_cast<const float*>(feat_lane + (nd[i].y & 0xFFFFu));
        } else {
          const int f = nd[i].y & 0xFFFFu;
          x = xrow[f];
          if (a.prep) { bool b = false; x = prep_value(x, a.prep[f], &b); }
        }
        const bool isn = (x != x);
        const bool nulled = act && isn && ((nd[i].y >> 30) & 1u);  // null prediction: walk ends, poisoned
        const bool right = (x >= __uint_as_float(nd[i].x)) || (isn && (nd[i].y >> 31));
        const int nc = right ? (int)nd[i].w : (int)nd[i].z;
        pz[i] = pz[i] || nulled;
        if (INL) {
          const bool to_leaf = act && !nulled && ((nd[i].y >> (right ? 28 : 29)) & 1u);
          inl[i] = inl[i] || to_leaf;
          lpay[i] = to_leaf ? (uint32_t)nc : lpay[i];
          code[i] = act ? ((nulled || to_leaf) ? -1 : nc) : code[i];
        } else {
          code[i] = act ? (nulled ? -1 : nc) : code[i];
        }
        live = live || code[i] >= 0;
      }
    }
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      if (i >= nt) break;
      if (pz[i]) {
        if (GENERAL) poisoned = true;
        else acc += __builtin_nanf("");
        continue;
      }
      if (INL && inl[i]) {
        if (GENERAL) accl[(a.tree_slot[t0 + i] + (int)lpay[i]) * TB + tid] += 1.f;
        else acc += __uint_as_float(lpay[i]);
        continue;
      }
      const int leaf = ~code[i];
      if (GENERAL) {
        const int slot = a.tree_slot[t0 + i];
        const float* lp = a.leaves + (size_t)leaf * a.P;
        if (a.leaf_onehot) {
          // a one-hot vote {class, weight}: one 8-byte gather and one slot update (the other
          // slots' += 0 of the dense form change nothing: the accumulators are never -0)
          const int2 lv = reinterpret_cast<const int2*>(a.leaves)[leaf];
          accl[(slot + lv.x) * TB + tid] += __int_as_float(lv.y);
        } else if (a.P == 3) {
          // the row's three payloads as ONE multi-dword gather (a loop over a runtime P issues
          // one 64-lane gather per class); per-slot sums keep the tree order
          const float v0 = lp[0], v1 = lp[1], v2 = lp[2];
          accl[slot * TB + tid] += v0;
          accl[(slot + 1) * TB + tid] += v1;
          accl[(slot + 2) * TB + tid] += v2;
        } else if (a.P == 2) {
          const float v0 = lp[0], v1 = lp[1];
          accl[slot * TB + tid] += v0;
          accl[(slot + 1) * TB + tid] += v1;
        } else {
          for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += lp[p];
        }
      } else {
        acc += a.leaves[leaf];
      }
    }
    if (LTOP) {
      // NBUF 2: the other buffer was last read by group grp - 1, which every wave finished before
      // the previous barrier; NBUF 1: wait until every wave is done with this group's nodes
      if (NBUF == 1) __syncthreads();
#pragma unroll
      for (int k = 0; k < TOPK; ++k)
        if (tid + k * TB < TOPN) topl[(NBUF == 2 ? ((grp + 1) & 1) * TOPN : 0) + tid + k * TB] = pre[k];
      __syncthreads();
    }
  }
  finish_row(a, acc, accl, split, GENERAL, row, row_ok && !poisoned);
}

template <bool GENERAL, bool FEAT_LDS, int PILP = 8, bool MASKED = false, bool USKIP = false, bool PEEL = false,
          bool INL = false, int LTOP = 0, int NBUF = 2>
__global__ __launch_bounds__(TB, 2) void tree_pointer_kernel(TreeArgs a) {
  pointer_walk<GENERAL, FEAT_LDS, PILP, MASKED, USKIP, PEEL, INL, LTOP, NBUF>(a);
}

// Several pointer-layout ensembles over the SAME rows in one launch — the segments of a segmented
// MiningModel (runtime/segmented.py: K segment walks + the fused reduction = 2 launches instead of
// K + 1). grid.z selects the segment; its static argument block (nodes, leaves, epilogue) lives in
// a device array built once per plan, the per-launch fields come from the kernel argument:
// member z scores into S[sidx[z]] / V[sidx[z]] (and probabilities at P + poff[z] * n_rows).
struct MultiTreeArgs {
  const TreeArgs* segs;
  const float* X;
  float* S;
  uint8_t* V;
  float* P;
  const long long* poff;  // nullable: per member, probability column offset (in rows of n_rows)
  const int* sidx;        // per member: its segment index (row of S / V)
  int n_rows, n_feat, ldx, count;
};

template <bool GENERAL>
__global__ __launch_bounds__(TB, 2) void tree_pointer_multi_kernel(MultiTreeArgs m) {
  const int z = blockIdx.z;
  TreeArgs a = m.segs[z];
  a.X = m.X;
  a.n_rows = m.n_rows;
  a.n_feat = m.n_feat;
  a.ldx = m.ldx;
  a.row_valid_in = nullptr;
  a.partial = nullptr;
  a.xcd_split = 0;
  a.trees_per_split = a.n_trees;
  const int seg = m.sidx[z];
  a.score = m.S + (size_t)seg * m.n_rows;
  a.valid = m.V + (size_t)seg * m.n_rows;
  a.probs = (m.P && m.poff) ? m.P + (size_t)m.poff[z] * m.n_rows : nullptr;
  a.epi.score2 = nullptr;
  a.epi.valid2 = nullptr;
  pointer_walk<GENERAL, true>(a);
}

// Compact pointer layout (runtime/hybrid.py::pack_compact_bfs): 8-byte slots {T | leaf value,
// meta}, trees stored level by level with a node's two children in adjacent slots, so the
// lock-step walk of a wave (every lane in the same level of the same tree) touches half the cache
// lines of the 16-byte layout and a node's children always share one. meta: feature (bits 0-5,
// LDS plane) | left-is-leaf (6) | right-is-leaf (7) | first child - slot (8-29) | null (30) |
// default right (31). The walk ends on a leaf's parent; the leaf slot's x is read after the
// loop (P = 1: the weighted value itself; P > 1: its row of `leaves`). Features in LDS only.
template <bool GENERAL>
__global__ __launch_bounds__(TB, 2) void tree_compact_kernel(TreeArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  float* accl = reinterpret_cast<float*>(bad + TB);
  const int tid = threadIdx.x;
  const int2 blk = tree_block(a);
  const int row0 = blk.x * TB;
  const int split = blk.y;
  const int row = row0 + tid;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  bool row_ok = bad[tid] == 0;
  if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
  const uint2* nodes = reinterpret_cast<const uint2*>(a.blob);
  const int tb = split * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);
  if (GENERAL) {
    for (int c = 0; c < a.C; ++c) accl[c * TB + tid] = 0.f;
  }
  float acc = 0.f;
  bool poisoned = false;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);
  constexpr int PILP = 8;
  for (int t0 = tb; t0 < te; t0 += PILP) {
    const int nt = min(PILP, te - t0);
    int pos[PILP];
    bool act[PILP], pz[PILP];
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      const int r = i < nt ? a.roots[t0 + i] : ~0;
      pos[i] = r >= 0 ? r : ~r;
      act[i] = r >= 0;  // a single-leaf tree starts on its leaf
      pz[i] = false;
    }
    bool live = true;
    while (live) {
      uint2 nd[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) nd[i] = nodes[act[i] ? pos[i] : 0];
      live = false;
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const uint32_t m = nd[i].y;
        const float x = *reinterpret_cast<const float*>(feat_lane + ((m & 63u) << 10));
        const bool isn = (x != x);
        const bool nulled = act[i] && isn && ((m >> 30) & 1u);
        const bool right = (x >= __uint_as_float(nd[i].x)) || (isn && (m >> 31));
        const int child = pos[i] + (int)((m >> 8) & 0x3FFFFFu) + (right ? 1 : 0);
        const bool leaf = right ? ((m >> 7) & 1u) : ((m >> 6) & 1u);
        pz[i] = pz[i] || nulled;
        pos[i] = act[i] && !nulled ? child : pos[i];
        act[i] = act[i] && !nulled && !leaf;
        live = live || act[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      if (i >= nt) break;
      if (pz[i]) {
        if (GENERAL) poisoned = true;
        else acc += __builtin_nanf("");
        continue;
      }
      const uint32_t lv = nodes[pos[i]].x;
      if (GENERAL) {
        const int slot = a.tree_slot[t0 + i];
        for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += a.leaves[(size_t)lv * a.P + p];
      } else {
        acc += __uint_as_float(lv);
      }
    }
  }
  finish_row(a, acc, accl, split, GENERAL, row, row_ok && !poisoned);
}

// SUPER pointer layout (runtime/hybrid.py::pack_super): two tree levels per 16-byte load. The
// deep-forest walk is bound by the vector memory pipe's cost per gather INSTRUCTION (profiles/r3u:
// ~20 TA cycles per 64-lane load, the same for 8- and 16-byte lanes and for exec-masked lanes), so
// a slot {T_j, T_l | leaf, T_r | leaf, meta} that carries a split and both children's splits halves
// the loads of a walk. Per step: x_j (LDS) picks the child c, x_c (LDS) picks the grandchild, the
// next slot is base + 1 + 4 * block + 2 (c == r) + (x_c >= T_c). meta: f_j | f_l << 5 | f_r << 10
// (LDS planes, <= 32 features) | l-leaf 15 | r-leaf 16 | self-leaf 17 | default-right j / l / r
// 18-20 | grandchild block 21-31. Root words: tree base slot | nullPrediction flag << 31. Lock-step
// walks, leaves accumulated in tree order (bit-identical to tree_pointer_kernel).
constexpr uint32_t SN_LLEAF = 1u << 15, SN_RLEAF = 1u << 16, SN_SELF = 1u << 17;
constexpr uint32_t SN_DRJ = 1u << 18, SN_DRL = 1u << 19, SN_DRR = 1u << 20;

template <bool GENERAL, int PILP = 8>
__global__ __launch_bounds__(TB, 2) void tree_super_kernel(TreeArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  float* accl = reinterpret_cast<float*>(bad + TB);
  const int tid = threadIdx.x;
  const int2 blk = tree_block(a);
  const int row0 = blk.x * TB;
  const int split = blk.y;
  const int row = row0 + tid;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  bool row_ok = bad[tid] == 0;
  if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
  const uint4* nodes = reinterpret_cast<const uint4*>(a.blob);
  const uint32_t* roots = reinterpret_cast<const uint32_t*>(a.roots);
  const int tb = split * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);
  if (GENERAL) {
    for (int c = 0; c < a.C; ++c) accl[c * TB + tid] = 0.f;
  }
  float acc = 0.f;
  bool poisoned = false;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);
  for (int t0 = tb; t0 < te; t0 += PILP) {
    const int nt = min(PILP, te - t0);
    int pos[PILP], base[PILP];
    uint32_t leafv[PILP];
    bool act[PILP], pz[PILP], nul[PILP];
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      const uint32_t r = i < nt ? roots[t0 + i] : 0u;
      base[i] = (int)(r & 0x7FFFFFFFu);
      pos[i] = base[i];
      nul[i] = (r >> 31) != 0u;
      act[i] = i < nt;
      pz[i] = false;
      leafv[i] = 0u;
    }
    bool live = nt > 0;
    while (live) {
      uint4 nd[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) nd[i] = nodes[act[i] ? pos[i] : 0];
      live = false;
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const uint32_t m = nd[i].w;
        const bool self_leaf = (m & SN_SELF) != 0u;
        // the three feature reads are independent (both children's features read speculatively):
        // one LDS round trip per step instead of two dependent ones
        const float xj = *reinterpret_cast<const float*>(feat_lane + ((m & 31u) << 10));
        const float xl = *reinterpret_cast<const float*>(feat_lane + (((m >> 5) & 31u) << 10));
        const float xr = *reinterpret_cast<const float*>(feat_lane + (((m >> 10) & 31u) << 10));
        const bool nj = (xj != xj);
        const bool r1 = (xj >= __uint_as_float(nd[i].x)) || (nj && (m & SN_DRJ));
        const uint32_t tc = r1 ? nd[i].z : nd[i].y;
        const bool cleaf = (m & (r1 ? SN_RLEAF : SN_LLEAF)) != 0u;
        const bool drc = (m & (r1 ? SN_DRR : SN_DRL)) != 0u;
        const float xc = r1 ? xr : xl;
        const bool nc = (xc != xc);
        const bool r2 = (xc >= __uint_as_float(tc)) || (nc && drc);
        const bool nulled = act[i] && !self_leaf && nul[i] && (nj || (!cleaf && nc));
        const bool done = self_leaf || cleaf;
        leafv[i] = act[i] ? (self_leaf ? nd[i].x : (cleaf ? tc : leafv[i])) : leafv[i];
        pz[i] = pz[i] || nulled;
        pos[i] = (act[i] && !done) ? base[i] + 1 + 4 * (int)(m >> 21) + (r1 ? 2 : 0) + (r2 ? 1 : 0) : pos[i];
        act[i] = act[i] && !done && !nulled;
        live = live || act[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      if (i >= nt) break;
      if (pz[i]) {
        if (GENERAL) poisoned = true;
        else acc += __builtin_nanf("");
        continue;
      }
      if (GENERAL) {
        const int slot = a.tree_slot[t0 + i];
        for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += a.leaves[(size_t)leafv[i] * a.P + p];
      } else {
        acc += __uint_as_float(leafv[i]);
      }
    }
  }
  finish_row(a, acc, accl, split, GENERAL, row, row_ok && !poisoned);
}

// RANK3 pointer layout (runtime/hybrid.py::pack_rank3): THREE tree levels per 16-byte record.
// Split thresholds are replaced by their rank among the feature's sorted unique thresholds: with
// t_0 < t_1 < ... and rank(x) = #{t_k <= x}, "x >= t_k" <=> "rank(x) >= k + 1" — exact, NaN kept
// as its own rank (RK_NAN, routed by the node's default-direction bit). A row's ranks are computed
// once per workgroup (a branchless binary search per feature) into LDS; then a record holds a
// 3-level subtree (7 nodes: 8-bit rank, 5-bit feature, default-right bit each) plus its exit
// block, so one 16-byte gather serves three levels (the deep-forest walk is bound by gather
// instructions / L1 line accesses per visited level, profiles/r3w). Record words: rank3_step; a
// leaf slot has bit 31 of w set and x = the weighted leaf value (or the leaf row for P > 1).
// Nodes: 0 the root,
// 1 / 2 its children, 3..6 the grandchildren; exit e = 4 b0 + 2 b1 + b2 lives at block +
// popcount(mask below e) (only live exits are stored; a block stays within one 128-byte line).
// Leaves above the third level are padded with never-right nodes (rank 255). The root record is
// read with a wave-uniform (scalar) load. Lock-step walks, leaves accumulated in tree order
// (bit-identical to tree_pointer_kernel).
constexpr uint32_t RK_NAN = 255;

// One record step: the three levels' decisions, then the exit's slot offset from the tree base.
// Every field sits inside one 32-bit word (runtime/hybrid.py record layout): x = ranks 0-3,
// y = ranks 4-6 | live-exit mask << 24, z = features 0-5 | default-right 0 / 1 << 30 / 31,
// w = feature 6 | default-right 2-6 << 5.. | block offset << 10 | leaf << 31.
__device__ __forceinline__ int rank3_step(const uint4 rec, const uint32_t* rk_lane) {
  auto decide = [](uint32_t k, uint32_t r, uint32_t d) -> uint32_t { return k == RK_NAN ? d : (uint32_t)(k >= r); };
  // level 0: node 0
  const uint32_t b0 = decide(rk_lane[(rec.z & 31u) * TB], rec.x & 255u, (rec.z >> 30) & 1u);
  // level 1: node 1 + b0 (features / ranks in z / x; default-right bit 31 of z or bit 5 of w)
  const uint32_t n1 = 1u + b0;
  const uint32_t b1 = decide(rk_lane[((rec.z >> (5u * n1)) & 31u) * TB], (rec.x >> (8u * n1)) & 255u,
                             b0 ? ((rec.w >> 5) & 1u) : (rec.z >> 31));
  // level 2: node 3 + 2 b0 + b1 (3 .. 6)
  const uint32_t n2 = 3u + 2u * b0 + b1;
  const uint32_t f2 = n2 == 6u ? (rec.w & 31u) : ((rec.z >> (5u * n2)) & 31u);
  const uint32_t r2 = n2 == 3u ? (rec.x >> 24) : ((rec.y >> (8u * (n2 - 4u))) & 255u);
  const uint32_t b2 = decide(rk_lane[f2 * TB], r2, (rec.w >> (n2 + 3u)) & 1u);
  const uint32_t e = 4u * b0 + 2u * b1 + b2;
  return (int)((rec.w >> 10) & 0x1FFFFFu) + __popc((rec.y >> 24) & ((1u << e) - 1u));
}

template <bool GENERAL, int PILP = 8>
__global__ __launch_bounds__(TB, 2) void tree_rank3_kernel(TreeArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + a.n_feat * TB);
  float* accl = reinterpret_cast<float*>(bad + TB);
  // ranks overwrite the feature planes in place (a lane only ever reads its own row): 32-bit
  // entries keep every lane on its own bank whatever feature it reads (16-bit planes put two
  // lanes on one bank: 2-way conflicts on every rank read of the walk)
  uint32_t* rk = reinterpret_cast<uint32_t*>(feat);  // [F][TB]
  const int tid = threadIdx.x;
  const int2 blk = tree_block(a);
  const int row0 = blk.x * TB;
  const int split = blk.y;
  const int row = row0 + tid;
  stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  bool row_ok = bad[tid] == 0;
  if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
  // ranks of this lane's row: 8 features' branchless binary searches advanced together (8
  // independent cached reads in flight per step; a dependent search per feature left every
  // workgroup idle for tens of microseconds before its first tree). The tables stay in global
  // memory (L1-resident; staging them in LDS cost a workgroup per CU, profiles/r4q). Only this
  // lane reads its ranks back: no barrier after.
  const float* thr_l = a.rank_thr;  // [F][rank_stride]
  const int stride = a.rank_stride;
  for (int f0 = 0; f0 < a.n_feat; f0 += 8) {
    float x[8];
    int pos[8], cnt[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool on = f0 + k < a.n_feat;
      x[k] = on ? feat[(f0 + k) * TB + tid] : 0.f;
      cnt[k] = on ? a.rank_cnt[f0 + k] : 0;
      pos[k] = 0;  // #{t <= x}
    }
#pragma unroll
    for (int step = 128; step > 0; step >>= 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = pos[k] + step;
        const int at = max(min(q, cnt[k]) - 1, 0);
        const float t = thr_l[(f0 + k) * stride + at];
        pos[k] = (q <= cnt[k] && t <= x[k]) ? q : pos[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (f0 + k < a.n_feat) rk[(f0 + k) * TB + tid] = x[k] != x[k] ? RK_NAN : (uint32_t)pos[k];
  }
  const uint32_t* rk_lane = rk + tid;
  const uint4* nodes = reinterpret_cast<const uint4*>(a.blob);
  const uint32_t* roots = reinterpret_cast<const uint32_t*>(a.roots);
  const int tb = split * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);
  if (GENERAL) {
    for (int c = 0; c < a.C; ++c) accl[c * TB + tid] = 0.f;
  }
  float acc = 0.f;
  for (int t0 = tb; t0 < te; t0 += PILP) {
    const int nt = min(PILP, te - t0);
    int pos[PILP], base[PILP];
    uint32_t leafv[PILP];
    bool act[PILP];
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      base[i] = i < nt ? (int)roots[t0 + i] : 0;
      pos[i] = base[i];
      act[i] = i < nt;
      leafv[i] = 0u;
    }
    // the root record: every lane of the wave starts on it — one uniform (scalar) load per tree
    // instead of a 64-lane gather
    {
      uint4 rt[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) rt[i] = nodes[__builtin_amdgcn_readfirstlane(base[i])];
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const bool leaf = (rt[i].w >> 31) != 0u;
        const int nxt = base[i] + rank3_step(rt[i], rk_lane);
        leafv[i] = (act[i] && leaf) ? rt[i].x : leafv[i];
        pos[i] = (act[i] && !leaf) ? nxt : pos[i];
        act[i] = act[i] && !leaf;
      }
    }
    bool live = false;
#pragma unroll
    for (int i = 0; i < PILP; ++i) live = live || act[i];
    while (live) {
      uint4 nd[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) nd[i] = nodes[act[i] ? pos[i] : 0];
      live = false;
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const bool leaf = (nd[i].w >> 31) != 0u;
        const int nxt = base[i] + rank3_step(nd[i], rk_lane);
        leafv[i] = (act[i] && leaf) ? nd[i].x : leafv[i];
        pos[i] = (act[i] && !leaf) ? nxt : pos[i];
        act[i] = act[i] && !leaf;
        live = live || act[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      if (i >= nt) break;
      if (GENERAL) {
        const int slot = a.tree_slot[t0 + i];
        for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += a.leaves[(size_t)leafv[i] * a.P + p];
      } else {
        acc += __uint_as_float(leafv[i]);
      }
    }
  }
  finish_row(a, acc, accl, split, GENERAL, row, row_ok);
}

// Pointer layout, refill schedule. The lock-step kernel above runs each group of PILP walks until
// the deepest of its 64 x PILP walks ends: at depth 14 with ~6-level average paths most lanes idle
// through half of every group. Here each of a lane's PILP slots is a work queue over the tree
// range: the step that reaches a leaf accumulates it and immediately loads the next tree's root,
// so every slot stays busy until the range is exhausted and the wave's loop count tracks the
// AVERAGE path length, not the maximum. Root indices are staged in LDS (the refill hop is an LDS
// read, not an L2 round trip). Leaves are added in completion order — deterministic for a given
// forest, but not the tree-order fp32 sum of the lock-step kernel.
constexpr int REFILL_ROOTS_LDS = 2048;

template <bool GENERAL, bool FEAT_LDS>
__global__ __launch_bounds__(TB, 2) void tree_pointer_refill_kernel(TreeArgs a) {
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + (FEAT_LDS ? a.n_feat * TB : 0));
  float* accl = reinterpret_cast<float*>(bad + TB);
  int* roots_l = reinterpret_cast<int*>(accl + (GENERAL ? a.C * TB : 0));
  const int tid = threadIdx.x;
  const int2 blk = tree_block(a);
  const int row0 = blk.x * TB;
  const int split = blk.y;
  const int row = row0 + tid;
  const int tb = split * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);
  const bool roots_in_lds = te - tb <= REFILL_ROOTS_LDS;
  if (roots_in_lds)
    for (int t = tid; t < te - tb; t += TB) roots_l[t] = a.roots[tb + t];
  if (FEAT_LDS) {
    stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);  // ends with a barrier
  } else {
    bad[tid] = 0;
    __syncthreads();
  }
  bool row_ok = bad[tid] == 0;
  const float* xrow = a.X + (size_t)min(row, a.n_rows - 1) * a.ldx;
  if (!FEAT_LDS && a.prep && row < a.n_rows) {
    for (int f = 0; f < a.n_feat; ++f) {
      bool b = false;
      (void)prep_value(xrow[f], a.prep[f], &b);
      if (b) row_ok = false;
    }
  }
  if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
  const uint4* nodes = reinterpret_cast<const uint4*>(a.blob);
  if (GENERAL) {
    for (int c = 0; c < a.C; ++c) accl[c * TB + tid] = 0.f;
  }
  auto root_of = [&](int t) { return roots_in_lds ? roots_l[t - tb] : a.roots[t]; };
  float acc = 0.f;
  bool poisoned = false;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);
  constexpr int PILP = 8;
  int code[PILP], tix[PILP];
  int next = tb;
#pragma unroll
  for (int i = 0; i < PILP; ++i) {
    const bool take = next < te;
    tix[i] = next;
    code[i] = take ? root_of(next) : -1;
    next += take ? 1 : 0;
  }
  bool live = te > tb;
  while (live) {
    uint4 nd[PILP];
#pragma unroll
    for (int i = 0; i < PILP; ++i) nd[i] = nodes[max(code[i], 0)];
    live = false;
#pragma unroll
    for (int i = 0; i < PILP; ++i) {
      const bool act = code[i] >= 0;
      float x;
      if (FEAT_LDS) {
        x = *reinterpret_cast<const float*>(feat_lane + (nd[i].y & 0xFFFFu));
      } else {
        const int f = nd[i].y & 0xFFFFu;
        x = xrow[f];
        if (a.prep) { bool b = false; x = prep_value(x, a.prep[f], &b); }
      }
      const bool isn = (x != x);
      const bool nulled = act && isn && ((nd[i].y >> 30) & 1u);
      const bool right = (x >= __uint_as_float(nd[i].x)) || (isn && (nd[i].y >> 31));
      const int nc = right ? (int)nd[i].w : (int)nd[i].z;
      const bool done = act && (nulled || nc < 0);
      if (done) {
        if (nulled) {
          if (GENERAL) poisoned = true;
          else acc += __builtin_nanf("");
        } else if (GENERAL) {
          const int slot = a.tree_slot[tix[i]];
          for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += a.leaves[(size_t)(~nc) * a.P + p];
        } else {
          acc += a.leaves[~nc];
        }
        const bool take = next < te;
        tix[i] = next;
        code[i] = take ? root_of(next) : -1;
        next += take ? 1 : 0;
      } else if (act) {
        code[i] = nc;
      }
      live = live || code[i] >= 0;
    }
  }
  finish_row(a, acc, accl, split, GENERAL, row, row_ok && !poisoned);
}

// Split-mode reduction: partial[splits][C+1][n_rows] -> epilogue.
__global__ __launch_bounds__(TB) void tree_reduce_kernel(TreeArgs a, int splits) {
  const int row = blockIdx.x * TB + threadIdx.x;
  if (row >= a.n_rows) return;
  const size_t stride = (size_t)a.n_rows;
  float acc[16];
  const int C = a.C;
  for (int c = 0; c < 16; ++c) acc[c] = 0.f;
  bool ok = true;
  for (int s = 0; s < splits; ++s) {
    const float* base = a.partial + (size_t)s * (C + 1) * stride;
    for (int c = 0; c < C && c < 16; ++c) acc[c] += base[c * stride + row];
    ok = ok && base[C * stride + row] == 0.f;
  }
  apply_epilogue(a.epi, [&](int c) { return acc[c]; }, ok, row, a.n_rows, a.score, a.valid, a.probs);
}


// ------------------------------------------------------------------------------------------
// GENERAL layout: any PMML TreeModel shape — multiway splits, SimpleSetPredicate, Compound
// and / or / xor / surrogate predicates, every missingValueStrategy except the two aggregating ones,
// both noTrueChildStrategy values, internal-node scores. Each lane walks its row through a node
// table, evaluating the children's predicates as postfix programs over PMML's three-valued logic
// (TRUE 1 / FALSE 0 / UNKNOWN 2, packed 2 bits per entry in a 64-bit register stack). Divergent,
// node tables read from L2 — the fallback for shapes the branch-free layouts cannot express.
enum : int {
  P_END = 0, P_TRUE, P_FALSE, P_GE, P_EQ, P_ISMISS, P_NOTMISS, P_SET, P_AND, P_OR, P_XOR, P_SURR,
};
enum : int { S_NONE = 0, S_LAST = 1, S_NULL = 2, S_DEFAULT = 3, S_WCONF = 4, S_AGG = 5 };
constexpr uint32_t V_F = 0u, V_T = 1u, V_U = 2u;
constexpr int MIX_STACK = 64;  // host-checked: 1 + sum over any path of (children - 1)

struct GenTreeArgs {
  TreeArgs t;                  // rows, prep, epilogue, payload (t.leaves [nodes][P]), slots, outputs
  const int4* nodes;           // {child_off, n_child | has_score << 16, pred_off, default_child}
  const int* children;         // child node indices
  const int4* preds;           // {op | neg << 8, field or n, pool offset / count, T bits}
  const float* pool;           // SimpleSetPredicate values
  const int2* trees;           // {root node, strategy (3 bits) | returnLastPrediction << 3}
  int max_steps, pad;
  // weightedConfidence / aggregateNodes trees (null when the ensemble has none):
  const float* mix_mass;       // [nodes][P] class mass of each node, tree category order
  const float* mix_w;          // [nodes] weight of a node as a mixture child
  const int4* mix_tab;         // [trees] {segment weight bits, vote, tree categories, remap offset}
  const int* remap;            // tree category -> accumulator slot
  const int* vcol;             // [nodes] input column added to the leaf value (complex scorecards), -1: none; nullable
};

template <bool FEAT_LDS>
__device__ __forceinline__ float gen_feature(const GenTreeArgs& a, const char* feat_lane, const float* xrow, int f) {
  if (FEAT_LDS) return *reinterpret_cast<const float*>(feat_lane + f * TB * 4);
  float x = xrow[f];
  if (a.t.prep) {
    bool b = false;
    x = prep_value(x, a.t.prep[f], &b);
  }
  return x;
}

template <bool FEAT_LDS>
__device__ uint32_t gen_eval(const GenTreeArgs& a, int pc, const char* feat_lane, const float* xrow) {
  uint64_t st = 0;
  for (;; ++pc) {
    const int4 in = a.preds[pc];
    const int op = in.x & 0xFF;
    const uint32_t neg = (uint32_t)(in.x >> 8) & 1u;
    uint32_t v;
    if (op == P_END) return (uint32_t)(st & 3u);
    if (op >= P_AND) {
      const int n = in.y;
      bool any_t = false, any_f = false, any_u = false;
      uint32_t par = 0u, sur = V_U;
      for (int i = 0; i < n; ++i) {
        const uint32_t e = (uint32_t)(st & 3u);
        st >>= 2;
        any_t |= e == V_T;
        any_f |= e == V_F;
        any_u |= e == V_U;
        par ^= (e == V_T) ? 1u : 0u;
        if (e != V_U) sur = e;  // popped top-down: ends at the first (bottom-most) known value
      }
      if (op == P_AND) v = any_f ? V_F : (any_u ? V_U : V_T);
      else if (op == P_OR) v = any_t ? V_T : (any_u ? V_U : V_F);
      else if (op == P_XOR) v = any_u ? V_U : par;
      else v = sur;
    } else if (op == P_TRUE) {
      v = V_T;
    } else if (op == P_FALSE) {
      v = V_F;
    } else {
      const float x = gen_feature<FEAT_LDS>(a, feat_lane, xrow, in.y);
      const bool miss = x != x;
      if (op == P_ISMISS) {
        v = miss ? V_T : V_F;
      } else if (op == P_NOTMISS) {
        v = miss ? V_F : V_T;
      } else if (miss) {
        v = V_U;
      } else {
        bool r;
        if (op == P_GE) {
          r = x >= __int_as_float(in.w);
        } else if (op == P_EQ) {
          r = x == __int_as_float(in.w);
        } else {  // P_SET
          r = false;
          for (int i = 0; i < in.w; ++i) r = r || (a.pool[in.z + i] == x);
        }
        v = (r ? 1u : 0u) ^ neg;
      }
    }
    st = (st << 2) | v;
  }
}

// Returns the scoring node of tree t for this lane's row, -1 (null prediction), or -2: a
// weightedConfidence / aggregateNodes tree met an UNKNOWN child (the caller runs gen_mixture).
template <bool FEAT_LDS>
__device__ int gen_walk(const GenTreeArgs& a, int t, const char* feat_lane, const float* xrow) {
  const int2 tr = a.trees[t];
  const int strat = tr.y & 7;
  const bool ret_last = ((tr.y >> 3) & 1) != 0;
  int node = tr.x;
  if (gen_eval<FEAT_LDS>(a, a.nodes[node].z, feat_lane, xrow) != V_T) return -1;
  for (int step = 0; step < a.max_steps; ++step) {
    const int4 nd = a.nodes[node];
    const int nc = nd.y & 0xFFFF;
    if (nc == 0) return node;
    int next = -1;
    for (int c = 0; c < nc; ++c) {
      const int ch = a.children[nd.x + c];
      const uint32_t v = gen_eval<FEAT_LDS>(a, a.nodes[ch].z, feat_lane, xrow);
      if (v == V_U && strat >= S_WCONF) return -2;
      if (v == V_U && strat != S_NONE) {
        if (strat == S_LAST) return node;
        if (strat == S_NULL) return -1;
        next = nd.w;  // defaultChild (-1 when absent: no prediction)
        if (next < 0) return -1;
        break;
      }
      if (v == V_T) {
        next = ch;
        break;
      }
    }
    if (next < 0) return ret_last ? node : -1;
    node = next;
  }
  return -1;
}

// weightedConfidence / aggregateNodes (models/tree.py::_mixture): the row restarts at the root
// as a depth-first walk over (node, weight, inside-a-mixture) entries. A TRUE child continues the
// path; at the first UNKNOWN child the path forks into that child and every later sibling that is
// not FALSE, each weighted by its mix_w; a leaf adds weight x its class mass. A node without a
// true child adds its own mass under returnLastPrediction, else voids the row on a pure TRUE path
// (the oracle's NaN) or contributes nothing inside a mixture (nan_to_num). Then the tree adds its
// normalised mass (or a vote for its first argmax) to the class slots. Returns false: no prediction.
template <bool FEAT_LDS>
__device__ bool gen_mixture(const GenTreeArgs& a, int t, const char* feat_lane, const float* xrow, float* accl,
                            int tid) {
  const int2 tr = a.trees[t];
  const bool ret_last = ((tr.y >> 3) & 1) != 0;
  const int4 mt = a.mix_tab[t];
  const int P = a.t.P;
  const int Ct = mt.z;
  float mass[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) mass[c] = 0.f;
  int st_node[MIX_STACK];
  float st_w[MIX_STACK];
  uint64_t st_in = 0;  // bit i: entry i is inside a mixture
  int sp = 0;
  st_node[0] = tr.x;
  st_w[0] = 1.f;
  sp = 1;
  int guard = 0;
  while (sp > 0 && guard < (1 << 20)) {
    ++guard;
    --sp;
    const int node = st_node[sp];
    const float w = st_w[sp];
    const bool inside = (st_in >> sp) & 1ull;
    st_in &= ~(1ull << sp);
    const int4 nd = a.nodes[node];
    const int nc = nd.y & 0xFFFF;
    if (nc == 0) {
      for (int c = 0; c < Ct; ++c) mass[c] += w * a.mix_mass[(size_t)node * P + c];
      continue;
    }
    int k = -1;
    uint32_t vk = V_F;
    for (int c = 0; c < nc; ++c) {
      vk = gen_eval<FEAT_LDS>(a, a.nodes[a.children[nd.x + c]].z, feat_lane, xrow);
      if (vk != V_F) {
        k = c;
        break;
      }
    }
    if (k < 0) {
      if (ret_last) {
        for (int c = 0; c < Ct; ++c) mass[c] += w * a.mix_mass[(size_t)node * P + c];
      } else if (!inside) {
        return false;
      }
      continue;
    }
    if (vk == V_T) {
      if (sp >= MIX_STACK) return false;  // host-checked bound; never reached
      st_node[sp] = a.children[nd.x + k];
      st_w[sp] = w;
      if (inside) st_in |= 1ull << sp;
      ++sp;
      continue;
    }
    // first UNKNOWN at child k: k and every later sibling that is not FALSE, pushed last-first
    // so child k is expanded first (the oracle's summation order)
    for (int c = nc - 1; c >= k; --c) {
      const int ch = a.children[nd.x + c];
      const uint32_t v = c == k ? V_U : gen_eval<FEAT_LDS>(a, a.nodes[ch].z, feat_lane, xrow);
      if (v == V_F) continue;
      if (sp >= MIX_STACK) return false;
      st_node[sp] = ch;
      st_w[sp] = w * a.mix_w[ch];
      st_in |= 1ull << sp;
      ++sp;
    }
  }
  float tot = 0.f;
  for (int c = 0; c < Ct; ++c) tot += mass[c];
  if (!(tot > 0.f) || !isfinite(tot)) return false;
  const float wt = __int_as_float(mt.x);
  const int* rm = a.remap + mt.w;
  if (mt.y) {
    int best = 0;
    for (int c = 1; c < Ct; ++c)
      if (mass[c] > mass[best]) best = c;
    accl[rm[best] * TB + tid] += wt;
  } else {
    const float inv = 1.f / tot;
    for (int c = 0; c < Ct; ++c) accl[rm[c] * TB + tid] += (mass[c] * inv) * wt;
  }
  return true;
}

template <bool GENERAL, bool FEAT_LDS>
__global__ __launch_bounds__(TB, 2) void tree_general_kernel(GenTreeArgs ga) {
  const TreeArgs& a = ga.t;
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + (FEAT_LDS ? a.n_feat * TB : 0));
  float* accl = reinterpret_cast<float*>(bad + TB);
  const int tid = threadIdx.x;
  const int row0 = blockIdx.x * TB;
  const int row = row0 + tid;
  if (FEAT_LDS) {
    stage_rows_T<TB>(a.X, a.n_rows, a.n_feat, a.ldx, a.prep, feat, bad, row0);
  } else {
    bad[tid] = 0;
    __syncthreads();
  }
  bool row_ok = bad[tid] == 0;
  const float* xrow = a.X + (size_t)min(row, a.n_rows - 1) * a.ldx;
  if (!FEAT_LDS && a.prep && row < a.n_rows) {
    for (int f = 0; f < a.n_feat; ++f) {
      bool b = false;
      (void)prep_value(xrow[f], a.prep[f], &b);
      if (b) row_ok = false;
    }
  }
  if (a.row_valid_in && row < a.n_rows) row_ok = row_ok && a.row_valid_in[row];
  if (GENERAL) {
    for (int c = 0; c < a.C; ++c) accl[c * TB + tid] = 0.f;
  }
  float acc = 0.f;
  bool poisoned = false;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);
  if (row < a.n_rows) {
    for (int t = 0; t < a.n_trees; ++t) {
      const int node = gen_walk<FEAT_LDS>(ga, t, feat_lane, xrow);
      if (GENERAL && node == -2) {  // sibling mixture (weightedConfidence / aggregateNodes)
        if (!gen_mixture<FEAT_LDS>(ga, t, feat_lane, xrow, accl, tid)) poisoned = true;
        continue;
      }
      if (node < 0 || ((ga.nodes[node].y >> 16) & 1) == 0) {  // null prediction
        if (GENERAL) poisoned = true;
        else acc += __builtin_nanf("");
        continue;
      }
      if (GENERAL) {
        const int slot = a.tree_slot[t];
        for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += a.leaves[(size_t)node * a.P + p];
      } else {
        acc += a.leaves[node];
        if (ga.vcol) {  // a leaf scored per record from an input column (NaN -> no prediction)
          const int vc = ga.vcol[node];
          if (vc >= 0) acc += gen_feature<FEAT_LDS>(ga, feat_lane, xrow, vc);
        }
      }
    }
  }
  finish_row(a, acc, accl, 0, GENERAL, row, row_ok && !poisoned);
}

}  // namespace
}  // namespace pmml_tree

using namespace pmml_tree;

PMML_API int pmml_tree_args_size() { return (int)sizeof(TreeArgs); }
PMML_API int pmml_tree_rows_per_block() { return TB; }

// layout: 0 = perfect (depth in [1,10]), 1 = pointer. splits >= 1 (tree-parallel split of the
// ensemble across grid.y; > 1 requires a.partial with room for splits*(C+1)*n_rows floats).
PMML_API int pmml_tree_launch(hipStream_t stream, const TreeArgs* args, int layout, int depth, int has_dr,
                              int splits) {
  TreeArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (splits < 1) splits = 1;
  if (splits > 1 && a.partial == nullptr) return -2;
  if (splits == 1) a.partial = nullptr;
  if (a.C > 16) return -3;
  a.trees_per_split = (a.n_trees + splits - 1) / splits;
  if (a.n_trees > 0) splits = (a.n_trees + a.trees_per_split - 1) / a.trees_per_split;  // no empty split
  if (splits == 1) a.partial = nullptr;
  const int row_blocks = (a.n_rows + TB - 1) / TB;
  if (layout == 0 || splits == 1) a.xcd_split = 0;  // PERFECT kernels: grid.y splits (forests fit L2)
  if (a.xcd_split > 0) a.xcd_split = splits;
  if (a.xcd_split > 0 && (long long)row_blocks * splits > 0x7FFFFFFFLL) return -11;
  dim3 grid = a.xcd_split > 0 ? dim3(row_blocks * splits) : dim3(row_blocks, splits);
  int err = 0;
  const size_t acc_lds = a.general ? (size_t)a.C * TB * 4 : 0;
  if (layout == 0) {
    const bool wide = (a.variant & 3) != 0;
    if (wide) {
      if (a.n_stage < 1 || a.n_stage > 256 || !(a.rows_wide == 256 || a.rows_wide == 128 || a.rows_wide == 64)) return -4;
      if (a.n_stage > (64 * 256) / a.rows_wide) return -4;  // planes <= 64 KiB (+ one pad float each)
    } else if (a.n_feat > 64) {
      return -4;
    }
    if (!wide && (size_t)a.chunk_trees * a.rec_words > (size_t)TB * 4 * PREFETCH_Q) return -9;
    const size_t lds = wide ? 0 : (size_t)a.n_feat * TB * 4 + 2 * (size_t)a.chunk_trees * a.rec_words * 4 + (TB + 4) * 4 + acc_lds;
    if (lds > 160 * 1024) return -5;
    switch (depth) {
      case 1: err = launch_perfect_d1(stream, a, grid, lds); break;
      case 2: err = launch_perfect_d2(stream, a, grid, lds); break;
      case 3: err = launch_perfect_d3(stream, a, grid, lds); break;
      case 4: err = launch_perfect_d4(stream, a, grid, lds); break;
      case 5: err = launch_perfect_d5(stream, a, grid, lds); break;
      case 6: err = launch_perfect_d6(stream, a, grid, lds); break;
      case 7: err = launch_perfect_d7(stream, a, grid, lds); break;
      case 8: err = launch_perfect_d8(stream, a, grid, lds); break;
      case 9: err = launch_perfect_d9(stream, a, grid, lds); break;
      case 10: err = launch_perfect_d10(stream, a, grid, lds); break;
      default: return -6;
    }
  } else {
    if (a.variant != 0 && a.variant != VAR_POINTER_REFILL && a.variant != VAR_POINTER_COMPACT &&
        a.variant != VAR_POINTER_MASKED && a.variant != VAR_POINTER_SUPER && a.variant != VAR_POINTER_USKIP &&
        a.variant != VAR_POINTER_PEEL && a.variant != VAR_POINTER_RANK3 &&
        a.variant != VAR_POINTER_INLINE && a.variant != VAR_POINTER_LTOP &&
        a.variant != (VAR_POINTER_LTOP | VAR_POINTER_INLINE))
      return -10;
    const bool feat_lds = a.n_feat <= 64;
    size_t lds = (feat_lds ? (size_t)a.n_feat * TB * 4 : 0) + TB * 4 + acc_lds;
    // pointer_walk kernels (PEEL / USKIP / INLINE / default): feature planes + accumulators only
    const size_t lds_pw = (feat_lds ? (size_t)a.n_feat * TB * 4 : 0) + acc_lds;
    if (a.variant == VAR_POINTER_RANK3) {
      if (a.n_feat > 32 || !a.rank_thr || !a.rank_cnt || a.rank_stride < 1 || a.rank_stride > 254) return -4;
      // (ranks replace the feature planes; the threshold tables are read from global memory)
      if (lds > 160 * 1024) return -5;
      if (a.general) {
        err = prepare_launch(tree_rank3_kernel<true>, lds);
        if (!err) hipLaunchKernelGGL((tree_rank3_kernel<true>), grid, dim3(TB), lds, stream, a);
      } else if (a.pilp == 16) {
        err = prepare_launch(tree_rank3_kernel<false, 16>, lds);
        if (!err) hipLaunchKernelGGL((tree_rank3_kernel<false, 16>), grid, dim3(TB), lds, stream, a);
      } else if (a.pilp == 4) {
        err = prepare_launch(tree_rank3_kernel<false, 4>, lds);
        if (!err) hipLaunchKernelGGL((tree_rank3_kernel<false, 4>), grid, dim3(TB), lds, stream, a);
      } else {
        err = prepare_launch(tree_rank3_kernel<false>, lds);
        if (!err) hipLaunchKernelGGL((tree_rank3_kernel<false>), grid, dim3(TB), lds, stream, a);
      }
    } else if (a.variant == VAR_POINTER_SUPER) {
      if (a.n_feat > 32) return -4;  // 5-bit feature fields
      if (a.general) {
        err = prepare_launch(tree_super_kernel<true>, lds);
        if (!err) hipLaunchKernelGGL((tree_super_kernel<true>), grid, dim3(TB), lds, stream, a);
      } else if (a.pilp == 16) {
        err = prepare_launch(tree_super_kernel<false, 16>, lds);
        if (!err) hipLaunchKernelGGL((tree_super_kernel<false, 16>), grid, dim3(TB), lds, stream, a);
      } else if (a.pilp == 4) {
        err = prepare_launch(tree_super_kernel<false, 4>, lds);
        if (!err) hipLaunchKernelGGL((tree_super_kernel<false, 4>), grid, dim3(TB), lds, stream, a);
      } else if (a.pilp == 2) {
        err = prepare_launch(tree_super_kernel<false, 2>, lds);
        if (!err) hipLaunchKernelGGL((tree_super_kernel<false, 2>), grid, dim3(TB), lds, stream, a);
      } else {
        err = prepare_launch(tree_super_kernel<false>, lds);
        if (!err) hipLaunchKernelGGL((tree_super_kernel<false>), grid, dim3(TB), lds, stream, a);
      }
    } else if (a.variant == VAR_POINTER_COMPACT) {
      if (!feat_lds) return -4;
      if (a.general) {
        err = prepare_launch(tree_compact_kernel<true>, lds);
        if (!err) hipLaunchKernelGGL((tree_compact_kernel<true>), grid, dim3(TB), lds, stream, a);
      } else {
        err = prepare_launch(tree_compact_kernel<false>, lds);
        if (!err) hipLaunchKernelGGL((tree_compact_kernel<false>), grid, dim3(TB), lds, stream, a);
      }
    } else if (a.variant == VAR_POINTER_REFILL) {
      lds += (size_t)REFILL_ROOTS_LDS * 4;
      if (a.general) {
        if (feat_lds) {
          err = prepare_launch(tree_pointer_refill_kernel<true, true>, lds);
          if (!err) hipLaunchKernelGGL((tree_pointer_refill_kernel<true, true>), grid, dim3(TB), lds, stream, a);
        } else {
          err = prepare_launch(tree_pointer_refill_kernel<true, false>, lds);
          if (!err) hipLaunchKernelGGL((tree_pointer_refill_kernel<true, false>), grid, dim3(TB), lds, stream, a);
        }
      } else {
        if (feat_lds) {
          err = prepare_launch(tree_pointer_refill_kernel<false, true>, lds);
          if (!err) hipLaunchKernelGGL((tree_pointer_refill_kernel<false, true>), grid, dim3(TB), lds, stream, a);
        } else {
          err = prepare_launch(tree_pointer_refill_kernel<false, false>, lds);
          if (!err) hipLaunchKernelGGL((tree_pointer_refill_kernel<false, false>), grid, dim3(TB), lds, stream, a);
        }
      }
    } else if (a.variant == (VAR_POINTER_LTOP | VAR_POINTER_INLINE) && feat_lds) {
      const size_t lt = lds_pw + (size_t)8 * 31 * 16;
      if (a.general) {
        err = prepare_launch(tree_pointer_kernel<true, true, 8, false, false, false, true, 5, 1>, lt);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<true, true, 8, false, false, false, true, 5, 1>), grid, dim3(TB), lt,
                             stream, a);
      } else {
        err = prepare_launch(tree_pointer_kernel<false, true, 8, false, false, false, true, 5, 1>, lt);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<false, true, 8, false, false, false, true, 5, 1>), grid, dim3(TB), lt,
                             stream, a);
      }
    } else if (a.variant == VAR_POINTER_LTOP && feat_lds) {
      // levels 0-4 (31 nodes a tree), one LDS buffer (profiles/r6l: two buffers or a sixth level
      // cost a workgroup per CU and measured no faster for sums, 16-20 % slower for votes)
      const size_t lt = lds_pw + (size_t)(a.pilp == 6 ? 6 : 8) * 31 * 16;
      if (a.pilp == 6) {
        if (a.general) {
          err = prepare_launch(tree_pointer_kernel<true, true, 6, false, false, false, false, 5, 1>, lt);
          if (!err)
            hipLaunchKernelGGL((tree_pointer_kernel<true, true, 6, false, false, false, false, 5, 1>), grid, dim3(TB),
                               lt, stream, a);
        } else {
          err = prepare_launch(tree_pointer_kernel<false, true, 6, false, false, false, false, 5, 1>, lt);
          if (!err)
            hipLaunchKernelGGL((tree_pointer_kernel<false, true, 6, false, false, false, false, 5, 1>), grid, dim3(TB),
                               lt, stream, a);
        }
      } else if (a.general) {
        err = prepare_launch(tree_pointer_kernel<true, true, 8, false, false, false, false, 5, 1>, lt);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<true, true, 8, false, false, false, false, 5, 1>), grid, dim3(TB), lt,
                             stream, a);
      } else {
        err = prepare_launch(tree_pointer_kernel<false, true, 8, false, false, false, false, 5, 1>, lt);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<false, true, 8, false, false, false, false, 5, 1>), grid, dim3(TB), lt,
                             stream, a);
      }
    } else if (a.variant == VAR_POINTER_PEEL && feat_lds) {
      if (a.general) {
        err = prepare_launch(tree_pointer_kernel<true, true, 8, false, false, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<true, true, 8, false, false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else {
        err = prepare_launch(tree_pointer_kernel<false, true, 8, false, false, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 8, false, false, true>), grid, dim3(TB), lds_pw, stream, a);
      }
    } else if (a.variant == VAR_POINTER_USKIP && feat_lds) {
      if (a.general) {
        err = prepare_launch(tree_pointer_kernel<true, true, 8, false, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<true, true, 8, false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else if (a.pilp == 4) {
        err = prepare_launch(tree_pointer_kernel<false, true, 4, false, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 4, false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else if (a.pilp == 16) {
        err = prepare_launch(tree_pointer_kernel<false, true, 16, false, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 16, false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else {
        err = prepare_launch(tree_pointer_kernel<false, true, 8, false, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 8, false, true>), grid, dim3(TB), lds_pw, stream, a);
      }
    } else if (a.variant == VAR_POINTER_INLINE) {
      if (feat_lds && a.general) {
        err = prepare_launch(tree_pointer_kernel<true, true, 8, false, false, false, true>, lds_pw);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<true, true, 8, false, false, false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else if (feat_lds) {
        err = prepare_launch(tree_pointer_kernel<false, true, 8, false, false, false, true>, lds_pw);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<false, true, 8, false, false, false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else if (a.general) {
        err = prepare_launch(tree_pointer_kernel<true, false, 8, false, false, false, true>, lds_pw);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<true, false, 8, false, false, false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else {
        err = prepare_launch(tree_pointer_kernel<false, false, 8, false, false, false, true>, lds_pw);
        if (!err)
          hipLaunchKernelGGL((tree_pointer_kernel<false, false, 8, false, false, false, true>), grid, dim3(TB), lds_pw, stream, a);
      }
    } else if (a.variant == VAR_POINTER_USKIP || a.variant == VAR_POINTER_PEEL || a.variant == VAR_POINTER_LTOP) {
      return -4;  // features in LDS only
    } else if (a.general) {
      if (feat_lds && (a.variant & VAR_POINTER_MASKED)) {
        err = prepare_launch(tree_pointer_kernel<true, true, 8, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<true, true, 8, true>), grid, dim3(TB), lds_pw, stream, a);
      } else if (feat_lds) {
        err = prepare_launch(tree_pointer_kernel<true, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<true, true>), grid, dim3(TB), lds_pw, stream, a);
      } else {
        err = prepare_launch(tree_pointer_kernel<true, false>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<true, false>), grid, dim3(TB), lds_pw, stream, a);
      }
    } else {
      if (feat_lds && a.pilp == 2) {
        err = prepare_launch(tree_pointer_kernel<false, true, 2>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 2>), grid, dim3(TB), lds_pw, stream, a);
      } else if (feat_lds && (a.variant & VAR_POINTER_MASKED)) {
        err = prepare_launch(tree_pointer_kernel<false, true, 8, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 8, true>), grid, dim3(TB), lds_pw, stream, a);
      } else if (feat_lds && a.pilp == 16) {
        err = prepare_launch(tree_pointer_kernel<false, true, 16>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 16>), grid, dim3(TB), lds_pw, stream, a);
      } else if (feat_lds && a.pilp == 4) {
        err = prepare_launch(tree_pointer_kernel<false, true, 4>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true, 4>), grid, dim3(TB), lds_pw, stream, a);
      } else if (feat_lds) {
        err = prepare_launch(tree_pointer_kernel<false, true>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, true>), grid, dim3(TB), lds_pw, stream, a);
      } else {
        err = prepare_launch(tree_pointer_kernel<false, false>, lds_pw);
        if (!err) hipLaunchKernelGGL((tree_pointer_kernel<false, false>), grid, dim3(TB), lds_pw, stream, a);
      }
    }
  }
  if (err) return err;
  if (hipGetLastError() != hipSuccess) return -7;
  if (splits > 1) {
    dim3 g2((a.n_rows + TB - 1) / TB);
    hipLaunchKernelGGL(tree_reduce_kernel, g2, dim3(TB), 0, stream, a, splits);
    if (hipGetLastError() != hipSuccess) return -8;
  }
  return 0;
}

// Many tree launches in one host call (mixed-model micro-batches, runtime/grouped.py): args[i] is a
// complete argument block, meta[4 i ..] = {layout, depth, has_dr, splits}. Stops at the first
// failing launch and returns (its index + 1) << 8 | (-its code).
PMML_API int pmml_tree_launch_many(hipStream_t stream, const TreeArgs* args, const int* meta, int count) {
  for (int i = 0; i < count; ++i) {
    const int* m = meta + 4 * i;
    const int rc = pmml_tree_launch(stream, args + i, m[0], m[1], m[2], m[3]);
    if (rc != 0) return ((i + 1) << 8) | (-rc & 0xFF);
  }
  return 0;
}

PMML_API int pmml_tree_grouped_args_size() { return (int)sizeof(GroupedTreeArgs); }

// Split reduction alone (partial[splits][C + 1][n_rows] -> epilogue), for kernels outside this
// translation unit (tree_lds.hip).
PMML_API int pmml_tree_reduce(hipStream_t stream, const TreeArgs* args, int splits) {
  const TreeArgs& a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.C > 16 || splits < 1) return -3;
  dim3 g2((a.n_rows + TB - 1) / TB);
  hipLaunchKernelGGL(tree_reduce_kernel, g2, dim3(TB), 0, stream, a, splits);
  return hipGetLastError() == hipSuccess ? 0 : -8;
}

// ONE wide-kernel launch over a mixed-model slice (tree_grouped_wide_kernel). host_models: the
// host copies of the n entries' args (the kernel reads the device copies, g->models); they must
// share depth, leaf format, tile rows and accumulation mode. tiles: grid upper bound
// (ceil(rows / tile rows) + n). Returns 0 or a negative code (-20: entries disagree).
PMML_API int pmml_tree_launch_grouped(hipStream_t stream, const TreeArgs* host_models, int n,
                                      const GroupedTreeArgs* g, int depth, int tiles) {
  if (n <= 0 || tiles <= 0) return 0;
  if (g->n_models != n || g->F < 1) return -2;
  const TreeArgs& a0 = host_models[0];
  size_t lds = 0;
  for (int i = 0; i < n; ++i) {
    const TreeArgs& a = host_models[i];
    if ((a.variant & 3) == 0 || (a.variant & 3) != (a0.variant & 3) || a.rows_wide != a0.rows_wide ||
        a.mode != a0.mode)
      return -20;
    if (a.n_stage < 1 || a.n_stage > g->F || a.n_stage > (64 * 256) / a.rows_wide) return -4;
    if (a.C > 16) return -3;
    size_t need = 0;
    int chk = 0;
    switch (depth) {
      case 1: chk = wide_check<1>(a, need); break;
      case 2: chk = wide_check<2>(a, need); break;
      case 3: chk = wide_check<3>(a, need); break;
      case 4: chk = wide_check<4>(a, need); break;
      case 5: chk = wide_check<5>(a, need); break;
      case 6: chk = wide_check<6>(a, need); break;
      case 7: chk = wide_check<7>(a, need); break;
      case 8: chk = wide_check<8>(a, need); break;
      case 9: chk = wide_check<9>(a, need); break;
      case 10: chk = wide_check<10>(a, need); break;
      default: return -6;
    }
    if (chk) return chk;
    lds = need > lds ? need : lds;
  }
  int err = 0;
  switch (depth) {
    case 1: err = launch_grouped_d1(stream, a0, *g, tiles, lds); break;
    case 2: err = launch_grouped_d2(stream, a0, *g, tiles, lds); break;
    case 3: err = launch_grouped_d3(stream, a0, *g, tiles, lds); break;
    case 4: err = launch_grouped_d4(stream, a0, *g, tiles, lds); break;
    case 5: err = launch_grouped_d5(stream, a0, *g, tiles, lds); break;
    case 6: err = launch_grouped_d6(stream, a0, *g, tiles, lds); break;
    case 7: err = launch_grouped_d7(stream, a0, *g, tiles, lds); break;
    case 8: err = launch_grouped_d8(stream, a0, *g, tiles, lds); break;
    case 9: err = launch_grouped_d9(stream, a0, *g, tiles, lds); break;
    case 10: err = launch_grouped_d10(stream, a0, *g, tiles, lds); break;
    default: return -6;
  }
  if (err) return err;
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

PMML_API int pmml_tree_general_args_size() { return (int)sizeof(GenTreeArgs); }

// GENERAL layout launch (one split; grid over rows only).
PMML_API int pmml_tree_general_launch(hipStream_t stream, const GenTreeArgs* args) {
  GenTreeArgs ga = *args;
  TreeArgs& a = ga.t;
  if (a.n_rows <= 0) return 0;
  if (a.C > 16) return -3;
  a.partial = nullptr;
  a.trees_per_split = a.n_trees;
  dim3 grid((a.n_rows + TB - 1) / TB);
  const bool feat_lds = a.n_feat <= 64;
  const size_t acc_lds = a.general ? (size_t)a.C * TB * 4 : 0;
  const size_t lds = (feat_lds ? (size_t)a.n_feat * TB * 4 : 0) + TB * 4 + acc_lds;
  int err = 0;
  if (a.general) {
    if (feat_lds) {
      err = prepare_launch(tree_general_kernel<true, true>, lds);
      if (!err) hipLaunchKernelGGL((tree_general_kernel<true, true>), grid, dim3(TB), lds, stream, ga);
    } else {
      err = prepare_launch(tree_general_kernel<true, false>, lds);
      if (!err) hipLaunchKernelGGL((tree_general_kernel<true, false>), grid, dim3(TB), lds, stream, ga);
    }
  } else {
    if (feat_lds) {
      err = prepare_launch(tree_general_kernel<false, true>, lds);
      if (!err) hipLaunchKernelGGL((tree_general_kernel<false, true>), grid, dim3(TB), lds, stream, ga);
    } else {
      err = prepare_launch(tree_general_kernel<false, false>, lds);
      if (!err) hipLaunchKernelGGL((tree_general_kernel<false, false>), grid, dim3(TB), lds, stream, ga);
    }
  }
  if (err) return err;
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

PMML_API int pmml_tree_multi_args_size() { return (int)sizeof(MultiTreeArgs); }

// One launch of tree_pointer_multi_kernel over m->count segments (features staged in LDS: n_feat
// <= 64; general: the multi-slot accumulator variant, max_C the largest slot count).
PMML_API int pmml_tree_pointer_multi(hipStream_t stream, const MultiTreeArgs* args, int general, int max_C) {
  const MultiTreeArgs m = *args;
  if (m.n_rows <= 0 || m.count <= 0) return 0;
  if (m.n_feat < 1 || m.n_feat > 64 || m.count > 65535 || max_C < 0 || max_C > 16 || !m.segs || !m.S || !m.V || !m.sidx)
    return -4;
  const size_t lds = (size_t)m.n_feat * TB * 4 + TB * 4 + (general ? (size_t)max_C * TB * 4 : 0);
  const dim3 grid((m.n_rows + TB - 1) / TB, 1, m.count);
  int err;
  if (general) {
    err = prepare_launch(tree_pointer_multi_kernel<true>, lds);
    if (!err) hipLaunchKernelGGL((tree_pointer_multi_kernel<true>), grid, dim3(TB), lds, stream, m);
  } else {
    err = prepare_launch(tree_pointer_multi_kernel<false>, lds);
    if (!err) hipLaunchKernelGGL((tree_pointer_multi_kernel<false>), grid, dim3(TB), lds, stream, m);
  }
  if (err) return err;
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
