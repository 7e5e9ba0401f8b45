// HYBRID tree layout for deep forests (scikit-learn RandomForest with max_depth=None, deep GBDTs):
// a PERFECT head of the top H levels staged in LDS + a POINTER tail read from L2.
//
// The pointer kernel walks every level with a divergent 16-byte node gather from L2: a wave64
// touches up to 64 distinct nodes per load, and measured on MI355X it is bound by those gathers,
// not by their latency (profiles/r2af: 300 trees, depth <= 14 -> 3.68 ms per 1M rows; 8 walks in
// lock-step moved it by 1.5-3 %). Most of a walk happens near the root, where the PERFECT
// kernel's recipe applies:
//
//  * head: the top H levels of every tree padded to a perfect binary tree ({T, meta} uint2 per node
//    in heap order) plus 2^H exit codes (tail node index, or ~leaf). A tree shallower than H below
//    some node is padded with "always left" nodes (T = NaN: x >= NaN is false, no default-right bit)
//    so the walk still takes exactly H branch-free steps and lands on that leaf's exit;
//  * tail: COMPACT depth-first subtrees of everything below depth H — uint2 {x, meta} nodes, the
//    left child right after its parent, the right child at a relative offset in the meta, leaves
//    holding their value (P = 1) or payload row: half a pointer node's bytes per gathered level and
//    no separate leaf gather; 8 trees walked in lock-step per lane;
//  * chunks of trees' head records are copied cooperatively into LDS; rows stay stationary (one
//    lane = one row, features transposed [F][256] in LDS — conflict-free reads).
//
// Splits are canonicalised on the host to "go right iff x >= T" (exact for fp32 inputs). Head meta =
// feature byte offset in the LDS tile (index when features stay global) | bit 30 null-on-missing |
// bit 31 missing goes right; head exits = tail subtree root, or ~leaf. Tail meta = feature index
// (bits 0-7) | right offset (8-27) | bit 28 right child is a leaf | bit 29 left child is a leaf |
// bits 30/31 as in the head (runtime/hybrid.py packs both). A walk stops at its leaf's parent and
// the leaves of the 8 lock-step trees are read together afterwards: no serial extra round trip.
// Epilogue, slots and split mode are the pointer kernel's.
#include "tree_common.h"

namespace pmml_tree {
namespace {

struct HybridArgs {
  TreeArgs t;               // blob = tail nodes (uint4), leaves, rows, epilogue, outputs
  const uint32_t* heads;    // [n_trees][head_words]: (2^H - 1) uint2 nodes, then 2^H int exit codes
  int head_words;
  int tail_format;          // 0: COMPACT depth-first uint2 tail, 1: 16-byte BFS POINTER tail, 2: same + USKIP
};

template <bool FEAT_LDS>
__device__ __forceinline__ float hy_feature(const TreeArgs& a, const char* feat_lane, const float* xrow,
                                            uint32_t meta) {
  if (FEAT_LDS) return *reinterpret_cast<const float*>(feat_lane + (meta & 0xFFFFu));
  const int f = meta & 0xFFFFu;
  float x = xrow[f];
  if (a.prep) {
    bool b = false;
    x = prep_value(x, a.prep[f], &b);
  }
  return x;
}

template <bool GENERAL, bool FEAT_LDS, int H>
__global__ __launch_bounds__(TB, 2) void tree_hybrid_kernel(HybridArgs ha) {
  const TreeArgs& a = ha.t;
  constexpr int NI = (1 << H) - 1;
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + (FEAT_LDS ? a.n_feat * TB : 0));
  float* accl = reinterpret_cast<float*>(bad + TB);
  uint32_t* hbuf = reinterpret_cast<uint32_t*>(accl + (GENERAL ? a.C * TB : 0));
  const int tid = threadIdx.x;
  const int2 blk = tree_block(a);
  const int row0 = blk.x * TB;
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
  const uint2* tail = reinterpret_cast<const uint2*>(a.blob);
  const int tb = blk.y * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);
  const int rw = ha.head_words;
  const int CT = a.chunk_trees;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);
  float acc = 0.f;
  bool poisoned = false;
  constexpr int PILP = 8;
  for (int c0 = tb; c0 < te; c0 += CT) {
    const int nt = min(CT, te - c0);
    // cooperative copy of the chunk's head records (16-byte words; records are 16-byte padded)
    __syncthreads();
    {
      const uint4* src = reinterpret_cast<const uint4*>(ha.heads + (size_t)c0 * rw);
      uint4* dst = reinterpret_cast<uint4*>(hbuf);
      const int n16 = (nt * rw) >> 2;
      for (int i = tid; i < n16; i += TB) dst[i] = src[i];
    }
    __syncthreads();
    for (int k = 0; k < nt; k += PILP) {
      const int m = min(PILP, nt - k);
      uint32_t j[PILP];
      bool pz[PILP];
      const uint32_t* rec[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        j[i] = 0u;
        pz[i] = false;
        rec[i] = hbuf + (size_t)(k + min(i, m - 1)) * rw;  // surplus walks repeat the last tree
      }
      // head: exactly H branch-free levels per tree, PILP trees interleaved (LDS latency hiding)
#pragma unroll
      for (int d = 0; d < H; ++d) {
#pragma unroll
        for (int i = 0; i < PILP; ++i) {
          const uint2 nd = reinterpret_cast<const uint2*>(rec[i])[j[i]];
          const float x = hy_feature<FEAT_LDS>(a, feat_lane, xrow, nd.y);
          const bool isn = x != x;
          pz[i] = pz[i] || (isn && ((nd.y >> 30) & 1u));
          const uint32_t right = ((x >= __uint_as_float(nd.x)) || (isn && (nd.y >> 31))) ? 1u : 0u;
          j[i] = 2u * j[i] + 1u + right;
        }
      }
      // tail: COMPACT depth-first subtrees from L2 — {x, meta} uint2 per node, left child adjacent,
      // right child at +rel; a walk stops at the parent of its leaf (child-is-leaf bits 28/29)
      int code[PILP];
      bool done[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const int e = reinterpret_cast<const int*>(rec[i] + 2 * NI)[j[i] - NI];
        done[i] = pz[i] || i >= m || e < 0;
        code[i] = e < 0 ? ~e : e;
      }
      bool live = false;
#pragma unroll
      for (int i = 0; i < PILP; ++i) live = live || !done[i];
      while (live) {
        uint2 nd[PILP];
#pragma unroll
        for (int i = 0; i < PILP; ++i) nd[i] = tail[code[i]];
        live = false;
#pragma unroll
        for (int i = 0; i < PILP; ++i) {
          const bool act = !done[i];
          float x;
          if (FEAT_LDS) {
            x = *reinterpret_cast<const float*>(feat_lane + ((nd[i].y & 0xFFu) << 10));  // f * TB * 4
          } else {
            x = hy_feature<false>(a, feat_lane, xrow, nd[i].y & 0xFFu);
          }
          const bool isn = x != x;
          const bool nulled = act && isn && ((nd[i].y >> 30) & 1u);
          const bool right = (x >= __uint_as_float(nd[i].x)) || (isn && (nd[i].y >> 31));
          const int next = right ? code[i] + (int)((nd[i].y >> 8) & 0xFFFFFu) : code[i] + 1;
          const bool child_leaf = ((nd[i].y >> (right ? 28 : 29)) & 1u) != 0u;
          pz[i] = pz[i] || nulled;
          code[i] = (act && !nulled) ? next : code[i];
          done[i] = done[i] || nulled || child_leaf;
          live = live || !done[i];
        }
      }
      uint32_t val[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) val[i] = tail[code[i]].x;  // the leaves, read together
      for (int i = 0; i < PILP; ++i) {
        if (i >= m) break;
        if (pz[i]) {
          if (GENERAL) poisoned = true;
          else acc += __builtin_nanf("");
          continue;
        }
        if (GENERAL) {
          const int slot = a.tree_slot[c0 + k + i];
          for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += a.leaves[(size_t)val[i] * a.P + p];
        } else if (a.P > 1) {
          acc += a.leaves[(size_t)val[i] * a.P];
        } else {
          acc += __uint_as_float(val[i]);
        }
      }
    }
  }
  finish_row(a, acc, accl, blk.y, GENERAL, row, row_ok && !poisoned);
}

// HYBRID head + 16-byte POINTER tail (runtime/hybrid.py::pack_trees with H > 0): the head is the
// kernel above; the exits are pointer codes (tail node index, or ~leaf) and the tail walk is the
// lock-step BFS pointer walk (uint4 {T, meta, left code, right code}, siblings adjacent — the node
// format the lanes of a wave share cache lines best in, profiles/r3w). The top H levels, where
// every lane of the wave reads one of a handful of nodes, come from LDS (broadcast reads) instead
// of costing one vector-memory gather per level each; a walk slot that has ended in every lane of
// the wave issues no tail load (USKIP: wave-uniform ballot branch; otherwise finished walks re-load
// node 0 like the pointer kernel). Leaves are read after the tail loop.
template <bool GENERAL, bool FEAT_LDS, int H, bool USKIP>
__global__ __launch_bounds__(TB, 2) void tree_hybrid_ptr_kernel(HybridArgs ha) {
  const TreeArgs& a = ha.t;
  constexpr int NI = (1 << H) - 1;
  extern __shared__ __align__(16) uint32_t smem[];
  float* feat = reinterpret_cast<float*>(smem);
  int* bad = reinterpret_cast<int*>(smem + (FEAT_LDS ? a.n_feat * TB : 0));
  float* accl = reinterpret_cast<float*>(bad + TB);
  uint32_t* hbuf = reinterpret_cast<uint32_t*>(accl + (GENERAL ? a.C * TB : 0));
  const int tid = threadIdx.x;
  const int2 blk = tree_block(a);
  const int row0 = blk.x * TB;
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
  const uint4* nodes = reinterpret_cast<const uint4*>(a.blob);
  const int tb = blk.y * a.trees_per_split;
  const int te = min(a.n_trees, tb + a.trees_per_split);
  const int rw = ha.head_words;
  const int CT = a.chunk_trees;
  const char* feat_lane = reinterpret_cast<const char*>(feat + tid);
  float acc = 0.f;
  bool poisoned = false;
  constexpr int PILP = 8;
  for (int c0 = tb; c0 < te; c0 += CT) {
    const int nt = min(CT, te - c0);
    __syncthreads();
    {
      const uint4* src = reinterpret_cast<const uint4*>(ha.heads + (size_t)c0 * rw);
      uint4* dst = reinterpret_cast<uint4*>(hbuf);
      const int n16 = (nt * rw) >> 2;
      for (int i = tid; i < n16; i += TB) dst[i] = src[i];
    }
    __syncthreads();
    for (int k = 0; k < nt; k += PILP) {
      const int m = min(PILP, nt - k);
      uint32_t j[PILP];
      bool pz[PILP];
      const uint32_t* rec[PILP];
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        j[i] = 0u;
        pz[i] = false;
        rec[i] = hbuf + (size_t)(k + min(i, m - 1)) * rw;
      }
#pragma unroll
      for (int d = 0; d < H; ++d) {
#pragma unroll
        for (int i = 0; i < PILP; ++i) {
          const uint2 nd = reinterpret_cast<const uint2*>(rec[i])[j[i]];
          const float x = hy_feature<FEAT_LDS>(a, feat_lane, xrow, nd.y);
          const bool isn = x != x;
          pz[i] = pz[i] || (isn && ((nd.y >> 30) & 1u));
          const uint32_t right = ((x >= __uint_as_float(nd.x)) || (isn && (nd.y >> 31))) ? 1u : 0u;
          j[i] = 2u * j[i] + 1u + right;
        }
      }
      int code[PILP];
      bool live = false;
#pragma unroll
      for (int i = 0; i < PILP; ++i) {
        const int e = reinterpret_cast<const int*>(rec[i] + 2 * NI)[j[i] - NI];
        code[i] = (pz[i] || i >= m) ? -1 : e;  // a poisoned / surplus walk carries no leaf
        live = live || code[i] >= 0;
      }
      while (live) {
        uint4 nd[PILP];
        bool any[PILP];
#pragma unroll
        for (int i = 0; i < PILP; ++i) any[i] = !USKIP || __builtin_amdgcn_ballot_w64(code[i] >= 0) != 0ull;
#pragma unroll
        for (int i = 0; i < PILP; ++i) {
          if (USKIP) {
            nd[i] = make_uint4(0u, 0u, 0u, 0u);
            if (any[i]) nd[i] = nodes[max(code[i], 0)];
          } else {
            nd[i] = nodes[max(code[i], 0)];
          }
        }
        live = false;
#pragma unroll
        for (int i = 0; i < PILP; ++i) {
          if (USKIP && !any[i]) continue;
          const bool act = code[i] >= 0;
          float x;
          if (FEAT_LDS) {
            x = *reinterpret_cast<const float*>(feat_lane + (nd[i].y & 0xFFFFu));
          } else {
            x = hy_feature<false>(a, feat_lane, xrow, nd[i].y & 0xFFFFu);
          }
          const bool isn = x != x;
          const bool nulled = act && isn && ((nd[i].y >> 30) & 1u);
          const bool right = (x >= __uint_as_float(nd[i].x)) || (isn && (nd[i].y >> 31));
          const int nc = right ? (int)nd[i].w : (int)nd[i].z;
          pz[i] = pz[i] || nulled;
          code[i] = act ? (nulled ? -1 : nc) : code[i];
          live = live || code[i] >= 0;
        }
      }
      for (int i = 0; i < PILP; ++i) {
        if (i >= m) break;
        if (pz[i]) {
          if (GENERAL) poisoned = true;
          else acc += __builtin_nanf("");
          continue;
        }
        const int leaf = ~code[i];
        if (GENERAL) {
          const int slot = a.tree_slot[c0 + k + i];
          for (int p = 0; p < a.P; ++p) accl[(slot + p) * TB + tid] += a.leaves[(size_t)leaf * a.P + p];
        } else {
          acc += a.leaves[leaf];
        }
      }
    }
  }
  finish_row(a, acc, accl, blk.y, GENERAL, row, row_ok && !poisoned);
}

// Split-mode reduction (same partial layout as the pointer kernel).
__global__ __launch_bounds__(TB) void tree_hybrid_reduce_kernel(TreeArgs a, int splits) {
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

template <bool GENERAL, bool FEAT_LDS, int H>
int launch_hybrid_t(hipStream_t stream, const HybridArgs& ha, dim3 grid, size_t lds) {
  if constexpr (H > 4) {
    if (ha.tail_format != 0) return -6;  // pointer tails: heads of 2-4 levels (profiles/r3ar)
  } else {
  if (ha.tail_format == 1) {  // 16-byte pointer tail, clamped loads
    int err = prepare_launch(tree_hybrid_ptr_kernel<GENERAL, FEAT_LDS, H, false>, lds);
    if (err) return err;
    hipLaunchKernelGGL((tree_hybrid_ptr_kernel<GENERAL, FEAT_LDS, H, false>), grid, dim3(TB), lds, stream, ha);
    return 0;
  }
  if (ha.tail_format == 2) {  // 16-byte pointer tail, wave-uniform skip of finished slots
    int err = prepare_launch(tree_hybrid_ptr_kernel<GENERAL, FEAT_LDS, H, true>, lds);
    if (err) return err;
    hipLaunchKernelGGL((tree_hybrid_ptr_kernel<GENERAL, FEAT_LDS, H, true>), grid, dim3(TB), lds, stream, ha);
    return 0;
  }
  }
  int err = prepare_launch(tree_hybrid_kernel<GENERAL, FEAT_LDS, H>, lds);
  if (err) return err;
  hipLaunchKernelGGL((tree_hybrid_kernel<GENERAL, FEAT_LDS, H>), grid, dim3(TB), lds, stream, ha);
  return 0;
}

template <int H>
int launch_hybrid_h(hipStream_t stream, const HybridArgs& ha, dim3 grid, size_t lds, bool general, bool feat_lds) {
  if (general) {
    return feat_lds ? launch_hybrid_t<true, true, H>(stream, ha, grid, lds)
                    : launch_hybrid_t<true, false, H>(stream, ha, grid, lds);
  }
  return feat_lds ? launch_hybrid_t<false, true, H>(stream, ha, grid, lds)
                  : launch_hybrid_t<false, false, H>(stream, ha, grid, lds);
}

}  // namespace
}  // namespace pmml_tree

using namespace pmml_tree;

PMML_API int pmml_tree_hybrid_args_size() { return (int)sizeof(HybridArgs); }

// head_depth in {2, 3, 4, 6, 8, 10} (2 and 3: pointer tail only, 6-10: compact tail only); splits >= 1 (grid.y tree groups, > 1 needs t.partial).
PMML_API int pmml_tree_hybrid_launch(hipStream_t stream, const HybridArgs* args, int head_depth, int splits) {
  HybridArgs ha = *args;
  TreeArgs& a = ha.t;
  if (a.n_rows <= 0) return 0;
  if (splits < 1) splits = 1;
  if (splits > 1 && a.partial == nullptr) return -2;
  if (splits == 1) a.partial = nullptr;
  if (a.C > 16) return -3;
  const int words = 2 * ((1 << head_depth) - 1) + (1 << head_depth);
  if (ha.head_words < words || (ha.head_words & 3) != 0) return -4;
  if (a.chunk_trees < 1) return -4;
  a.trees_per_split = (a.n_trees + splits - 1) / splits;
  if (a.n_trees > 0) splits = (a.n_trees + a.trees_per_split - 1) / a.trees_per_split;  // no empty split
  if (splits == 1) a.partial = nullptr;
  const bool feat_lds = a.n_feat <= 64;
  const size_t lds = (feat_lds ? (size_t)a.n_feat * TB * 4 : 0) + TB * 4 + (a.general ? (size_t)a.C * TB * 4 : 0) +
                     (size_t)a.chunk_trees * ha.head_words * 4;
  if (lds > 160 * 1024) return -5;
  const int row_blocks = (a.n_rows + TB - 1) / TB;
  if (splits == 1) a.xcd_split = 0;
  if (a.xcd_split > 0) a.xcd_split = splits;
  if (a.xcd_split > 0 && (long long)row_blocks * splits > 0x7FFFFFFFLL) return -11;
  dim3 grid = a.xcd_split > 0 ? dim3(row_blocks * splits) : dim3(row_blocks, splits);
  if (ha.tail_format < 0 || ha.tail_format > 2) return -4;
  if (head_depth < 4 && ha.tail_format == 0) return -6;
  int err;
  switch (head_depth) {
    case 2: err = launch_hybrid_h<2>(stream, ha, grid, lds, a.general != 0, feat_lds); break;
    case 3: err = launch_hybrid_h<3>(stream, ha, grid, lds, a.general != 0, feat_lds); break;
    case 4: err = launch_hybrid_h<4>(stream, ha, grid, lds, a.general != 0, feat_lds); break;
    case 6: err = launch_hybrid_h<6>(stream, ha, grid, lds, a.general != 0, feat_lds); break;
    case 8: err = launch_hybrid_h<8>(stream, ha, grid, lds, a.general != 0, feat_lds); break;
    case 10: err = launch_hybrid_h<10>(stream, ha, grid, lds, a.general != 0, feat_lds); break;
    default: return -6;
  }
  if (err) return err;
  if (hipGetLastError() != hipSuccess) return -7;
  if (splits > 1) {
    dim3 g2((a.n_rows + TB - 1) / TB);
    hipLaunchKernelGGL(tree_hybrid_reduce_kernel, g2, dim3(TB), 0, stream, a, splits);
    if (hipGetLastError() != hipSuccess) return -8;
  }
  return 0;
}
