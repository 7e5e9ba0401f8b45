// LDS-resident walk of deep forests (runtime/hybrid.py::pack_lds_chunks, TreePlan node_format="lds").
//
// The pointer walk of a deep forest (300 trees x depth 14, ~5000 nodes a tree, 12 MB) is bound by
// the vector L1's tag rate: below the top levels every lane of a gather sits on its own 128-byte
// line, about one line per clock per CU (profiles/r3w, r4j). LDS serves a wave64 `ds_read_b64` of
// random addresses in a few cycles instead, so here the trees are walked out of LDS:
//
//  * the forest is cut into XCD slices (contiguous tree ranges of about equal bytes; workgroup L
//    takes row tile L / S and slice L % S, so with S = 8 slice s is always walked on XCD s and its
//    1/8 of the forest stays in that XCD's 4 MiB L2) and every slice into chunks of whole trees
//    that fit the LDS chunk buffer (compact 8-byte BFS slots, tree.hip::tree_compact_kernel format);
//  * a workgroup (1024 threads) owns a ROWS-row tile: the rows' prepared features sit in LDS as
//    [F][ROWS] planes (a lane's read feat[f][lane] is conflict free whatever f), the thread groups
//    G = 1024 / ROWS split every chunk's trees round-robin; a lane walks its trees one after
//    another, starting the next the step the last one ends (LDS has no shared-line benefit that
//    would favour lock-step walks; profiles/r5d: lock-step batches over a chunk's 2-3 trees were
//    VALU bound, 7x the pointer walk's instructions);
//  * chunks stream global -> VGPRs -> LDS: the whole next chunk (<= 96 KiB, 6 x 16 B per thread)
//    and its roots are loaded into registers while the current chunk is walked, so a chunk switch
//    costs two barriers and the LDS stores, not an L2 round trip (profiles/r5e: the synchronous
//    remainder of each chunk copy was most of the time);
//  * each (tile, slice) workgroup writes the slice's partial row sums (+ an invalid flag) in the
//    split layout [S][C + 1][n], and tree_reduce_kernel (tree.hip) applies the epilogue.
//
// Sums: tree order within a thread group, groups in order, slices in order (not the single
// tree-order sum of the pointer kernel: results agree to fp32 rounding, the oracle check is the
// contract). Votes / class slots (GENERAL): per-thread register accumulators, C <= 8.

#include "tree_common.h"

namespace pmml_tree {
namespace {

struct LdsTreeArgs {
  TreeArgs t;
  const int4* chunks;      // [n_chunks] {aligned slot start (even), uint4 count, tree begin, tree end}
  const int* slice_chunk;  // [n_slices + 1] chunk range of every tree slice
  int n_slices, chunk_u4;  // uint4 capacity of the LDS chunk buffer
  int rows, pad;           // row tile: 512 or 256
};

constexpr int LT = 1024;
constexpr int LCMAX = 8;
constexpr int LPREF = 6;  // uint4 per thread: the WHOLE next chunk is prefetched into registers
                          // during a walk (chunk_u4 <= LPREF * LT, host-enforced)
constexpr int LROOTS = 256;  // trees per chunk (host-enforced): their chunk-local roots in LDS

template <bool GENERAL, int ROWS>
__global__ __launch_bounds__(LT, 1) void tree_lds_kernel(LdsTreeArgs la) {
  const TreeArgs& a = la.t;
  constexpr int G = LT / ROWS;
  extern __shared__ __align__(16) uint32_t smem[];
  const int F = a.n_feat;
  const int CA = GENERAL ? a.C : 1;
  float* feat = reinterpret_cast<float*>(smem);           // [F][ROWS]
  int* bad = reinterpret_cast<int*>(feat + F * ROWS);     // [ROWS]
  float* part = reinterpret_cast<float*>(bad + ROWS);     // [G][CA][ROWS]
  int* roots_l = reinterpret_cast<int*>(part + G * CA * ROWS);    // [LROOTS] chunk-local roots
  uint4* cbuf = reinterpret_cast<uint4*>(roots_l + LROOTS);
  const uint2* nodes = reinterpret_cast<const uint2*>(cbuf);
  const int tid = threadIdx.x;
  const int S = la.n_slices;
  const int L = blockIdx.x;
  const int tile = L / S, slice = L % S;
  const int row0 = tile * ROWS;
  const int r = tid % ROWS;
  const int g = __builtin_amdgcn_readfirstlane(tid / ROWS);
  const int row = row0 + r;

  // ---- stage the tile's prepared features: [F][ROWS] planes
  for (int e = tid; e < ROWS; e += LT) bad[e] = 0;
  __syncthreads();
  {
    const bool vec4 = (F & 3) == 0 && (a.ldx & 3) == 0 && (reinterpret_cast<uintptr_t>(a.X) & 15) == 0;
    const int F4 = (F + 3) >> 2;
    for (int e = tid; vec4 && e < ROWS * F4; e += LT) {
      const int q = e >> 5;
      const int rh = q / F4;
      const int fq = q - rh * F4;
      const int rr = 32 * rh + (e & 31);
      const int rw = row0 + rr;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rw < a.n_rows) v = *reinterpret_cast<const float4*>(a.X + (size_t)rw * a.ldx + 4 * fq);
      bool b = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int f = 4 * fq + k;
        float x = k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
        if (rw < a.n_rows && a.prep) x = prep_value(x, a.prep[f], &b);
        feat[f * ROWS + rr] = x;
      }
      if (b) bad[rr] = 1;
    }
    for (int e = tid; !vec4 && e < ROWS * F; e += LT) {
      const int q = e >> 5;
      const int rh = q / F;
      const int f = q - rh * F;
      const int rr = 32 * rh + (e & 31);
      const int rw = row0 + rr;
      float x = 0.f;
      bool b = false;
      if (rw < a.n_rows) {
        x = a.X[(size_t)rw * a.ldx + f];
        if (a.prep) x = prep_value(x, a.prep[f], &b);
      }
      feat[f * ROWS + rr] = x;
      if (b) bad[rr] = 1;
    }
  }

  const char* feat_lane = reinterpret_cast<const char*>(feat + r);
  float acc = 0.f;
  float accv[LCMAX];
#pragma unroll
  for (int k = 0; k < LCMAX; ++k) accv[k] = 0.f;
  bool poisoned = false;

  const int c0 = la.slice_chunk[slice], c1 = la.slice_chunk[slice + 1];
  // named registers (an array here was put in scratch by the compiler); rtp: the chunk's root
  uint4 pf0, pf1, pf2, pf3, pf4, pf5;
  int rtp = 0;
#define LDS_PREFETCH(CH)                                                                      \
  {                                                                                           \
    const uint4* src_ = reinterpret_cast<const uint4*>(a.blob) + ((CH).x >> 1);             \
    const int last_ = max((CH).y - 1, 0); /* clamped, unconditional loads */                 \
    pf0 = src_[min(tid, last_)];                                                              \
    pf1 = src_[min(tid + LT, last_)];                                                         \
    pf2 = src_[min(tid + 2 * LT, last_)];                                                     \
    pf3 = src_[min(tid + 3 * LT, last_)];                                                     \
    pf4 = src_[min(tid + 4 * LT, last_)];                                                     \
    pf5 = src_[min(tid + 5 * LT, last_)];                                                     \
    rtp = a.roots[min((CH).z + tid, max((CH).w - 1, 0))];                                    \
  }
  int4 ch = c0 < c1 ? la.chunks[c0] : make_int4(0, 0, 0, 0);
  LDS_PREFETCH(ch)  // first chunk (consumed below like every later chunk)
  for (int c = c0; c < c1; ++c) {
    // ---- chunk c into LDS: the prefetched head from registers, the rest straight through
    __syncthreads();  // the previous chunk's walks are done (and, first time, the feature planes)
    {
      if (tid < ch.w - ch.z)  // chunk-local root codes (~slot: single-leaf tree)
        roots_l[tid] = rtp >= 0 ? rtp - ch.x : ~((~rtp) - ch.x);
      if (tid < ch.y) cbuf[tid] = pf0;
      if (tid + LT < ch.y) cbuf[tid + LT] = pf1;
      if (tid + 2 * LT < ch.y) cbuf[tid + 2 * LT] = pf2;
      if (tid + 3 * LT < ch.y) cbuf[tid + 3 * LT] = pf3;
      if (tid + 4 * LT < ch.y) cbuf[tid + 4 * LT] = pf4;
      if (tid + 5 * LT < ch.y) cbuf[tid + 5 * LT] = pf5;
    }
    __syncthreads();
    const int tb = ch.z, te = ch.w;
    // ---- next chunk's head into registers: its loads overlap this chunk's walks
    int4 nch = make_int4(0, 0, 0, 0);
    if (c + 1 < c1) {
      nch = la.chunks[c + 1];
      LDS_PREFETCH(nch)
    }
    // ---- walk this group's trees of the chunk (tb + g, tb + g + G, ...) one after another per
    // lane: a lane whose walk ends adds its leaf and starts its next tree at once (the chunk's
    // roots sit in LDS), so a wave iterates about the SUM of its lanes' path lengths rather than
    // the deepest walk of every lock-step batch; leaves still add in tree order per lane.
    {
      int t = tb + g;
      int pos = 0;
      bool act = false, pz = false;
      if (t < te) {
        const int rc = roots_l[t - tb];
        pos = rc >= 0 ? rc : ~rc;
        act = rc >= 0;  // a single-leaf tree starts on its leaf
      }
      while (t < te) {
        if (act) {
          const uint2 nd = nodes[pos];
          const uint32_t m = nd.y;
          const float x = *reinterpret_cast<const float*>(feat_lane + (m & 63u) * (ROWS * 4));
          const bool isn = (x != x);
          const bool nulled = isn && ((m >> 30) & 1u);
          const bool right = (x >= __uint_as_float(nd.x)) || (isn && (m >> 31));
          const int child = pos + (int)((m >> 8) & 0x3FFFFFu) + (right ? 1 : 0);
          const bool leaf = right ? ((m >> 7) & 1u) : ((m >> 6) & 1u);
          pz = pz || nulled;
          pos = nulled ? pos : child;
          act = !nulled && !leaf;
        } else {
          if (pz) {
            if (GENERAL) poisoned = true;
            else acc += __builtin_nanf("");
          } else {
            const uint32_t lv = nodes[pos].x;
            if (GENERAL) {
              const int slot = a.tree_slot[t];
              const float* lp = a.leaves + (size_t)lv * a.P;
#pragma unroll
              for (int k = 0; k < LCMAX; ++k) {
                const int p = k - slot;
                if (p >= 0 && p < a.P) accv[k] += lp[p];
              }
            } else {
              acc += __uint_as_float(lv);
            }
          }
          t += G;
          pz = false;
          if (t < te) {
            const int rc = roots_l[t - tb];
            pos = rc >= 0 ? rc : ~rc;
            act = rc >= 0;
          }
        }
      }
    }
    ch = nch;
  }
#undef LDS_PREFETCH

  // ---- combine the thread groups (in order), then this slice's partial for the row
  if (GENERAL) {
#pragma unroll
    for (int k = 0; k < LCMAX; ++k)
      if (k < CA) part[(g * CA + k) * ROWS + r] = accv[k];
  } else {
    part[g * ROWS + r] = acc;
  }
  if (poisoned) bad[r] = 1;  // benign race: every writer stores 1
  __syncthreads();
  if (g != 0 || row >= a.n_rows) return;
  bool row_ok = bad[r] == 0;
  if (a.row_valid_in) row_ok = row_ok && a.row_valid_in[row];
  const size_t stride = (size_t)a.n_rows;
  if (a.partial) {
    float* pb = a.partial + (size_t)slice * (CA + 1) * stride;
    for (int k = 0; k < CA; ++k) {
      float s = 0.f;
      for (int q = 0; q < G; ++q) s += part[(q * CA + k) * ROWS + r];
      pb[k * stride + row] = s;
    }
    pb[CA * stride + row] = row_ok ? 0.f : 1.f;
    return;
  }
  if (GENERAL) {
    float tot[LCMAX];
#pragma unroll
    for (int k = 0; k < LCMAX; ++k) {
      tot[k] = 0.f;
      if (k < CA)
        for (int q = 0; q < G; ++q) tot[k] += part[(q * CA + k) * ROWS + r];
    }
    apply_epilogue(a.epi, [&](int c) {
      float v = tot[0];
#pragma unroll
      for (int k = 1; k < LCMAX; ++k) v = (c == k) ? tot[k] : v;
      return v;
    }, row_ok, row, a.n_rows, a.score, a.valid, a.probs);
  } else {
    float s = 0.f;
    for (int q = 0; q < G; ++q) s += part[q * ROWS + r];
    apply_epilogue(a.epi, [&](int) { return s; }, row_ok, row, a.n_rows, a.score, a.valid, a.probs);
  }
}

template <bool GENERAL, int ROWS>
int launch_lds(hipStream_t st, const LdsTreeArgs& la, dim3 grid, size_t lds) {
  auto k = tree_lds_kernel<GENERAL, ROWS>;
  int err = prepare_launch(k, lds);
  if (!err) hipLaunchKernelGGL(k, grid, dim3(LT), lds, st, la);
  return err;
}

}  // namespace
}  // namespace pmml_tree

using namespace pmml_tree;

PMML_API int pmml_tree_reduce(hipStream_t stream, const TreeArgs* args, int splits);

PMML_API int pmml_tree_lds_args_size() { return (int)sizeof(LdsTreeArgs); }

// LDS bytes of one launch (0: does not fit).
PMML_API long long pmml_tree_lds_bytes(int n_feat, int rows, int C, int general, int chunk_u4) {
  const int G = LT / rows;
  const int CA = general ? C : 1;
  const long long head = (long long)n_feat * rows * 4 + rows * 4 + (long long)G * CA * rows * 4 + LROOTS * 4;
  const long long total = head + (long long)chunk_u4 * 16;
  return total <= 160 * 1024 ? total : 0;
}

// One launch over all rows x slices (+ the split reduction when n_slices > 1: t.partial must hold
// n_slices x (C' + 1) x n_rows floats, C' = general ? C : 1).
PMML_API int pmml_tree_lds_launch(hipStream_t stream, const LdsTreeArgs* args) {
  LdsTreeArgs la = *args;
  TreeArgs& a = la.t;
  if (a.n_rows <= 0) return 0;
  if (la.n_slices < 1 || la.chunk_u4 < 1 || la.chunk_u4 > LPREF * LT) return -2;
  if (!(la.rows == 512 || la.rows == 256)) return -4;
  if (a.n_feat < 1 || a.n_feat > 64) return -4;
  if (a.general && (a.C > LCMAX || a.P > LCMAX)) return -3;
  if (la.n_slices > 1 && a.partial == nullptr) return -2;
  if (la.n_slices == 1) a.partial = nullptr;
  const long long lds = pmml_tree_lds_bytes(a.n_feat, la.rows, a.C, a.general, la.chunk_u4);
  if (lds <= 0) return -5;
  const long long tiles = (a.n_rows + la.rows - 1) / la.rows;
  if (tiles * la.n_slices > 0x7FFFFFFFLL) return -11;
  const dim3 grid((unsigned)(tiles * la.n_slices));
  int err;
  if (la.rows == 512) {
    err = a.general ? launch_lds<true, 512>(stream, la, grid, (size_t)lds) : launch_lds<false, 512>(stream, la, grid, (size_t)lds);
  } else {
    err = a.general ? launch_lds<true, 256>(stream, la, grid, (size_t)lds) : launch_lds<false, 256>(stream, la, grid, (size_t)lds);
  }
  if (err) return err;
  if (hipGetLastError() != hipSuccess) return -7;
  if (la.n_slices > 1) {
    TreeArgs ra = a;
    if (!a.general) ra.C = 1;  // sums: one partial plane + the flag plane
    return pmml_tree_reduce(stream, &ra, la.n_slices);
  }
  return 0;
}
