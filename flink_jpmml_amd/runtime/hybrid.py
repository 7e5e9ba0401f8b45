"""Vectorised packers of the POINTER and HYBRID tree layouts (``ops/csrc/tree_hybrid.hip``).

* POINTER: every internal node is a ``uint4 {T bits, meta, left code, right code}`` (code >= 0:
  node index, < 0: ``~leaf``); ``roots[t]`` is tree t's root code.
* HYBRID(H): the top ``H`` levels of each tree become a PERFECT head record staged in LDS —
  ``2^H - 1`` ``uint2 {T bits, meta}`` nodes in heap order, then ``2^H`` int32 exit codes (tail node
  or ``~leaf``), padded to 16 bytes — and everything deeper is POINTER tail. A leaf above depth H
  is reached through "always left" padding nodes (``T = NaN``: ``x >= NaN`` is false, no
  default-right bit) and owns the exit its leftmost descendant would have.

Splits are canonicalised to "go right iff ``x >= T``" with fp32-exact thresholds
(:func:`~flink_jpmml_amd.runtime.plans.canonical_threshold`); meta = feature byte offset in the
``[F][256]`` LDS tile (feature index when the features stay in global memory) | bit 30 null-on-
missing | bit 31 missing goes right. Per tree the work is a handful of numpy operations per level
(no per-node Python): a 300-tree depth-14 forest packs in well under a second.
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

TB = 256
NAN_BITS = np.uint32(0x7FC00000)


def head_words(H: int) -> int:
    w = 2 * ((1 << H) - 1) + (1 << H)
    return (w + 3) // 4 * 4


INLINE_LEFT_BIT, INLINE_RIGHT_BIT = 29, 28  # tree.hip pointer_walk<..., INL>


def pack_trees(trees, weights: List[float], P: int, H: int, feat_lds: bool, order: str = "bfs",
               inline_leaves: bool = False) -> Tuple[Optional[np.ndarray], np.ndarray, np.ndarray, np.ndarray, bool]:
    """``(heads [n_trees, head_words] u32 or None when H == 0, tail nodes [n, 4] u32,
    leaves [n_leaves, P] f32, root codes [n_trees] i32, has_default_right)``.

    ``order``: node / leaf order inside a tree. ``"bfs"`` (default) stores the tree level by level
    with the two children of every node adjacent: the lock-step walk moves all lanes of a wave
    through the same level of the same tree together, so their loads share cache lines (the
    top levels of a tree sit in a few lines; a node's two children always share one). ``"dfs"``:
    the lowered tree's own (preorder) order.

    ``inline_leaves`` (pointer layout, ``VAR_POINTER_INLINE``): a leaf child's payload is stored
    in its parent's child field with meta bit 29 (left) / 28 (right) set -- the fp32 bits of the
    weighted leaf value (``P == 1``), or the class index of a unit one-hot vote (``P > 1``); other
    leaves keep their ``~leaf`` code into the leaf table."""
    if order not in ("bfs", "dfs"):
        raise ValueError("order must be 'bfs' or 'dfs'")
    from .plans import _canonical_vec

    NI, NL = (1 << H) - 1, 1 << H
    rw = head_words(H) if H else 0
    heads = np.zeros((len(trees), rw), dtype=np.uint32) if H else None
    tails: List[np.ndarray] = []
    leaves: List[np.ndarray] = []
    roots = np.zeros(len(trees), dtype=np.int32)
    n_tail = n_leaf = 0
    has_dr = False
    for ti, (t, w) in enumerate(zip(trees, weights)):
        feat = np.asarray(t.feature, dtype=np.int64)
        n = feat.shape[0]
        internal = feat >= 0
        T, swap = _canonical_vec(np.asarray(t.op), np.asarray(t.threshold, dtype=np.float64))
        left, right = np.asarray(t.left, dtype=np.int64), np.asarray(t.right, dtype=np.int64)
        dflt_left = np.asarray(t.default_left, dtype=bool)
        lc = np.where(swap, right, left)
        rc = np.where(swap, left, right)
        dr = np.where(swap, dflt_left, ~dflt_left) & internal
        has_dr = has_dr or bool(dr.any())
        f = np.where(internal, feat, 0)
        off = (f * TB * 4) if feat_lds else f
        meta = (off.astype(np.uint64) | (dr.astype(np.uint64) << 31)
                | ((np.uint64(1) << 30) * np.uint64(bool(t.null_missing)) * internal.astype(np.uint64)))
        meta = meta.astype(np.uint32)
        # level and heap position (heap positions only within the head)
        lvl = np.full(n, -1, dtype=np.int64)
        heap = np.full(n, -1, dtype=np.int64)
        lvl[0], heap[0] = 0, 0
        rank = np.arange(n, dtype=np.int64)  # storage order key ("dfs": the lowered order)
        if order == "bfs":
            rank[0], seen = 0, 1
        frontier = np.array([0], dtype=np.int64)
        L = 0
        while frontier.size:
            fi = frontier[internal[frontier]]
            if fi.size == 0:
                break
            a, b = lc[fi], rc[fi]
            lvl[a] = lvl[b] = L + 1
            if L + 1 <= H:
                heap[a] = 2 * heap[fi] + 1
                heap[b] = 2 * heap[fi] + 2
            frontier = np.stack([a, b], axis=1).reshape(-1)  # siblings adjacent
            if order == "bfs":
                rank[frontier] = seen + np.arange(frontier.size)
                seen += frontier.size
            L += 1
        is_leaf = ~internal
        tail_mask = internal & (lvl >= H)
        leaf_rank = np.zeros(n, dtype=np.int64)
        tail_rank = np.zeros(n, dtype=np.int64)
        lk_sorted = np.nonzero(is_leaf)[0]
        lk_sorted = lk_sorted[np.argsort(rank[lk_sorted], kind="stable")]
        leaf_rank[lk_sorted] = np.arange(lk_sorted.size)
        tk_sorted = np.nonzero(tail_mask)[0]
        tk_sorted = tk_sorted[np.argsort(rank[tk_sorted], kind="stable")]
        tail_rank[tk_sorted] = np.arange(tk_sorted.size)
        code = np.where(is_leaf, ~(n_leaf + leaf_rank), n_tail + tail_rank).astype(np.int64)
        # leaves (storage order), weighted payloads
        lk = lk_sorted
        if t.leaf_probs is not None and P > 1:
            vals = np.asarray(t.leaf_probs, dtype=np.float64)[lk, :P] * w
        else:
            vals = np.asarray(t.leaf_value, dtype=np.float64)[lk, None] * w
        leaves.append(vals)
        # tail nodes (storage order)
        tk = tk_sorted
        if tk.size:
            nd = np.empty((tk.size, 4), dtype=np.uint32)
            nd[:, 0] = T[tk].view(np.uint32)
            nd[:, 1] = meta[tk]
            nd[:, 2] = code[lc[tk]].astype(np.int32).view(np.uint32)
            nd[:, 3] = code[rc[tk]].astype(np.int32).view(np.uint32)
            if inline_leaves and H == 0:
                pay = np.zeros(n, dtype=np.uint32)
                ok = np.zeros(n, dtype=bool)
                if P == 1:
                    pay[lk] = vals[:, 0].astype(np.float32).view(np.uint32)
                    ok[lk] = True
                else:  # unit one-hot votes: the class index
                    one = (np.count_nonzero(vals, axis=1) == 1) & (vals.max(axis=1) == 1.0)
                    pay[lk[one]] = np.argmax(vals[one], axis=1).astype(np.uint32)
                    ok[lk[one]] = True
                for col, child, bit in ((2, lc[tk], INLINE_LEFT_BIT), (3, rc[tk], INLINE_RIGHT_BIT)):
                    m = ok[child]
                    nd[m, col] = pay[child[m]]
                    nd[m, 1] |= np.uint32(1 << bit)
            tails.append(nd)
        roots[ti] = code[0]  # POINTER layout entry (the HYBRID walk starts in the head)
        if H:
            rec = heads[ti]
            hT = np.full(NI, NAN_BITS, dtype=np.uint32)
            hM = np.zeros(NI, dtype=np.uint32)
            hk = np.nonzero(internal & (lvl < H))[0]
            hT[heap[hk]] = T[hk].view(np.uint32)
            hM[heap[hk]] = meta[hk]
            exits = np.full(NL, int(code[lk[0]]) if lk.size else 0, dtype=np.int64)
            at = np.nonzero(lvl == H)[0]
            exits[heap[at] - NI] = code[at]
            up = lk[lvl[lk] < H]
            e = (heap[up] + 1) * (np.int64(1) << (H - lvl[up])) - 1 - NI
            exits[e] = code[up]
            rec[0: 2 * NI: 2] = hT
            rec[1: 2 * NI: 2] = hM
            rec[2 * NI: 2 * NI + NL] = exits.astype(np.int32).view(np.uint32)
        n_leaf += lk.size
        n_tail += tk.size
    nodes = np.concatenate(tails) if tails else np.zeros((1, 4), np.uint32)
    lv = np.concatenate(leaves).astype(np.float32) if leaves else np.zeros((1, P), np.float32)
    return heads, nodes, lv, roots, has_dr


def _levels_and_heap(lc, rc, internal, H):
    n = lc.shape[0]
    lvl = np.full(n, -1, dtype=np.int64)
    heap = np.full(n, -1, dtype=np.int64)
    lvl[0], heap[0] = 0, 0
    frontier = np.array([0], dtype=np.int64)
    by_level = [frontier]
    L = 0
    while frontier.size:
        fi = frontier[internal[frontier]]
        if fi.size == 0:
            break
        a, b = lc[fi], rc[fi]
        lvl[a] = lvl[b] = L + 1
        if L + 1 <= H:
            heap[a] = 2 * heap[fi] + 1
            heap[b] = 2 * heap[fi] + 2
        frontier = np.concatenate([a, b])
        by_level.append(frontier)
        L += 1
    return lvl, heap, by_level


COMPACT_REL_BITS = 20  # right-child offset field of a compact tail node


def pack_hybrid_compact(trees, weights: List[float], P: int, H: int, n_features: int):
    """HYBRID layout with a COMPACT tail: ``uint2 {x, meta}`` nodes in depth-first preorder per
    subtree, the left child right after its parent and the right child at ``+ rel``:

    * internal: ``x`` = threshold bits; meta = feature index (bits 0-7) | right-child offset
      (bits 8-27) | bit 28 right child is a leaf | bit 29 left child is a leaf | bit 30
      null-on-missing | bit 31 missing goes right;
    * leaf: ``x`` = the weighted leaf value (P = 1) or the leaf's payload row (P > 1).

    Half the bytes of a POINTER node per visited level. The walk stops at the parent of a leaf
    (the child-is-leaf bits): the leaf itself is read once after the lock-step loop, with the
    other trees' leaves, never as an extra serial L2 round trip. Head exits hold the index of a
    tail subtree root, or ``~index`` of a leaf (a leaf above depth H).
    Returns ``(heads, tail [n, 2] u32, payload [n_leaves, P] f32 or None, has_dr)``; raises
    ``ValueError`` when a subtree outgrows the offset field or the features the index field."""
    from .plans import _canonical_vec

    if n_features > 256:
        raise ValueError("compact tail nodes index at most 256 features")
    NI, NL = (1 << H) - 1, 1 << H
    rw = head_words(H)
    heads = np.zeros((len(trees), rw), dtype=np.uint32)
    tails: List[np.ndarray] = []
    payload: List[np.ndarray] = []
    n_tail = n_leaf = 0
    has_dr = False
    for ti, (t, w) in enumerate(zip(trees, weights)):
        feat = np.asarray(t.feature, dtype=np.int64)
        n = feat.shape[0]
        internal = feat >= 0
        T, swap = _canonical_vec(np.asarray(t.op), np.asarray(t.threshold, dtype=np.float64))
        left, right = np.asarray(t.left, dtype=np.int64), np.asarray(t.right, dtype=np.int64)
        dflt_left = np.asarray(t.default_left, dtype=bool)
        lc = np.where(swap, right, left)
        rc = np.where(swap, left, right)
        dr = np.where(swap, dflt_left, ~dflt_left) & internal
        has_dr = has_dr or bool(dr.any())
        lvl, heap, by_level = _levels_and_heap(lc, rc, internal, H)
        # subtree sizes bottom-up, then depth-first positions top-down (left child adjacent)
        size = np.ones(n, dtype=np.int64)
        for nodes in reversed(by_level):
            k = nodes[internal[nodes]]
            size[k] = 1 + size[lc[k]] + size[rc[k]]
        is_leaf = ~internal
        tail_node = lvl >= H
        roots = np.nonzero((lvl == H) | (is_leaf & (lvl < H)))[0]
        pos = np.full(n, -1, dtype=np.int64)
        pos[roots] = np.concatenate([[0], np.cumsum(size[roots])[:-1]]) if roots.size else roots
        for nodes in by_level:
            k = nodes[internal[nodes] & (pos[nodes] >= 0)]
            pos[lc[k]] = pos[k] + 1
            pos[rc[k]] = pos[k] + 1 + size[lc[k]]
        members = np.nonzero((pos >= 0) & (tail_node | is_leaf))[0]
        m = int(size[roots].sum()) if roots.size else 0
        if members.size != m:
            raise AssertionError("hybrid tail packing lost nodes")
        nd = np.zeros((m, 2), dtype=np.uint32)
        ik = members[internal[members]]
        rel = pos[rc[ik]] - pos[ik]
        if rel.size and rel.max() >= (1 << COMPACT_REL_BITS):
            raise ValueError("subtree too large for the compact tail's right-child offset")
        nd[pos[ik], 0] = T[ik].view(np.uint32)
        nd[pos[ik], 1] = (feat[ik].astype(np.uint64) | (rel.astype(np.uint64) << 8)
                          | (is_leaf[rc[ik]].astype(np.uint64) << 28) | (is_leaf[lc[ik]].astype(np.uint64) << 29)
                          | (dr[ik].astype(np.uint64) << 31)
                          | (np.uint64(bool(t.null_missing)) << np.uint64(30))).astype(np.uint32)
        lk = members[is_leaf[members]]
        if P > 1:
            probs = np.asarray(t.leaf_probs, dtype=np.float64)[lk, :P] * w
            payload.append(probs)
            nd[pos[lk], 0] = (n_leaf + np.arange(lk.size)).astype(np.uint32)
            n_leaf += lk.size
        else:
            nd[pos[lk], 0] = (np.asarray(t.leaf_value, dtype=np.float64)[lk] * w).astype(np.float32).view(np.uint32)
        tails.append(nd)
        code = np.where(is_leaf, ~(n_tail + pos), n_tail + pos)  # exits: ~leaf / subtree root
        # head
        rec = heads[ti]
        hT = np.full(NI, NAN_BITS, dtype=np.uint32)
        hM = np.zeros(NI, dtype=np.uint32)
        hk = np.nonzero(internal & (lvl < H))[0]
        hT[heap[hk]] = T[hk].view(np.uint32)
        hM[heap[hk]] = (feat[hk] * TB * 4 if n_features <= 64 else feat[hk]).astype(np.uint32) \
            | (dr[hk].astype(np.uint32) << np.uint32(31)) | (np.uint32(bool(t.null_missing)) << np.uint32(30))
        exits = np.full(NL, n_tail, dtype=np.int64)  # unreachable exits: any valid tail node
        at = np.nonzero(lvl == H)[0]
        exits[heap[at] - NI] = code[at]
        up = np.nonzero(is_leaf & (lvl < H))[0]
        exits[(heap[up] + 1) * (np.int64(1) << (H - lvl[up])) - 1 - NI] = code[up]
        rec[0: 2 * NI: 2] = hT
        rec[1: 2 * NI: 2] = hM
        rec[2 * NI: 2 * NI + NL] = exits.astype(np.int32).view(np.uint32)
        n_tail += m
    tail = np.concatenate(tails) if tails else np.zeros((1, 2), np.uint32)
    pay = np.concatenate(payload).astype(np.float32) if payload else None
    return heads, tail, pay, has_dr


__all__ = ["head_words", "pack_hybrid_compact", "pack_trees"]


# --------------------------------------------------------------------------- compact BFS pointer layout

C2_FEAT_MASK = 63        # bits 0-5: feature (LDS plane index)
C2_LLEAF, C2_RLEAF = 1 << 6, 1 << 7
C2_REL_SHIFT, C2_REL_BITS = 8, 22
C2_NULL, C2_DR = 1 << 30, 1 << 31


def pack_compact_bfs(trees, weights: List[float], P: int):
    """8-byte pointer nodes, each tree stored level by level with the two children of a node in
    adjacent slots (``tree.hip::tree_compact_kernel``).

    A slot is ``uint2 {x, meta}``. Internal node: ``x`` = canonical fp32 threshold ("go right iff
    x >= T"), ``meta`` = feature | left-is-leaf | right-is-leaf | (first child - this slot) << 8 |
    null-on-missing | default-right. Leaf slot: ``x`` = the weighted leaf value (P == 1) or the
    row of ``leaves`` (P > 1). The walk stops on the parent of a leaf and reads ``x`` of the
    leaf slot after the lock-step loop. Root codes: slot index, or ``~slot`` for a single-leaf tree.

    Returns ``(nodes [n, 2] u32, leaves [n_leaves, P] f32 or None, roots [n_trees] i32, has_dr)``;
    ``ValueError`` when a tree has more than 2^22 slots or a feature index >= 64."""
    from .plans import _canonical_vec

    slots_all: List[np.ndarray] = []
    leaves_all: List[np.ndarray] = []
    roots = np.zeros(len(trees), dtype=np.int32)
    base = n_leaf = 0
    has_dr = False
    for ti, (t, w) in enumerate(zip(trees, weights)):
        feat = np.asarray(t.feature, dtype=np.int64)
        n = feat.shape[0]
        internal = feat >= 0
        if internal.any() and feat[internal].max() > C2_FEAT_MASK:
            raise ValueError("compact pointer layout: feature index >= 64")
        T, swap = _canonical_vec(np.asarray(t.op), np.asarray(t.threshold, dtype=np.float64))
        left, right = np.asarray(t.left, dtype=np.int64), np.asarray(t.right, dtype=np.int64)
        lc = np.where(swap, right, left)
        rc = np.where(swap, left, right)
        dr = np.where(swap, np.asarray(t.default_left, bool), ~np.asarray(t.default_left, bool)) & internal
        has_dr = has_dr or bool(dr.any())
        # slots: root, then per level the (left, right) pairs of the level's internal nodes
        pos = np.full(n, -1, dtype=np.int64)
        pos[0] = 0
        first = np.full(n, -1, dtype=np.int64)
        nxt = 1
        frontier = np.array([0], dtype=np.int64)
        while frontier.size:
            fi = frontier[internal[frontier]]
            if fi.size == 0:
                break
            first[fi] = nxt + 2 * np.arange(fi.size)
            pos[lc[fi]] = first[fi]
            pos[rc[fi]] = first[fi] + 1
            nxt += 2 * fi.size
            frontier = np.stack([lc[fi], rc[fi]], axis=1).reshape(-1)
        if nxt > (1 << C2_REL_BITS):
            raise ValueError("compact pointer layout: tree larger than 2^22 slots")
        slots = np.zeros((nxt, 2), dtype=np.uint32)
        ik = np.nonzero(internal & (pos >= 0))[0]
        rel = (first[ik] - pos[ik]).astype(np.uint64)
        meta = (feat[ik].astype(np.uint64)
                | (np.uint64(C2_LLEAF) * (~internal[lc[ik]]).astype(np.uint64))
                | (np.uint64(C2_RLEAF) * (~internal[rc[ik]]).astype(np.uint64))
                | (rel << np.uint64(C2_REL_SHIFT))
                | (np.uint64(C2_NULL) * np.uint64(bool(t.null_missing)))
                | (np.uint64(C2_DR) * dr[ik].astype(np.uint64)))
        slots[pos[ik], 0] = T[ik].view(np.uint32)
        slots[pos[ik], 1] = meta.astype(np.uint32)
        lk = np.nonzero(~internal & (pos >= 0))[0]
        if P == 1:
            vals = (np.asarray(t.leaf_value, dtype=np.float64)[lk] * w).astype(np.float32)
            slots[pos[lk], 0] = vals.view(np.uint32)
        else:
            lk = lk[np.argsort(pos[lk], kind="stable")]
            vals = np.asarray(t.leaf_probs, dtype=np.float64)[lk, :P] * w
            slots[pos[lk], 0] = (n_leaf + np.arange(lk.size)).astype(np.uint32)
            leaves_all.append(vals)
            n_leaf += lk.size
        roots[ti] = base if internal[0] else ~base
        slots_all.append(slots)
        base += nxt
    nodes = np.concatenate(slots_all) if slots_all else np.zeros((1, 2), np.uint32)
    leaves = np.concatenate(leaves_all).astype(np.float32) if leaves_all else None
    return nodes, leaves, roots, has_dr


def pack_lds_chunks(n_slots: int, roots: np.ndarray, chunk_u4: int, n_slices: int = 8, max_trees: int = 256):
    """Chunk table of the LDS-resident walk (``tree_lds.hip``) over a :func:`pack_compact_bfs`
    forest: trees in order, cut into ``n_slices`` contiguous slices of about equal slots (one per
    XCD) and every slice into chunks of whole trees whose slots — copied from an even start, as
    16-byte words — fit ``chunk_u4`` uint4 of LDS (and at most ``max_trees`` trees: their roots are
    staged in LDS too).

    Returns ``(chunks int32[n, 4] {even slot start, uint4 count, tree begin, tree end},
    slice_chunk int32[S + 1])``; ``ValueError`` when one tree alone exceeds the buffer."""
    roots = np.asarray(roots, dtype=np.int64)
    T = roots.size
    start = np.where(roots >= 0, roots, ~roots)
    end = np.append(start[1:], n_slots)
    sizes = end - start

    def u4(a: int, b: int) -> int:  # uint4 words covering slots [a, b) copied from an even start
        return (b - (a & ~1) + 1) // 2

    if T and max(u4(int(a), int(b)) for a, b in zip(start, end)) > chunk_u4:
        raise ValueError("a tree exceeds the LDS chunk buffer")
    # slices first (contiguous tree ranges of ~equal slots), then greedy chunks inside each
    S = int(max(1, min(n_slices, T)))
    cum = np.cumsum(sizes)
    cuts = [0] + [int(np.searchsorted(cum, cum[-1] * k / S, side="left")) + 1 for k in range(1, S)] + [T]
    cuts = sorted(set(min(max(c, 0), T) for c in cuts))
    chunks: List[tuple] = []
    slice_chunk = [0]
    for a, b in zip(cuts[:-1], cuts[1:]):
        t = a
        while t < b:
            e = t + 1
            while e < b and e - t < max_trees and u4(int(start[t]), int(end[e])) <= chunk_u4:
                e += 1
            chunks.append((int(start[t]) & ~1, u4(int(start[t]), int(end[e - 1])), t, e))
            t = e
        slice_chunk.append(len(chunks))
    return np.asarray(chunks, dtype=np.int32).reshape(-1, 4), np.asarray(slice_chunk, dtype=np.int32)


# --------------------------------------------------------------------------- SUPER pointer layout
# Two tree levels per 16-byte load (``tree.hip::tree_super_kernel``). The deep-forest walk is bound
# by the vector memory pipe's cost per load INSTRUCTION (profiles/r3u: ~20 TA cycles per 64-lane
# gather whether the lanes fetch 8 or 16 bytes, whether finished lanes are masked or not), so the
# lever is fewer loads per walk: a super-node packs a split and both of its children's splits.

SN_FEAT_BITS = 5               # feature index fields (LDS planes): f_j bits 0-4, f_l 5-9, f_r 10-14
SN_LLEAF, SN_RLEAF, SN_SELF = 1 << 15, 1 << 16, 1 << 17
SN_DRJ, SN_DRL, SN_DRR = 1 << 18, 1 << 19, 1 << 20
SN_BLOCK_SHIFT, SN_BLOCK_BITS = 21, 11
SN_NULL_ROOT = np.uint32(1 << 31)  # root word flag: the tree's nullPrediction missing strategy


def pack_super(trees, weights: List[float], P: int):
    """``uint4`` super-node slots, per tree: slot 0 the root super-node, then blocks of 4 slots
    (block b = slots 1 + 4b .. 4 + 4b) holding the four grandchildren of one super-node, blocks in
    breadth-first order.

    Internal super-node at node j with children l, r: ``x`` = T_j, ``y`` = T_l (or l's leaf value
    when l is a leaf), ``z`` = T_r (or r's leaf value), ``w`` = f_j | f_l << 5 | f_r << 10 |
    l-is-leaf | r-is-leaf | default-right bits of j, l, r | grandchild block << 21. The walk at j
    picks c = r if x_j >= T_j, then the grandchild 2 (c == r) + (x_c >= T_c) of the block; a leaf
    child ends the walk with its value in hand, a leaf grandchild is a slot flagged SN_SELF whose
    ``x`` is the value. Leaf values: the weighted fp32 value (P == 1) or the row of ``leaves``.
    Canonical splits ("go right iff x >= T", fp32-exact thresholds) as the other layouts.

    Returns ``(nodes [n, 4] u32, leaves [n_leaves, P] f32 or None, roots [n_trees] u32 (slot |
    SN_NULL_ROOT), has_dr)``; ``ValueError`` when a feature index is >= 32 or a tree needs more
    than 2^11 blocks."""
    from .plans import _canonical_vec

    slots_all: List[np.ndarray] = []
    leaves_all: List[np.ndarray] = []
    roots = np.zeros(len(trees), dtype=np.uint32)
    base = n_leaf = 0
    has_dr = False
    fmax = (1 << SN_FEAT_BITS) - 1
    for ti, (t, w) in enumerate(zip(trees, weights)):
        feat = np.asarray(t.feature, dtype=np.int64)
        n = feat.shape[0]
        internal = feat >= 0
        if internal.any() and feat[internal].max() > fmax:
            raise ValueError(f"super layout: feature index > {fmax}")
        T, swap = _canonical_vec(np.asarray(t.op), np.asarray(t.threshold, dtype=np.float64))
        left, right = np.asarray(t.left, dtype=np.int64), np.asarray(t.right, dtype=np.int64)
        lc = np.where(swap, right, left)
        rc = np.where(swap, left, right)
        dr = np.where(swap, np.asarray(t.default_left, bool), ~np.asarray(t.default_left, bool)) & internal
        has_dr = has_dr or bool(dr.any())
        # leaf payloads: value bits (P == 1) or payload row (P > 1), one per leaf node
        leafword = np.zeros(n, dtype=np.uint32)
        lk = np.nonzero(~internal)[0]
        if P == 1:
            leafword[lk] = (np.asarray(t.leaf_value, dtype=np.float64)[lk] * w).astype(np.float32).view(np.uint32)
        else:
            leafword[lk] = (n_leaf + np.arange(lk.size)).astype(np.uint32)
            leaves_all.append(np.asarray(t.leaf_probs, dtype=np.float64)[lk, :P] * w)
            n_leaf += lk.size
        fi = np.where(internal, feat, 0).astype(np.uint64)
        Tw = T.view(np.uint32) if T.dtype == np.float32 else T.astype(np.float32).view(np.uint32)
        word = np.where(internal, Tw, leafword)  # y / z of a parent: T of an internal child, else its value
        # breadth-first over super-nodes
        recs: List[np.ndarray] = []
        slot_of = {}
        frontier = np.array([0], dtype=np.int64)   # super-node roots (or leaf slots) of this level
        fslots = np.array([0], dtype=np.int64)
        n_slots, n_blocks = 1, 0
        while frontier.size:
            rec = np.zeros((frontier.size, 4), dtype=np.uint32)
            isl = ~internal[frontier]
            rec[isl, 0] = leafword[frontier[isl]]
            rec[isl, 3] = SN_SELF
            j = frontier[~isl]
            l, r = lc[j], rc[j]
            il, ir = internal[l], internal[r]
            need = il | ir
            blk = np.full(j.size, 0, dtype=np.int64)
            blk[need] = n_blocks + np.arange(int(need.sum()))
            n_blocks += int(need.sum())
            if n_blocks > (1 << SN_BLOCK_BITS):
                raise ValueError("super layout: tree needs more than 2^11 grandchild blocks")
            w3 = (fi[j] | (fi[l] * il) << np.uint64(5) | (fi[r] * ir) << np.uint64(10)
                  | np.uint64(SN_LLEAF) * (~il).astype(np.uint64) | np.uint64(SN_RLEAF) * (~ir).astype(np.uint64)
                  | np.uint64(SN_DRJ) * dr[j].astype(np.uint64) | np.uint64(SN_DRL) * (dr[l] & il).astype(np.uint64)
                  | np.uint64(SN_DRR) * (dr[r] & ir).astype(np.uint64)
                  | blk.astype(np.uint64) << np.uint64(SN_BLOCK_SHIFT))
            rec[~isl, 0] = Tw[j]
            rec[~isl, 1] = word[l]
            rec[~isl, 2] = word[r]
            rec[~isl, 3] = w3.astype(np.uint32)
            recs.append((fslots, rec))
            # next level: the 4 grandchild slots of every super-node that has a block
            jn, bn = j[need], blk[need]
            ln, rn = lc[jn], rc[jn]
            kids, kslots = [], []
            for k, (c, ok) in enumerate(((ln, internal[ln]), (rn, internal[rn]))):
                for h, g in enumerate((lc, rc)):
                    sel = ok
                    kids.append(g[c[sel]])
                    kslots.append(1 + 4 * bn[sel] + 2 * k + h)
            frontier = np.concatenate(kids) if kids else np.zeros(0, np.int64)
            fslots = np.concatenate(kslots) if kslots else np.zeros(0, np.int64)
            n_slots = max(n_slots, 1 + 4 * n_blocks)
        slots = np.zeros((n_slots, 4), dtype=np.uint32)
        for s, rec in recs:
            slots[s] = rec
        roots[ti] = np.uint32(base) | (SN_NULL_ROOT if bool(t.null_missing) else np.uint32(0))
        slots_all.append(slots)
        base += n_slots
        if base >= (1 << 31):
            raise ValueError("super layout: more than 2^31 slots")
    nodes = np.concatenate(slots_all) if slots_all else np.zeros((1, 4), np.uint32)
    leaves = np.concatenate(leaves_all).astype(np.float32) if leaves_all else None
    return nodes, leaves, roots, has_dr


__all__ += ["pack_compact_bfs", "pack_super"]


# ------------------------------------------------------------------------------------------------
# RANK3: three tree levels per 16-byte record on per-feature threshold ranks (tree.hip
# tree_rank3_kernel). Words (every field inside one 32-bit word, so the walk extracts it with one
# shift-and-mask): x = ranks of nodes 0-3 (8 bits each); y = ranks of nodes 4-6 | live-exit mask
# << 24; z = features of nodes 0-5 (5 bits each) | default-right of nodes 0 / 1 at bits 30 / 31;
# w = feature of node 6 | default-right of nodes 2-6 at bits 5-9 | exit block offset from the
# tree's base slot << 10 (21 bits) | leaf slot << 31 (a leaf slot's x = weighted value / leaf row). Only the live exits of a record are stored: exit e sits at
# block + popcount(mask & ((1 << e) - 1)); a block never straddles a 128-byte line.
RK_NAN = 255        # a missing value's rank (csrc RK_NAN)
RK_NEVER = 255      # a padding node's rank: never "right" (ranks of values are <= 254)
RK_MAX_UNIQUE = 254
RK_LINE = 8         # 16-byte slots per 128-byte line
RK_OFF_BITS = 21
# bit of node n's feature / default-right flag in hi = words 2-3 (every field inside one 32-bit word)
_RK_FSHIFT = np.array([0, 5, 10, 15, 20, 25, 32], dtype=np.uint64)
_RK_DSHIFT = np.array([30, 31, 37, 38, 39, 40, 41], dtype=np.uint64)


def rank_tables(trees, n_features: int):
    """Per feature: the sorted unique canonical (fp32, "go right iff x >= T") thresholds of every
    split. Returns ``(uniq list, thr [F, stride] f32, cnt [F] i32)``; ``ValueError`` beyond
    RK_MAX_UNIQUE thresholds on a feature (XGBoost / LightGBM histogram models have <= 255 bins)."""
    from .plans import _canonical_vec

    per = [[] for _ in range(n_features)]
    for t in trees:
        feat = np.asarray(t.feature, dtype=np.int64)
        internal = feat >= 0
        if not internal.any():
            continue
        T, _ = _canonical_vec(np.asarray(t.op)[internal], np.asarray(t.threshold, dtype=np.float64)[internal])
        for f in np.unique(feat[internal]):
            per[int(f)].append(T[feat[internal] == f])
    uniq = [np.unique(np.concatenate(p)).astype(np.float32) if p else np.zeros(0, np.float32) for p in per]
    cnt = np.array([u.size for u in uniq], dtype=np.int32)
    if cnt.size and cnt.max() > RK_MAX_UNIQUE:
        raise ValueError(f"rank3 layout: {int(cnt.max())} unique thresholds on one feature (max {RK_MAX_UNIQUE})")
    stride = max(1, int(cnt.max()) if cnt.size else 1)
    thr = np.full((n_features, stride), np.inf, dtype=np.float32)
    for f, u in enumerate(uniq):
        thr[f, : u.size] = u
    return uniq, thr, cnt


_K_N, _K_P, _K_X = 0, 1, 2  # record entries: a real split, a pad carrying a leaf left, a dead pad


def _rank3_tree(feat, internal, lc, rc, dr, rank, t, w, P, leaf0):
    """One tree's RANK3 slots, a breadth-first level of records at a time (numpy over the level;
    only the line-padded block allocation is a scalar loop). Same slots, same leaf-row order as
    the reference builder of :func:`pack_rank3`. Returns ``(slots [n, 4] u32, leaf rows or None)``."""
    leafvals = []

    def leaf_words(nodes):
        nodes = np.asarray(nodes, dtype=np.int64)
        wv = np.zeros(nodes.size, dtype=np.uint32)
        if P == 1:
            wv[:] = (np.asarray(t.leaf_value, dtype=np.float64)[nodes] * w).astype(np.float32).view(np.uint32)
        else:
            base = leaf0 + sum(v.shape[0] for v in leafvals)
            wv[:] = base + np.arange(nodes.size, dtype=np.uint32)
            leafvals.append(np.asarray(t.leaf_probs, dtype=np.float64)[nodes, :P] * w)
        return wv

    chunks = []  # (slot indices, [k, 4] words)
    if not internal[0]:
        s0 = np.zeros((1, 4), np.uint32)
        s0[0, 0] = leaf_words([0])[0]
        s0[0, 3] = np.uint32(1 << 31)
        arr = np.zeros((RK_LINE, 4), np.uint32)
        arr[0] = s0[0]
        return arr, (np.concatenate(leafvals) if leafvals else None)
    n_slots = 1
    fj = np.array([0], dtype=np.int64)    # record roots of this level
    fs = np.array([0], dtype=np.int64)    # their slots

    def below(k, v):
        """children entries of entries (k, v): ([..., 2] kinds, [..., 2] values)."""
        isn = k == _K_N
        vv = np.where(isn, v, 0)
        cl, cr = lc[vv], rc[vv]
        kl = np.where(isn, np.where(internal[cl], _K_N, _K_P), np.where(k == _K_P, _K_P, _K_X))
        kr = np.where(isn, np.where(internal[cr], _K_N, _K_P), _K_X)
        vl = np.where(isn, cl, np.where(k == _K_P, v, -1))
        vr = np.where(isn, cr, -1)
        return np.stack([kl, kr], -1), np.stack([vl, vr], -1)

    while fj.size:
        K = fj.size
        k0 = np.full((K, 1), _K_N)
        v0 = fj[:, None]
        k1, v1 = below(k0[:, 0], v0[:, 0])                              # [K, 2]
        k2, v2 = below(k1.reshape(-1), v1.reshape(-1))                  # [2K, 2]
        k2, v2 = k2.reshape(K, 4), v2.reshape(K, 4)
        kind = np.concatenate([k0, k1, k2], 1)                          # [K, 7]
        val = np.concatenate([v0, v1, v2], 1)
        vv = np.where(k2 == _K_N, v2, 0)
        ex = np.stack([np.where(k2 == _K_N, lc[vv], np.where(k2 == _K_P, v2, -1)),
                       np.where(k2 == _K_N, rc[vv], -1)], -1).reshape(K, 8)
        live = ex >= 0
        nl = live.sum(1)
        bases = np.empty(K, dtype=np.int64)
        pos = n_slots
        for i in range(K):  # a block never straddles a line
            if pos % RK_LINE + nl[i] > RK_LINE:
                pos += RK_LINE - pos % RK_LINE
            bases[i] = pos
            pos += nl[i]
        n_slots = pos
        if n_slots >= (1 << RK_OFF_BITS):
            raise ValueError("rank3 layout: tree needs more than 2^21 slots")
        isn = kind == _K_N
        vn = np.where(isn, val, 0)
        r = np.where(isn, rank[vn], np.uint64(RK_NEVER)).astype(np.uint64)
        f = np.where(isn, feat[vn], 0).astype(np.uint64)
        d = np.where(isn, dr[vn], False).astype(np.uint64)
        sh = np.arange(7, dtype=np.uint64)
        mask = (live.astype(np.uint64) << np.arange(8, dtype=np.uint64)).sum(1)
        lo = (r << (np.uint64(8) * sh)).sum(1) | (mask << np.uint64(56))
        hi = (f << _RK_FSHIFT).sum(1) | (d << _RK_DSHIFT).sum(1) | (bases.astype(np.uint64) << np.uint64(42))
        rec = np.stack([lo & np.uint64(0xFFFFFFFF), lo >> np.uint64(32), hi & np.uint64(0xFFFFFFFF),
                        hi >> np.uint64(32)], 1).astype(np.uint32)
        chunks.append((fs, rec))
        # exits, row-major (the reference builder's queue order): records -> next level, leaves -> slots
        es = bases[:, None] + np.cumsum(live, 1) - 1
        child, cslot = ex[live], es[live]
        isr = internal[child]
        if (~isr).any():
            lw = np.zeros((int((~isr).sum()), 4), np.uint32)
            lw[:, 0] = leaf_words(child[~isr])
            lw[:, 3] = np.uint32(1 << 31)
            chunks.append((cslot[~isr], lw))
        fj, fs = child[isr], cslot[isr]
    n_slots += (-n_slots) % RK_LINE
    arr = np.zeros((n_slots, 4), dtype=np.uint32)
    for sl, words in chunks:
        arr[sl] = words
    return arr, (np.concatenate(leafvals) if leafvals else None)


def pack_rank3(trees, weights: List[float], P: int, n_features: int, vectorized: bool = True):
    """RANK3 records of every tree: per tree, slot 0 is the root record (or the root leaf slot),
    then the exit blocks in breadth-first order; a record's block holds its live exits (the next
    records and leaf slots) and never straddles a 128-byte line.

    Returns ``(nodes [n, 4] u32, leaves [n_leaves, P] f32 or None, roots [n_trees] i32 (base slot of
    each tree), thr [F, stride] f32, cnt [F] i32, has_dr)``; ``ValueError`` when a feature index
    is >= 32, a feature has more than 254 unique thresholds, a tree is null-on-missing or needs
    more than 2^21 slots. ``vectorized=False``: the record-by-record reference builder (the same
    arrays, tests/test_rank3.py)."""
    from .plans import _canonical_vec

    if n_features > 32:
        raise ValueError("rank3 layout: more than 32 features")
    if any(t.null_missing for t in trees):
        raise ValueError("rank3 layout: null-on-missing trees")
    uniq, thr, cnt = rank_tables(trees, n_features)
    slots_all: List[np.ndarray] = []
    leaves_all: List[np.ndarray] = []
    roots = np.zeros(len(trees), dtype=np.int32)
    total = n_leaf = 0
    has_dr = False
    for ti, (t, w) in enumerate(zip(trees, weights)):
        feat = np.asarray(t.feature, dtype=np.int64)
        internal = feat >= 0
        T, swap = _canonical_vec(np.asarray(t.op), np.asarray(t.threshold, dtype=np.float64))
        left, right = np.asarray(t.left, dtype=np.int64), np.asarray(t.right, dtype=np.int64)
        lc = np.where(swap, right, left)
        rc = np.where(swap, left, right)
        dr = np.where(swap, np.asarray(t.default_left, bool), ~np.asarray(t.default_left, bool)) & internal
        has_dr = has_dr or bool(dr.any())
        rank = np.zeros(feat.shape[0], dtype=np.uint64)
        for f in np.unique(feat[internal]):
            m = feat == f
            rank[m] = (np.searchsorted(uniq[int(f)], T[m]) + 1).astype(np.uint64)
        if vectorized:
            arr, lv = _rank3_tree(feat, internal, lc, rc, dr, rank, t, w, P, n_leaf)
            if lv is not None:
                leaves_all.append(lv)
                n_leaf += lv.shape[0]
            roots[ti] = total
            total += arr.shape[0]
            if total >= (1 << 31):
                raise ValueError("rank3 layout: more than 2^31 slots")
            slots_all.append(arr)
            continue
        n_slots = 1  # slot 0: the root
        slots = {}

        def leaf_slot(k: int) -> np.ndarray:
            nonlocal n_leaf
            s = np.zeros(4, dtype=np.uint32)
            if P == 1:
                s[0] = np.float32(float(t.leaf_value[k]) * w).view(np.uint32)
            else:
                s[0] = n_leaf
                leaves_all.append(np.asarray(t.leaf_probs[k], dtype=np.float64)[:P] * w)
                n_leaf += 1
            s[3] = np.uint32(1 << 31)
            return s

        queue = [(0, 0)]  # (node, slot)
        while queue:
            k, s = queue.pop(0)
            if not internal[k]:
                slots[s] = leaf_slot(k)
                continue
            # the 7 nodes of this record: ("n", node) a real split, ("p", leaf) a never-right pad
            # carrying a leaf down its left side, ("x", -1) a pad nobody reaches
            def below(entries):
                out = []
                for kind, v in entries:
                    if kind == "n":
                        out += [("n", int(c)) if internal[c] else ("p", int(c)) for c in (lc[v], rc[v])]
                    elif kind == "p":
                        out += [("p", v), ("x", -1)]
                    else:
                        out += [("x", -1), ("x", -1)]
                return out

            lvl1 = below([("n", k)])
            lvl2 = below(lvl1)
            nodes7 = [("n", k)] + lvl1 + lvl2
            exits = []
            for kind, v in lvl2:  # exit e = 2 * (third-level entry) + right
                if kind == "n":
                    exits += [int(lc[v]), int(rc[v])]
                elif kind == "p":
                    exits += [v, -1]
                else:
                    exits += [-1, -1]
            live = [c for c in exits if c >= 0]
            mask = sum(1 << e for e, c in enumerate(exits) if c >= 0)
            if n_slots % RK_LINE + len(live) > RK_LINE:  # keep the block inside one line
                n_slots += RK_LINE - n_slots % RK_LINE
            base = n_slots
            n_slots += len(live)
            if base >= (1 << RK_OFF_BITS):
                raise ValueError("rank3 layout: tree needs more than 2^21 slots")
            lo = mask << 56
            hi = 0
            for n, (kind, v) in enumerate(nodes7):
                if kind == "n":
                    lo |= int(rank[v]) << (8 * n)
                    hi |= int(feat[v]) << int(_RK_FSHIFT[n])
                    hi |= int(dr[v]) << int(_RK_DSHIFT[n])
                else:
                    lo |= RK_NEVER << (8 * n)
            hi |= base << 42
            rec = np.array([lo & 0xFFFFFFFF, lo >> 32, hi & 0xFFFFFFFF, hi >> 32], dtype=np.uint64).astype(np.uint32)
            slots[s] = rec
            for j, c in enumerate(live):
                queue.append((c, base + j))
        n_slots += (-n_slots) % RK_LINE  # the next tree starts on a line
        arr = np.zeros((n_slots, 4), dtype=np.uint32)
        for s, v in slots.items():
            arr[s] = v
        roots[ti] = total
        total += n_slots
        if total >= (1 << 31):
            raise ValueError("rank3 layout: more than 2^31 slots")
        slots_all.append(arr)
    nodes = np.concatenate(slots_all) if slots_all else np.zeros((1, 4), np.uint32)
    leaves = np.concatenate([np.atleast_2d(x) for x in leaves_all]).astype(np.float32) if leaves_all else None
    return nodes, leaves, roots, thr, cnt, has_dr


__all__ += ["pack_rank3", "rank_tables"]
