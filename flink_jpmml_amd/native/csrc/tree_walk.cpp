// Native host walker of the float64 oracle's TreeModel semantics (linked into `_fastpath`).
//
// The reference evaluates every record through JPMML on the JVM (`S/api/PmmlModel.scala:159-160`):
// one tree walk per record in compiled code. The oracle here (`models/tree.py::leaf_index`) walks
// trees with numpy masks — exact, but one Python iteration per node per tree, ~1 k records/s on a
// 1000-tree GBDT. This file is the same walk in C++, row by row, over the oracle's own prepared
// float64 columns, so every decision is the oracle's float64 comparison and the chosen node is
// bit-identical by construction (tests/test_native_walk.py checks it against the numpy walk).
//
// A tree is a "program" built once per TreeEvaluator (models/native_tree.py):
//
//   nodes_i  int32 [N, 8]  {n_children, first kid, default child (node or -1), flags, field, c0, c1, pred}
//   nodes_d  f64   [N]     split value of a FAST node
//   kids     int32 [...]   child node indices, in document order
//   preds_i  int32 [M, 4]  {kind, operator, field, aux start}   (kind: see PK_*; aux for sets /
//   preds_d  f64   [M]     the literal                           compound predicates)
//   aux_i    int32 [...]   compound: child predicate ids; set: {count} then values in aux_d
//   aux_d    f64   [...]   set values
//
// FAST nodes (flags bit 0) are the exporters' binary split: first child `x OP v` with OP one of
// < <= > >= and a numeric literal, second child `True` (flags bit 3 clear) or the exact complement
// (bit 3 set). Their non-missing step is branch-free: node = (x OP v) ? c0 : c1. Everything else
// (any child count, set / compound / surrogate predicates) takes the general child loop with the
// oracle's three-valued logic. Missing values follow missingValueStrategy / noTrueChildStrategy
// exactly as `leaf_index` does (weightedConfidence / aggregateNodes rows return -1: the Python
// mixture handles them).
//
// Entry points (METH_VARARGS):
//   forest_leaves(nodes_i, nodes_d, kids, preds_i, preds_d, aux_i, aux_d, roots, modes, X, k, out)
//       out int32 [T, n]: the scoring node of row r in tree t, LOCAL to the tree (node - roots[t]),
//       or -1 (null prediction). X is C-contiguous float64 [n, k]; `field` indexes its k columns.
//   forest_values(..., roots, modes, X, k, leafval, out)
//       out f64 [n, T]: leafval[node] (NaN where the walk returned -1).
// modes[t] = strategy | noTrueChild << 4 (strategy: 0 none, 1 lastPrediction, 2 defaultChild,
// 3 nullPrediction / weightedConfidence / aggregateNodes; noTrueChild: 1 = returnLastPrediction).

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <thread>
#include <new>
#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

enum PredKind : int32_t {
    PK_TRUE = 0,
    PK_FALSE = 1,
    PK_SIMPLE = 2,
    PK_IS_MISSING = 3,
    PK_IS_NOT_MISSING = 4,
    PK_SET_IN = 5,
    PK_SET_NOT_IN = 6,
    PK_AND = 7,
    PK_OR = 8,
    PK_XOR = 9,
    PK_SURROGATE = 10,
};
enum SimpleOp : int32_t { OP_EQ = 0, OP_NE = 1, OP_LT = 2, OP_LE = 3, OP_GT = 4, OP_GE = 5 };
enum Tri : int { T_FALSE = 0, T_TRUE = 1, T_UNKNOWN = 2 };
enum Strategy : int { S_NONE = 0, S_LAST = 1, S_DEFAULT = 2, S_NULL = 3 };

struct Program {
    const int32_t *ni;
    const double *nd;
    const int32_t *kids;
    const int32_t *pi;
    const double *pd;
    const int32_t *ai;
    const double *ad;
    Py_ssize_t n_nodes, n_kids, n_preds, n_ai, n_ad;
};

// Three-valued predicate evaluation (fields.py::eval_predicate, row form).
int eval_pred(const Program &p, int32_t id, const double *x, int depth) {
    const int32_t *r = p.pi + 4 * static_cast<Py_ssize_t>(id);
    switch (r[0]) {
        case PK_TRUE:
            return T_TRUE;
        case PK_FALSE:
            return T_FALSE;
        case PK_SIMPLE: {
            const double v = x[r[2]];
            if (std::isnan(v)) return T_UNKNOWN;
            const double lit = p.pd[id];
            bool t;
            switch (r[1]) {
                case OP_EQ: t = v == lit; break;
                case OP_NE: t = v != lit; break;
                case OP_LT: t = v < lit; break;
                case OP_LE: t = v <= lit; break;
                case OP_GT: t = v > lit; break;
                default: t = v >= lit; break;
            }
            return t ? T_TRUE : T_FALSE;
        }
        case PK_IS_MISSING:
            return std::isnan(x[r[2]]) ? T_TRUE : T_FALSE;
        case PK_IS_NOT_MISSING:
            return std::isnan(x[r[2]]) ? T_FALSE : T_TRUE;
        case PK_SET_IN:
        case PK_SET_NOT_IN: {
            const double v = x[r[2]];
            if (std::isnan(v)) return T_UNKNOWN;
            const int32_t start = r[3];
            const int32_t cnt = p.ai[start];
            const int32_t voff = p.ai[start + 1];
            bool inside = false;
            for (int32_t k = 0; k < cnt; ++k) inside |= (v == p.ad[voff + k]);
            return (inside == (r[0] == PK_SET_IN)) ? T_TRUE : T_FALSE;
        }
        default:
            break;
    }
    // compound: aux = {count, child ids...}
    if (depth > 64) return T_UNKNOWN;  // host-checked at build; a bound for malformed programs
    const int32_t start = r[3];
    const int32_t cnt = p.ai[start];
    const int32_t *ch = p.ai + start + 1;
    switch (r[0]) {
        case PK_AND: {
            bool anyfalse = false, anyunk = false;
            for (int32_t k = 0; k < cnt; ++k) {
                const int t = eval_pred(p, ch[k], x, depth + 1);
                anyfalse |= t == T_FALSE;
                anyunk |= t == T_UNKNOWN;
            }
            return anyfalse ? T_FALSE : (anyunk ? T_UNKNOWN : T_TRUE);
        }
        case PK_OR: {
            bool anytrue = false, anyunk = false;
            for (int32_t k = 0; k < cnt; ++k) {
                const int t = eval_pred(p, ch[k], x, depth + 1);
                anytrue |= t == T_TRUE;
                anyunk |= t == T_UNKNOWN;
            }
            return anytrue ? T_TRUE : (anyunk ? T_UNKNOWN : T_FALSE);
        }
        case PK_XOR: {
            bool acc = false, unk = false;
            for (int32_t k = 0; k < cnt; ++k) {
                const int t = eval_pred(p, ch[k], x, depth + 1);
                acc ^= t == T_TRUE;
                unk |= t == T_UNKNOWN;
            }
            return unk ? T_UNKNOWN : (acc ? T_TRUE : T_FALSE);
        }
        case PK_SURROGATE: {
            for (int32_t k = 0; k < cnt; ++k) {
                const int t = eval_pred(p, ch[k], x, depth + 1);
                if (t != T_UNKNOWN) return t;
            }
            return T_UNKNOWN;
        }
        default:
            return T_UNKNOWN;
    }
}

// One row through one tree (models/tree.py::leaf_index, row form). Returns the GLOBAL node index
// of the scoring node, or -1.
inline int32_t walk(const Program &p, int32_t root, const double *x, int strat, int notrue) {
    // the root's own predicate selects the rows that reach it (TRUE only)
    const int32_t *rr = p.ni + 8 * static_cast<Py_ssize_t>(root);
    if (rr[7] >= 0 && eval_pred(p, rr[7], x, 0) != T_TRUE) return -1;
    int32_t node = root;
    for (int guard = 0; guard < (1 << 20); ++guard) {
        const int32_t *r = p.ni + 8 * static_cast<Py_ssize_t>(node);
        const int32_t nch = r[0];
        if (nch == 0) return node;
        const int32_t flags = r[3];
        if (flags & 1) {  // FAST binary split
            const double v = x[r[4]];
            if (__builtin_expect(!std::isnan(v), 1)) {
                const double t = p.nd[node];
                const bool lt = v < t, eq = v == t;
                bool res;
                switch ((flags >> 1) & 3) {
                    case 0: res = lt; break;
                    case 1: res = lt | eq; break;
                    case 2: res = !(lt | eq); break;
                    default: res = !lt; break;
                }
                node = res ? r[5] : r[6];
                continue;
            }
            // first child's predicate is UNKNOWN
            if (strat == S_LAST) return node;
            if (strat == S_DEFAULT) {
                if (r[2] < 0) return -1;
                node = r[2];
                continue;
            }
            if (strat == S_NULL) return -1;
            // 'none': UNKNOWN counts as FALSE; a True second child is taken, a complement one is
            // UNKNOWN too -> no true child
            if (!(flags & 8)) {
                node = r[6];
                continue;
            }
            return notrue ? node : -1;
        }
        const int32_t *kid = p.kids + r[1];
        int32_t next = -2;
        for (int32_t k = 0; k < nch; ++k) {
            const int32_t c = kid[k];
            const int t = eval_pred(p, p.ni[8 * static_cast<Py_ssize_t>(c) + 7], x, 0);
            if (t == T_UNKNOWN && strat != S_NONE) {
                if (strat == S_LAST) return node;
                if (strat == S_DEFAULT) {
                    if (r[2] < 0) return -1;
                    next = r[2];
                    break;
                }
                return -1;
            }
            if (t == T_TRUE) {
                next = c;
                break;
            }
        }
        if (next == -2) return notrue ? node : -1;
        node = next;
    }
    return -1;
}

// ---------------------------------------------------------------------------------------------
// Fixed-depth interleaved walk. A tree whose root predicate is True and whose internal nodes are
// all FAST, under a strategy whose missing-value step is a plain child choice, is compiled into
// compact 32-byte nodes {t, field, flags, next[3]} with next = {c0, c1, on-missing}: leaves (and a
// shared NULL node standing for "no prediction") loop onto themselves, so G rows step through the
// tree together for exactly its depth, with no data-dependent branch (the select is an indexed
// load). Trees outside that form take walk() above; the result is the same node.
struct Compact {
    double t;
    int32_t field;
    int32_t flags;  // bit0 incl (x == t counts as "less"), bit1 neg (take the complement)
    int32_t next[3];
    int32_t pad;
};
static_assert(sizeof(Compact) == 32, "compact node layout");

constexpr int32_t NULL_NODE_TAG = -1;

// Compiles tree t (rooted at `root`) into `cn` (appending); returns its depth, or -1 if the tree is
// not in fixed-depth form. `null_slot` is the index of the shared NULL node in `cn`.
int compile_fixed(const Program &p, int32_t root, int strat, int notrue, std::vector<Compact> &cn,
                  std::vector<int32_t> &gmap, int32_t null_slot) {
    const int32_t *rr = p.ni + 8 * static_cast<Py_ssize_t>(root);
    if (rr[7] >= 0 && p.pi[4 * static_cast<Py_ssize_t>(rr[7])] != PK_TRUE) return -1;
    if (strat == S_LAST) return -1;
    // pass 1: the subtree's nodes (preorder from root), check the form, find the depth
    std::vector<std::pair<int32_t, int>> stack{{root, 0}};
    std::vector<int32_t> order;
    int depth = 0;
    while (!stack.empty()) {
        auto [nd, d] = stack.back();
        stack.pop_back();
        if (d > 60) return -1;
        order.push_back(nd);
        depth = d > depth ? d : depth;
        const int32_t *r = p.ni + 8 * static_cast<Py_ssize_t>(nd);
        if (r[0] == 0) continue;
        if (!(r[3] & 1)) return -1;
        if (strat == S_NONE && (r[3] & 8) && notrue) return -1;  // missing -> this node's own score
        stack.push_back({r[5], d + 1});
        stack.push_back({r[6], d + 1});
        if (strat == S_DEFAULT && r[2] >= 0 && r[2] != r[5] && r[2] != r[6]) return -1;
    }
    const int32_t base = static_cast<int32_t>(cn.size());
    std::unordered_map<int32_t, int32_t> local;
    local.reserve(order.size() * 2);
    for (size_t i = 0; i < order.size(); ++i) local.emplace(order[i], base + static_cast<int32_t>(i));
    cn.resize(cn.size() + order.size());
    gmap.resize(cn.size());
    for (size_t i = 0; i < order.size(); ++i) {
        const int32_t nd = order[i];
        const int32_t *r = p.ni + 8 * static_cast<Py_ssize_t>(nd);
        Compact &c = cn[base + i];
        gmap[base + i] = nd;
        const int32_t self = base + static_cast<int32_t>(i);
        if (r[0] == 0) {
            c = Compact{0.0, 0, 0, {self, self, self}, 0};
            continue;
        }
        const int op = (r[3] >> 1) & 3;  // 0 <, 1 <=, 2 >, 3 >=
        const int32_t c0 = local.at(r[5]), c1 = local.at(r[6]);
        int32_t miss;
        if (strat == S_DEFAULT) {
            miss = r[2] < 0 ? null_slot : local.at(r[2]);
        } else if (strat == S_NULL) {
            miss = null_slot;
        } else {  // 'none': a True second child is taken; a complement one -> no true child -> null
            miss = (r[3] & 8) ? null_slot : c1;
        }
        c = Compact{p.nd[nd], r[4], (op == 1 || op == 2 ? 1 : 0) | (op >= 2 ? 2 : 0), {c0, c1, miss}, 0};
    }
    return depth;
}

// G independent walks through one compiled tree; leaves / NULL loop onto themselves.
template <int G>
inline void walk_fixed(const Compact *cn, int32_t root, int depth, const double *X, Py_ssize_t k,
                       Py_ssize_t r0, int32_t *node) {
    for (int j = 0; j < G; ++j) node[j] = root;
    for (int d = 0; d < depth; ++d) {
#pragma GCC unroll 16
        for (int j = 0; j < G; ++j) {
            const Compact &c = cn[node[j]];
            const double v = X[(r0 + j) * k + c.field];
            const int lt = v < c.t, eq = v == c.t;
            const int res = (lt | (eq & c.flags)) ^ (c.flags >> 1);  // 1: first child
            const int sel = (v != v) ? 2 : (res ^ 1);                // 0 c0, 1 c1, 2 missing
            node[j] = c.next[sel];
        }
    }
}

struct Buf {
    Py_buffer b{};
    bool ok = false;
    ~Buf() {
        if (ok) PyBuffer_Release(&b);
    }
    bool get(PyObject *o, const char *fmt, Py_ssize_t itemsize, bool writable, const char *what) {
        if (PyObject_GetBuffer(o, &b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT | (writable ? PyBUF_WRITABLE : 0)) != 0)
            return false;
        ok = true;
        const char *f = b.format ? b.format : "B";
        if (*f == '<' || *f == '=' || *f == '@') ++f;  // native / little-endian byte order only
        if (b.itemsize != itemsize || f[0] == '\0' || f[1] != '\0' || std::strchr(fmt, f[0]) == nullptr) {
            PyErr_Format(PyExc_TypeError, "tree walk: %s must be a C-contiguous %s buffer", what, fmt);
            return false;
        }
        return true;
    }
    Py_ssize_t n() const { return b.len / b.itemsize; }
};

constexpr Py_ssize_t ROW_BLOCK = 256;

enum class Kind { LEAVES, VALUES, SUMS, VOTES };

// Common front half of the entry points: parse + validate the program and the input matrix.
struct Call {
    Buf ni, nd, kids, pi, pd, ai, ad, roots, modes, X, out, leafval, weights;
    Buf cls, wsum, cnt, miss;  // VOTES: node -> class table and the per-row outputs
    Program prog{};
    Py_ssize_t T = 0, n = 0, k = 0, C = 0;
    bool has_weights = false;

    PyObject *cache = Py_None;  // forest_compile's capsule of this program, or None

    bool parse(PyObject *args, Kind kind) {
        PyObject *o[18] = {};
        bool okp;
        if (kind == Kind::VOTES)
            okp = PyArg_ParseTuple(args, "OOOOOOOOOOnOOnOOOO|O", &o[0], &o[1], &o[2], &o[3], &o[4], &o[5], &o[6],
                                   &o[7], &o[8], &o[9], &k, &o[11], &o[12], &C, &o[13], &o[14], &o[15], &o[16],
                                   &cache);
        else if (kind == Kind::LEAVES)
            okp = PyArg_ParseTuple(args, "OOOOOOOOOOnO|O", &o[0], &o[1], &o[2], &o[3], &o[4], &o[5], &o[6], &o[7],
                                   &o[8], &o[9], &k, &o[11], &cache);
        else if (kind == Kind::VALUES)
            okp = PyArg_ParseTuple(args, "OOOOOOOOOOnOO|O", &o[0], &o[1], &o[2], &o[3], &o[4], &o[5], &o[6], &o[7],
                                   &o[8], &o[9], &k, &o[11], &o[12], &cache);
        else
            okp = PyArg_ParseTuple(args, "OOOOOOOOOOnOOO|O", &o[0], &o[1], &o[2], &o[3], &o[4], &o[5], &o[6], &o[7],
                                   &o[8], &o[9], &k, &o[11], &o[12], &o[13], &cache);
        if (!okp) return false;
        if (!ni.get(o[0], "i", 4, false, "nodes_i") || !nd.get(o[1], "d", 8, false, "nodes_d") ||
            !kids.get(o[2], "i", 4, false, "kids") || !pi.get(o[3], "i", 4, false, "preds_i") ||
            !pd.get(o[4], "d", 8, false, "preds_d") || !ai.get(o[5], "i", 4, false, "aux_i") ||
            !ad.get(o[6], "d", 8, false, "aux_d") || !roots.get(o[7], "i", 4, false, "roots") ||
            !modes.get(o[8], "i", 4, false, "modes") || !X.get(o[9], "d", 8, false, "X"))
            return false;
        if (kind == Kind::VOTES) {
            if (!cls.get(o[11], "i", 4, false, "cls") || !weights.get(o[12], "d", 8, false, "weights") ||
                !out.get(o[13], "d", 8, true, "acc") || !wsum.get(o[14], "d", 8, true, "wsum") ||
                !cnt.get(o[15], "i", 4, true, "count") || !miss.get(o[16], "B", 1, true, "anymiss"))
                return false;
            has_weights = true;
        } else if (kind == Kind::LEAVES) {
            if (!out.get(o[11], "i", 4, true, "out")) return false;
        } else if (kind == Kind::VALUES) {
            if (!leafval.get(o[11], "d", 8, false, "leafval") || !out.get(o[12], "d", 8, true, "out")) return false;
        } else {
            if (!leafval.get(o[11], "d", 8, false, "leafval")) return false;
            if (o[12] != Py_None) {
                if (!weights.get(o[12], "d", 8, false, "weights")) return false;
                has_weights = true;
            }
            if (!out.get(o[13], "d", 8, true, "out")) return false;
        }
        prog = Program{static_cast<const int32_t *>(ni.b.buf),  static_cast<const double *>(nd.b.buf),
                       static_cast<const int32_t *>(kids.b.buf), static_cast<const int32_t *>(pi.b.buf),
                       static_cast<const double *>(pd.b.buf),   static_cast<const int32_t *>(ai.b.buf),
                       static_cast<const double *>(ad.b.buf),   ni.n() / 8, kids.n(), pi.n() / 4, ai.n(), ad.n()};
        T = roots.n();
        if (modes.n() != T || nd.n() != prog.n_nodes || pd.n() != prog.n_preds || k < 1 || X.n() % k) {
            PyErr_SetString(PyExc_ValueError, "tree walk: inconsistent program / matrix shapes");
            return false;
        }
        n = X.n() / k;
        if (kind == Kind::VOTES) {
            if (C < 1 || cls.n() != prog.n_nodes || weights.n() != T || out.n() != n * C || wsum.n() != n ||
                cnt.n() != n || miss.n() != n) {
                PyErr_SetString(PyExc_ValueError, "tree walk: vote table / output shape mismatch");
                return false;
            }
            const int32_t *ct = static_cast<const int32_t *>(cls.b.buf);
            for (Py_ssize_t i = 0; i < prog.n_nodes; ++i)
                if (ct[i] < -1 || ct[i] >= C) {
                    PyErr_SetString(PyExc_ValueError, "tree walk: vote class out of range");
                    return false;
                }
            return cache_matches() || validate();
        }
        const Py_ssize_t want = kind == Kind::SUMS ? n : T * n;
        if (out.n() != want || (kind != Kind::LEAVES && leafval.n() != prog.n_nodes) ||
            (has_weights && weights.n() != T)) {
            PyErr_SetString(PyExc_ValueError, "tree walk: output / leaf-value / weight shape mismatch");
            return false;
        }
        // a program compiled by forest_compile was validated then (same buffers, same k): the
        // per-call check of every node would cost more than scoring one row
        return cache_matches() || validate();
    }

    bool cache_matches() const;

    // Every index the walk can follow stays inside its array (a malformed program raises here
    // instead of reading out of bounds).
    bool validate() const {
        const Program &p = prog;
        auto bad = [](const char *m) {
            PyErr_Format(PyExc_ValueError, "tree walk: malformed program (%s)", m);
            return false;
        };
        for (Py_ssize_t i = 0; i < p.n_nodes; ++i) {
            const int32_t *r = p.ni + 8 * i;
            if (r[0] < 0 || r[1] < 0 || static_cast<Py_ssize_t>(r[1]) + r[0] > p.n_kids) return bad("kids range");
            if (r[2] < -1 || r[2] >= p.n_nodes) return bad("default child");
            if (r[7] < -1 || r[7] >= p.n_preds) return bad("node predicate");
            if (r[0] > 0 && (r[3] & 1)) {
                if (r[4] < 0 || r[4] >= k || r[5] < 0 || r[5] >= p.n_nodes || r[6] < 0 || r[6] >= p.n_nodes)
                    return bad("fast split");
            }
        }
        for (Py_ssize_t i = 0; i < p.n_kids; ++i)
            if (p.kids[i] < 0 || p.kids[i] >= p.n_nodes || p.ni[8 * static_cast<Py_ssize_t>(p.kids[i]) + 7] < 0)
                return bad("kid");
        for (Py_ssize_t i = 0; i < p.n_preds; ++i) {
            const int32_t *r = p.pi + 4 * i;
            if (r[0] < PK_TRUE || r[0] > PK_SURROGATE) return bad("predicate kind");
            if ((r[0] >= PK_SIMPLE && r[0] <= PK_SET_NOT_IN) && (r[2] < 0 || r[2] >= k)) return bad("field");
            if (r[0] == PK_SET_IN || r[0] == PK_SET_NOT_IN) {
                if (r[3] < 0 || r[3] + 2 > p.n_ai) return bad("set aux");
                const int32_t cnt = p.ai[r[3]], off = p.ai[r[3] + 1];
                if (cnt < 0 || off < 0 || static_cast<Py_ssize_t>(off) + cnt > p.n_ad) return bad("set values");
            } else if (r[0] >= PK_AND) {
                if (r[3] < 0 || r[3] + 1 > p.n_ai) return bad("compound aux");
                const int32_t cnt = p.ai[r[3]];
                if (cnt < 0 || static_cast<Py_ssize_t>(r[3]) + 1 + cnt > p.n_ai) return bad("compound children");
                for (int32_t c = 0; c < cnt; ++c)
                    if (p.ai[r[3] + 1 + c] < 0 || p.ai[r[3] + 1 + c] >= p.n_preds) return bad("compound child");
            }
        }
        const int32_t *rt = static_cast<const int32_t *>(roots.b.buf);
        for (Py_ssize_t t = 0; t < T; ++t)
            if (rt[t] < 0 || rt[t] >= p.n_nodes) return bad("root");
        return true;
    }
};

// ---------------------------------------------------------------------------------------------
// PERFECT form of a fixed-depth tree of depth D <= PERFECT_MAX_D: heap-ordered slots (root 0,
// children 2j+1 / 2j+2), NI = 2^D - 1 split slots {t, meta} and 2^D leaf slots holding the scoring
// node. A leaf above depth D is replicated over its padded subtree (whose splits then do not
// matter; their missing action is "left", so a NaN they read never changes the result). meta =
// field | incl << 16 | neg << 17 | missing action << 18 (0 left, 1 right, 2 null prediction). The
// step is j = 2j + 1 + right: no next-pointer load, and 8 rows per AVX-512 vector.
constexpr int PERFECT_MAX_D = 10;

struct Fixed {
    std::vector<Compact> cn;
    std::vector<int32_t> gmap;  // compact node -> global node (NULL -> -1)
    std::vector<int32_t> croot;
    std::vector<int> depth;
    int32_t null_slot = 0;
    // perfect form (per tree: pbase[t] >= 0)
    std::vector<double> pt;
    std::vector<int32_t> pmeta, pleaf;
    std::vector<Py_ssize_t> pbase, plbase;
};

void fill_perfect(const Fixed &f, int32_t c, int64_t j, int D, Py_ssize_t tb, Py_ssize_t lb, std::vector<double> &pt,
                  std::vector<int32_t> &pmeta, std::vector<int32_t> &pleaf) {
    const int64_t NI = (int64_t(1) << D) - 1;
    if (j >= NI) {
        pleaf[lb + (j - NI)] = f.gmap[c];
        return;
    }
    const Compact &n = f.cn[c];
    const bool leaf = n.next[0] == c && n.next[1] == c;
    if (leaf) {
        pt[tb + j] = 0.0;
        pmeta[tb + j] = 0;  // field 0, missing -> left: irrelevant, every slot below holds this leaf
        fill_perfect(f, c, 2 * j + 1, D, tb, lb, pt, pmeta, pleaf);
        fill_perfect(f, c, 2 * j + 2, D, tb, lb, pt, pmeta, pleaf);
        return;
    }
    const int miss = n.next[2] == n.next[0] ? 0 : (n.next[2] == n.next[1] ? 1 : 2);
    pt[tb + j] = n.t;
    pmeta[tb + j] = n.field | ((n.flags & 1) << 16) | (((n.flags >> 1) & 1) << 17) | (miss << 18);
    fill_perfect(f, n.next[0], 2 * j + 1, D, tb, lb, pt, pmeta, pleaf);
    fill_perfect(f, n.next[1], 2 * j + 2, D, tb, lb, pt, pmeta, pleaf);
}

// Compiles every tree that has a fixed-depth form (depth[t] >= 0, compact root in croot[t]) and,
// when it is shallow enough, its perfect form.
void compile_all(const Call &c, Fixed &f) {
    const int32_t *roots = static_cast<const int32_t *>(c.roots.b.buf);
    const int32_t *modes = static_cast<const int32_t *>(c.modes.b.buf);
    f.cn.push_back(Compact{0.0, 0, 0, {0, 0, 0}, 0});  // the shared NULL node (slot 0)
    f.gmap.push_back(NULL_NODE_TAG);
    f.null_slot = 0;
    f.croot.assign(c.T, -1);
    f.depth.assign(c.T, -1);
    f.pbase.assign(c.T, -1);
    f.plbase.assign(c.T, -1);
    for (Py_ssize_t t = 0; t < c.T; ++t) {
        const size_t mark = f.cn.size();
        const int d = compile_fixed(c.prog, roots[t], modes[t] & 15, (modes[t] >> 4) & 1, f.cn, f.gmap, f.null_slot);
        if (d < 0) {
            f.cn.resize(mark);
            f.gmap.resize(mark);
            continue;
        }
        f.croot[t] = static_cast<int32_t>(mark);
        f.depth[t] = d;
    }
    const bool narrow_fields = c.k < (1 << 16);
    for (Py_ssize_t t = 0; t < c.T; ++t) {
        const int D = f.depth[t];
        if (D < 1 || D > PERFECT_MAX_D || !narrow_fields) continue;
        const Py_ssize_t NI = (Py_ssize_t(1) << D) - 1;
        f.pbase[t] = static_cast<Py_ssize_t>(f.pt.size());
        f.plbase[t] = static_cast<Py_ssize_t>(f.pleaf.size());
        f.pt.resize(f.pt.size() + NI);
        f.pmeta.resize(f.pmeta.size() + NI);
        f.pleaf.resize(f.pleaf.size() + NI + 1);
        fill_perfect(f, f.croot[t], 0, D, f.pbase[t], f.plbase[t], f.pt, f.pmeta, f.pleaf);
    }
    if (std::getenv("FJA_WALK_DEBUG")) {
        Py_ssize_t fixed = 0, perfect = 0;
        for (Py_ssize_t t = 0; t < c.T; ++t) {
            fixed += f.depth[t] >= 0;
            perfect += f.pbase[t] >= 0;
        }
        std::fprintf(stderr, "tree_walk: %zd of %zd trees fixed-depth, %zd perfect, %zu compact nodes, avx512 %d\n",
                     fixed, c.T, perfect, f.cn.size(), (int)__builtin_cpu_supports("avx512f"));
    }
}

// A compiled program kept across calls (forest_compile): the fixed-depth / perfect tables of a
// 1000-tree ensemble take milliseconds to build, so per-record scoring must not rebuild them.
// The fingerprint ties the tables to the exact program buffers they were built from.
struct Cached {
    Fixed f;
    const void *ni, *kids, *pi, *roots, *modes, *nd, *pd, *ai, *ad;
    Py_ssize_t n_nodes, T, k, n_kids, n_preds, n_ai, n_ad;
};
constexpr const char *CAPSULE = "fja.forest_program";

void drop_cached(PyObject *cap) { delete static_cast<Cached *>(PyCapsule_GetPointer(cap, CAPSULE)); }

const Fixed *cached_fixed(const Call &c) {
    if (c.cache == nullptr || c.cache == Py_None || !PyCapsule_IsValid(c.cache, CAPSULE)) return nullptr;
    const Cached *h = static_cast<const Cached *>(PyCapsule_GetPointer(c.cache, CAPSULE));
    if (h == nullptr || h->ni != c.ni.b.buf || h->kids != c.kids.b.buf || h->pi != c.pi.b.buf ||
        h->roots != c.roots.b.buf || h->n_nodes != c.prog.n_nodes || h->T != c.T || h->k != c.k ||
        h->n_kids != c.prog.n_kids || h->n_preds != c.prog.n_preds || h->n_ai != c.prog.n_ai ||
        h->n_ad != c.prog.n_ad || h->modes != c.modes.b.buf || h->nd != c.nd.b.buf || h->pd != c.pd.b.buf ||
        h->ai != c.ai.b.buf || h->ad != c.ad.b.buf)
        return nullptr;  // not this program: the caller validates and compiles afresh
    return &h->f;
}

bool Call::cache_matches() const { return cached_fixed(*this) != nullptr; }

constexpr int G = 16;

// G rows through one perfect tree (scalar, interleaved). Writes the scoring node (or -1).
template <int Gn>
inline void walk_perfect(const double *pt, const int32_t *pm, const int32_t *pl, int D, const double *X, Py_ssize_t k,
                         Py_ssize_t r0, int32_t *res) {
    int32_t s[Gn];
    int32_t poison[Gn];
    const double *xr[Gn];
    for (int j = 0; j < Gn; ++j) {
        s[j] = 0;
        poison[j] = 0;
        xr[j] = X + (r0 + j) * k;
    }
    for (int d = 0; d < D; ++d) {
#pragma GCC unroll 16
        for (int j = 0; j < Gn; ++j) {
            const int32_t m = pm[s[j]];
            const double t = pt[s[j]];
            const double v = xr[j][m & 0xFFFF];
            const int lt = v < t, eq = v == t;
            const int pred = (lt | (eq & (m >> 16))) ^ ((m >> 17) & 1);
            const int miss = (m >> 18) & 3;
            const int nan = v != v;
            const int right = nan ? (miss == 1) : (pred ^ 1);
            poison[j] |= nan & (miss == 2);
            s[j] = 2 * s[j] + 1 + right;
        }
    }
    const int32_t NI = (int32_t(1) << D) - 1;
    for (int j = 0; j < Gn; ++j) res[j] = poison[j] ? -1 : pl[s[j] - NI];
}

#if defined(__x86_64__)
// 32 rows (4 x 8 lanes) through one perfect tree with AVX-512 gathers. Same arithmetic as
// walk_perfect: float64 compares of the oracle's values against the oracle's literals.
__attribute__((target("avx512f,avx512vl"))) void walk_perfect_avx512(const double *pt, const int32_t *pm,
                                                                     const int32_t *pl, int D, const double *X,
                                                                     Py_ssize_t k, Py_ssize_t r0, int32_t *res) {
    constexpr int V = 4;
    __m256i s[V], rowoff[V];
    __mmask8 poison[V];
    const __m256i lane = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
    const __m256i kk = _mm256_set1_epi32(static_cast<int32_t>(k));
    const __m256i one = _mm256_set1_epi32(1), fmask = _mm256_set1_epi32(0xFFFF), three = _mm256_set1_epi32(3);
    const __m256i two = _mm256_set1_epi32(2);
    for (int v = 0; v < V; ++v) {
        s[v] = _mm256_setzero_si256();
        poison[v] = 0;
        // row index relative to r0: X is addressed from X + r0 * k (int32 offsets stay small)
        rowoff[v] = _mm256_mullo_epi32(_mm256_add_epi32(lane, _mm256_set1_epi32(8 * v)), kk);
    }
    const double *Xb = X + r0 * k;
    for (int d = 0; d < D; ++d) {
        // Levels of at most 32 nodes live in registers: every lane's node is a permute of the
        // level's thresholds / metadata (no gather); deeper levels gather from the tables.
        const int W = 1 << d, base = W - 1;
        const bool regs = W <= 32;
        __m512d T0 = _mm512_setzero_pd(), T1 = T0, T2 = T0, T3 = T0;
        __m512i M0 = _mm512_setzero_si512(), M1 = M0;
        if (regs) {
            T0 = _mm512_maskz_loadu_pd(static_cast<__mmask8>(W >= 8 ? 0xFF : (1u << W) - 1), pt + base);
            M0 = _mm512_maskz_loadu_epi32(static_cast<__mmask16>(W >= 16 ? 0xFFFF : (1u << W) - 1), pm + base);
            if (W >= 16) T1 = _mm512_loadu_pd(pt + base + 8);
            if (W == 32) {
                T2 = _mm512_loadu_pd(pt + base + 16);
                T3 = _mm512_loadu_pd(pt + base + 24);
                M1 = _mm512_loadu_si512(pm + base + 16);
            }
        }
        const __m256i vbase = _mm256_set1_epi32(base);
        for (int v = 0; v < V; ++v) {
            __m256i m;
            __m512d t;
            if (regs) {
                const __m256i li = _mm256_sub_epi32(s[v], vbase);  // index within the level
                const __m512i li512 = _mm512_castsi256_si512(li);
                const __m512i li64 = _mm512_cvtepi32_epi64(li);
                if (W <= 16) {
                    m = _mm512_castsi512_si256(_mm512_permutexvar_epi32(li512, M0));
                    t = W <= 8 ? _mm512_permutexvar_pd(li64, T0) : _mm512_permutex2var_pd(T0, li64, T1);
                } else {
                    m = _mm512_castsi512_si256(_mm512_permutex2var_epi32(M0, li512, M1));
                    const __mmask8 hi = _mm256_test_epi32_mask(li, _mm256_set1_epi32(16));
                    t = _mm512_mask_blend_pd(hi, _mm512_permutex2var_pd(T0, li64, T1),
                                             _mm512_permutex2var_pd(T2, li64, T3));
                }
            } else {
                m = _mm256_i32gather_epi32(pm, s[v], 4);
                t = _mm512_i32gather_pd(s[v], pt, 8);
            }
            const __m256i xi = _mm256_add_epi32(rowoff[v], _mm256_and_si256(m, fmask));
            const __m512d x = _mm512_i32gather_pd(xi, Xb, 8);
            const __mmask8 lt = _mm512_cmp_pd_mask(x, t, _CMP_LT_OQ);
            const __mmask8 eq = _mm512_cmp_pd_mask(x, t, _CMP_EQ_OQ);
            const __mmask8 un = _mm512_cmp_pd_mask(x, x, _CMP_UNORD_Q);
            const __mmask8 incl = _mm256_test_epi32_mask(m, _mm256_set1_epi32(1 << 16));
            const __mmask8 neg = _mm256_test_epi32_mask(m, _mm256_set1_epi32(1 << 17));
            const __m256i miss = _mm256_and_si256(_mm256_srli_epi32(m, 18), three);
            const __mmask8 mright = _mm256_cmpeq_epi32_mask(miss, one);
            const __mmask8 mnull = _mm256_cmpeq_epi32_mask(miss, two);
            const __mmask8 pred = (lt | (eq & incl)) ^ neg;
            const __mmask8 right = static_cast<__mmask8>((~pred & ~un) | (un & mright));
            poison[v] |= un & mnull;
            s[v] = _mm256_mask_add_epi32(_mm256_add_epi32(_mm256_add_epi32(s[v], s[v]), one), right,
                                         _mm256_add_epi32(_mm256_add_epi32(s[v], s[v]), one), one);
        }
    }
    const __m256i NI = _mm256_set1_epi32((int32_t(1) << D) - 1);
    for (int v = 0; v < V; ++v) {
        __m256i leaf = _mm256_i32gather_epi32(pl, _mm256_sub_epi32(s[v], NI), 4);
        leaf = _mm256_mask_mov_epi32(leaf, poison[v], _mm256_set1_epi32(-1));
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(res + 8 * v), leaf);
    }
}
#endif

#if defined(__x86_64__)
// ONE row through 8 perfect trees of equal depth D (a lane per tree: the single-record call, where
// row-parallel lanes have nothing to work on). Same arithmetic as walk_perfect; pb / lb: the 8
// trees' offsets into the concatenated perfect tables.
__attribute__((target("avx512f,avx512vl"))) void walk_trees8_avx512(const double *pt, const int32_t *pm,
                                                                    const int32_t *pl, const int32_t *pb,
                                                                    const int32_t *lb, int D, const double *xr,
                                                                    int32_t *res) {
    const __m256i base = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(pb));
    const __m256i one = _mm256_set1_epi32(1), fmask = _mm256_set1_epi32(0xFFFF), three = _mm256_set1_epi32(3);
    const __m256i two = _mm256_set1_epi32(2);
    __m256i s = _mm256_setzero_si256();
    __mmask8 poison = 0;
    for (int d = 0; d < D; ++d) {
        const __m256i idx = _mm256_add_epi32(base, s);
        const __m256i m = _mm256_i32gather_epi32(pm, idx, 4);
        const __m512d t = _mm512_i32gather_pd(idx, pt, 8);
        const __m512d x = _mm512_i32gather_pd(_mm256_and_si256(m, fmask), xr, 8);
        const __mmask8 lt = _mm512_cmp_pd_mask(x, t, _CMP_LT_OQ);
        const __mmask8 eq = _mm512_cmp_pd_mask(x, t, _CMP_EQ_OQ);
        const __mmask8 un = _mm512_cmp_pd_mask(x, x, _CMP_UNORD_Q);
        const __mmask8 incl = _mm256_test_epi32_mask(m, _mm256_set1_epi32(1 << 16));
        const __mmask8 neg = _mm256_test_epi32_mask(m, _mm256_set1_epi32(1 << 17));
        const __m256i miss = _mm256_and_si256(_mm256_srli_epi32(m, 18), three);
        const __mmask8 mright = _mm256_cmpeq_epi32_mask(miss, one);
        const __mmask8 mnull = _mm256_cmpeq_epi32_mask(miss, two);
        const __mmask8 pred = (lt | (eq & incl)) ^ neg;
        const __mmask8 right = static_cast<__mmask8>((~pred & ~un) | (un & mright));
        poison |= un & mnull;
        const __m256i s2 = _mm256_add_epi32(_mm256_add_epi32(s, s), one);
        s = _mm256_mask_add_epi32(s2, right, s2, one);
    }
    const __m256i NI = _mm256_set1_epi32((int32_t(1) << D) - 1);
    const __m256i lidx = _mm256_add_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(lb)), _mm256_sub_epi32(s, NI));
    __m256i leaf = _mm256_i32gather_epi32(pl, lidx, 4);
    leaf = _mm256_mask_mov_epi32(leaf, poison, _mm256_set1_epi32(-1));
    _mm256_storeu_si256(reinterpret_cast<__m256i *>(res), leaf);
}
#endif

// Runs every tree over rows [r0, r1) and hands (tree, row, global node or -1) to `emit`.
template <class Emit>
void run_block(const Call &c, const Fixed &f, const double *X, Py_ssize_t r0, Py_ssize_t r1, bool avx512,
               Emit &&emit) {
    const int32_t *roots = static_cast<const int32_t *>(c.roots.b.buf);
    const int32_t *modes = static_cast<const int32_t *>(c.modes.b.buf);
    const Py_ssize_t k = c.k;
    int32_t node[32];
    for (Py_ssize_t t = 0; t < c.T; ++t) {
#if defined(__x86_64__)
        // fewer rows than one row-parallel call: 8 trees at a time per row (perfect, equal depth,
        // table offsets within int32)
        if (avx512 && r1 - r0 < 32 && t + 8 <= c.T && f.pt.size() < (size_t(1) << 31) &&
            f.pleaf.size() < (size_t(1) << 31)) {
            bool same = true;
            for (int j = 0; j < 8 && same; ++j)
                same = f.pbase[t + j] >= 0 && f.depth[t + j] == f.depth[t];
            if (same) {
                int32_t pb[8], lb[8];
                for (int j = 0; j < 8; ++j) {
                    pb[j] = static_cast<int32_t>(f.pbase[t + j]);
                    lb[j] = static_cast<int32_t>(f.plbase[t + j]);
                }
                for (Py_ssize_t r = r0; r < r1; ++r) {
                    walk_trees8_avx512(f.pt.data(), f.pmeta.data(), f.pleaf.data(), pb, lb, f.depth[t], X + r * k, node);
                    for (int j = 0; j < 8; ++j) emit(t + j, r, node[j]);
                }
                t += 7;
                continue;
            }
        }
#endif
        Py_ssize_t r = r0;
        if (f.pbase[t] >= 0) {
            const double *pt = f.pt.data() + f.pbase[t];
            const int32_t *pm = f.pmeta.data() + f.pbase[t];
            const int32_t *pl = f.pleaf.data() + f.plbase[t];
#if defined(__x86_64__)
            if (avx512) {
                for (; r + 32 <= r1; r += 32) {
                    walk_perfect_avx512(pt, pm, pl, f.depth[t], X, k, r, node);
                    for (int j = 0; j < 32; ++j) emit(t, r + j, node[j]);
                }
            }
#endif
            for (; r + G <= r1; r += G) {
                walk_perfect<G>(pt, pm, pl, f.depth[t], X, k, r, node);
                for (int j = 0; j < G; ++j) emit(t, r + j, node[j]);
            }
            for (; r < r1; ++r) {  // the block's tail (and single-record calls): one row at a time
                walk_perfect<1>(pt, pm, pl, f.depth[t], X, k, r, node);
                emit(t, r, node[0]);
            }
        } else if (f.depth[t] >= 0) {
            for (; r + G <= r1; r += G) {
                walk_fixed<G>(f.cn.data(), f.croot[t], f.depth[t], X, k, r, node);
                for (int j = 0; j < G; ++j) emit(t, r + j, f.gmap[node[j]]);
            }
        }
        const int strat = modes[t] & 15, notrue = (modes[t] >> 4) & 1;
        for (; r < r1; ++r) emit(t, r, walk(c.prog, roots[t], X + r * k, strat, notrue));
    }
}

bool use_avx512(const Call &c) {
#if defined(__x86_64__)
    // int32 gather offsets: the matrix must stay below 2^31 elements; FJA_WALK_SCALAR=1 forces
    // the scalar walk (tests compare the two)
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") && c.n * c.k < (Py_ssize_t(1) << 31) &&
           !std::getenv("FJA_WALK_SCALAR");
#else
    (void)c;
    return false;
#endif
}

// numpy's pairwise summation of a contiguous float64 run (the algorithm np.add.reduce applies to
// every row of a C-contiguous [rows, T] matrix): 8 partial sums below 128 elements, halving above.
// Reproducing it keeps the native ensemble sum bit-identical to `_regress`'s np.sum.
double pairwise_sum(const double *a, Py_ssize_t n) {
    if (n < 8) {
        double res = 0.;
        for (Py_ssize_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        Py_ssize_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    Py_ssize_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

// Row blocks over worker threads (set_walk_threads / FJA_HOST_THREADS, default 1: the
// reference's one-record-at-a-time subtask is single-threaded). fn(r0, r1, worker); every block
// writes only its own rows, so the result does not depend on the thread count.
std::atomic<int> g_walk_threads{-1};

int walk_threads() {
    int t = g_walk_threads.load(std::memory_order_relaxed);
    if (t < 0) {
        const char *e = std::getenv("FJA_HOST_THREADS");
        t = e ? std::atoi(e) : 1;
        t = t < 1 ? 1 : (t > 256 ? 256 : t);
        g_walk_threads.store(t, std::memory_order_relaxed);
    }
    return t;
}

template <class Fn>
void for_blocks(Py_ssize_t n, Fn &&fn) {
    const Py_ssize_t nb = (n + ROW_BLOCK - 1) / ROW_BLOCK;
    Py_ssize_t threads = walk_threads();
    const Py_ssize_t by_size = nb / 16;  // >= 16 blocks (4096 rows) per extra thread
    if (threads > by_size) threads = by_size;
    if (threads <= 1) {
        for (Py_ssize_t b = 0; b < nb; ++b) fn(b * ROW_BLOCK, std::min(n, (b + 1) * ROW_BLOCK), 0);
        return;
    }
    std::atomic<Py_ssize_t> next{0};
    std::vector<std::thread> pool;
    pool.reserve(static_cast<size_t>(threads));
    for (Py_ssize_t w = 0; w < threads; ++w)
        pool.emplace_back([&, w] {
            for (;;) {
                const Py_ssize_t b = next.fetch_add(1);
                if (b >= nb) break;
                fn(b * ROW_BLOCK, std::min(n, (b + 1) * ROW_BLOCK), static_cast<int>(w));
            }
        });
    for (auto &t : pool) t.join();
}

PyObject *set_walk_threads(PyObject *, PyObject *args) {
    int t;
    if (!PyArg_ParseTuple(args, "i", &t)) return nullptr;
    g_walk_threads.store(t < 1 ? 1 : (t > 256 ? 256 : t));
    Py_RETURN_NONE;
}

PyObject *forest_leaves(PyObject *, PyObject *args) {
    Call c;
    if (!c.parse(args, Kind::LEAVES)) return nullptr;
    const int32_t *roots = static_cast<const int32_t *>(c.roots.b.buf);
    const double *X = static_cast<const double *>(c.X.b.buf);
    int32_t *out = static_cast<int32_t *>(c.out.b.buf);
    const Py_ssize_t n = c.n;
    const bool avx = use_avx512(c);
    const Fixed *fc = cached_fixed(c);
    Py_BEGIN_ALLOW_THREADS
    Fixed local;
    if (fc == nullptr) compile_all(c, local);
    const Fixed &f = fc ? *fc : local;
    for_blocks(n, [&](Py_ssize_t r0, Py_ssize_t r1, int) {
        run_block(c, f, X, r0, r1, avx, [&](Py_ssize_t t, Py_ssize_t r, int32_t g) {
            out[t * n + r] = g < 0 ? -1 : g - roots[t];
        });
    });
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

PyObject *forest_values(PyObject *, PyObject *args) {
    Call c;
    if (!c.parse(args, Kind::VALUES)) return nullptr;
    const double *X = static_cast<const double *>(c.X.b.buf);
    const double *lv = static_cast<const double *>(c.leafval.b.buf);
    double *out = static_cast<double *>(c.out.b.buf);
    const Py_ssize_t n = c.n, T = c.T;
    const bool avx = use_avx512(c);
    const Fixed *fc = cached_fixed(c);
    Py_BEGIN_ALLOW_THREADS
    Fixed local;
    if (fc == nullptr) compile_all(c, local);
    const Fixed &f = fc ? *fc : local;
    for_blocks(n, [&](Py_ssize_t r0, Py_ssize_t r1, int) {
        run_block(c, f, X, r0, r1, avx, [&](Py_ssize_t t, Py_ssize_t r, int32_t g) {
            out[r * T + t] = g < 0 ? NAN : lv[g];
        });
    });
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

// forest_sums(..., X, k, leafval, weights or None, out f64 [n]): per row, the numpy pairwise sum of
// the T tree values (times weights[t] when given) in tree order; NaN where any tree is null.
PyObject *forest_sums(PyObject *, PyObject *args) {
    Call c;
    if (!c.parse(args, Kind::SUMS)) return nullptr;
    const double *X = static_cast<const double *>(c.X.b.buf);
    const double *lv = static_cast<const double *>(c.leafval.b.buf);
    const double *w = c.has_weights ? static_cast<const double *>(c.weights.b.buf) : nullptr;
    double *out = static_cast<double *>(c.out.b.buf);
    const Py_ssize_t n = c.n, T = c.T;
    const bool avx = use_avx512(c);
    std::vector<double> buf;  // one ROW_BLOCK x T slab per worker (rows of one block at most)
    const size_t slab_rows = static_cast<size_t>(n < ROW_BLOCK ? (n > 0 ? n : 1) : ROW_BLOCK);
    try {
        buf.resize(slab_rows * static_cast<size_t>(T) * static_cast<size_t>(walk_threads()));
    } catch (const std::bad_alloc &) {
        return PyErr_NoMemory();
    }
    const Fixed *fc = cached_fixed(c);
    Py_BEGIN_ALLOW_THREADS
    Fixed local;
    if (fc == nullptr) compile_all(c, local);
    const Fixed &f = fc ? *fc : local;
    for_blocks(n, [&](Py_ssize_t r0, Py_ssize_t r1, int worker) {
        double *bb = buf.data() + static_cast<size_t>(worker) * slab_rows * static_cast<size_t>(T);
        run_block(c, f, X, r0, r1, avx, [&](Py_ssize_t t, Py_ssize_t r, int32_t g) {
            const double v = g < 0 ? NAN : lv[g];
            bb[(r - r0) * T + t] = w ? v * w[t] : v;
        });
        for (Py_ssize_t r = r0; r < r1; ++r) out[r] = pairwise_sum(bb + (r - r0) * T, T);
    });
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

// forest_votes(..., X, k, cls int32 [n_nodes] (class of a scoring node, -1 = no score), weights f64 [T],
// C, acc f64 [n, C], wsum f64 [n], count int32 [n], anymiss u8 [n]): a (weighted) majority vote --
// acc[r, cls] += w[t] and wsum[r] += w[t] for every tree with a class, in tree order per row (the
// additions of MiningEvaluator._classify / _vote_native), count = such trees, anymiss = some tree
// without one. Outputs are overwritten.
PyObject *forest_votes(PyObject *, PyObject *args) {
    Call c;
    if (!c.parse(args, Kind::VOTES)) return nullptr;
    const double *X = static_cast<const double *>(c.X.b.buf);
    const int32_t *ct = static_cast<const int32_t *>(c.cls.b.buf);
    const double *w = static_cast<const double *>(c.weights.b.buf);
    double *acc = static_cast<double *>(c.out.b.buf);
    double *ws = static_cast<double *>(c.wsum.b.buf);
    int32_t *cnt = static_cast<int32_t *>(c.cnt.b.buf);
    uint8_t *miss = static_cast<uint8_t *>(c.miss.b.buf);
    const Py_ssize_t n = c.n, C = c.C;
    const bool avx = use_avx512(c);
    const Fixed *fc = cached_fixed(c);
    Py_BEGIN_ALLOW_THREADS
    Fixed local;
    if (fc == nullptr) compile_all(c, local);
    const Fixed &f = fc ? *fc : local;
    for_blocks(n, [&](Py_ssize_t r0, Py_ssize_t r1, int) {
        for (Py_ssize_t r = r0; r < r1; ++r) {
            for (Py_ssize_t j = 0; j < C; ++j) acc[r * C + j] = 0.0;
            ws[r] = 0.0;
            cnt[r] = 0;
            miss[r] = 0;
        }
        run_block(c, f, X, r0, r1, avx, [&](Py_ssize_t t, Py_ssize_t r, int32_t g) {
            const int32_t k = g < 0 ? -1 : ct[g];
            if (k < 0) {
                miss[r] = 1;
                return;
            }
            acc[r * C + k] += w[t];
            ws[r] += w[t];
            ++cnt[r];
        });
    });
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

// forest_compile(nodes_i, nodes_d, kids, preds_i, preds_d, aux_i, aux_d, roots, modes, k) -> capsule
PyObject *forest_compile(PyObject *, PyObject *args) {
    PyObject *o[9];
    Call c;
    if (!PyArg_ParseTuple(args, "OOOOOOOOOn", &o[0], &o[1], &o[2], &o[3], &o[4], &o[5], &o[6], &o[7], &o[8], &c.k))
        return nullptr;
    if (!c.ni.get(o[0], "i", 4, false, "nodes_i") || !c.nd.get(o[1], "d", 8, false, "nodes_d") ||
        !c.kids.get(o[2], "i", 4, false, "kids") || !c.pi.get(o[3], "i", 4, false, "preds_i") ||
        !c.pd.get(o[4], "d", 8, false, "preds_d") || !c.ai.get(o[5], "i", 4, false, "aux_i") ||
        !c.ad.get(o[6], "d", 8, false, "aux_d") || !c.roots.get(o[7], "i", 4, false, "roots") ||
        !c.modes.get(o[8], "i", 4, false, "modes"))
        return nullptr;
    c.prog = Program{static_cast<const int32_t *>(c.ni.b.buf),  static_cast<const double *>(c.nd.b.buf),
                     static_cast<const int32_t *>(c.kids.b.buf), static_cast<const int32_t *>(c.pi.b.buf),
                     static_cast<const double *>(c.pd.b.buf),   static_cast<const int32_t *>(c.ai.b.buf),
                     static_cast<const double *>(c.ad.b.buf),   c.ni.n() / 8, c.kids.n(), c.pi.n() / 4, c.ai.n(),
                     c.ad.n()};
    c.T = c.roots.n();
    if (c.modes.n() != c.T || c.nd.n() != c.prog.n_nodes || c.pd.n() != c.prog.n_preds || c.k < 1) {
        PyErr_SetString(PyExc_ValueError, "tree walk: inconsistent program shapes");
        return nullptr;
    }
    if (!c.validate()) return nullptr;
    Cached *h = new (std::nothrow) Cached();
    if (h == nullptr) return PyErr_NoMemory();
    compile_all(c, h->f);
    h->ni = c.ni.b.buf;
    h->kids = c.kids.b.buf;
    h->pi = c.pi.b.buf;
    h->roots = c.roots.b.buf;
    h->modes = c.modes.b.buf;
    h->nd = c.nd.b.buf;
    h->pd = c.pd.b.buf;
    h->ai = c.ai.b.buf;
    h->ad = c.ad.b.buf;
    h->n_nodes = c.prog.n_nodes;
    h->T = c.T;
    h->k = c.k;
    h->n_kids = c.prog.n_kids;
    h->n_preds = c.prog.n_preds;
    h->n_ai = c.prog.n_ai;
    h->n_ad = c.prog.n_ad;
    PyObject *cap = PyCapsule_New(h, CAPSULE, drop_cached);
    if (cap == nullptr) delete h;
    return cap;
}

}  // namespace

PyObject *fja_forest_compile(PyObject *self, PyObject *args) { return forest_compile(self, args); }
PyObject *fja_set_walk_threads(PyObject *self, PyObject *args) { return set_walk_threads(self, args); }
PyObject *fja_forest_leaves(PyObject *self, PyObject *args) { return forest_leaves(self, args); }
PyObject *fja_forest_values(PyObject *self, PyObject *args) { return forest_values(self, args); }
PyObject *fja_forest_sums(PyObject *self, PyObject *args) { return forest_sums(self, args); }
PyObject *fja_forest_votes(PyObject *self, PyObject *args) { return forest_votes(self, args); }
