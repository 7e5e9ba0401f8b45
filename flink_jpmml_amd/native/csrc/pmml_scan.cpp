// Streaming PMML tree reader: decision-tree bodies straight into flat arrays, no DOM.
//
// The reference loads models of "several hundreds of MegaBytes" (`README.md:239-242`) through
// JAXB into a full object graph (`S/api/PmmlModel.scala:53-58`). Nearly all of such a document is
// <Node> elements of TreeModels (random forests / GBDTs). This scanner makes one pass over the
// document bytes and
//
//   * parses every TreeModel's root <Node> subtree into per-tree flat arrays (preorder):
//     parent, children (CSR), id / score / defaultChild (interned strings, score also as a double),
//     recordCount, the node predicate (True / False / SimplePredicate field-operator-value with the
//     value also as a double; SimpleSetPredicate / CompoundPredicate as a byte span of the source for
//     the Python parser), ScoreDistributions (value, recordCount, probability, confidence);
//   * writes a *skeleton* copy of the document in which each such subtree is replaced by
//     <Node fjaFlat="k"/>. The skeleton (DataDictionary, MiningSchemas, Outputs, Targets, …) is
//     small and goes through the regular Python parser, which attaches flat tree k to TreeModel k.
//
// Anything unexpected inside a tree (embedded models, malformed markup) makes scan_trees return
// None and the caller parses the document the ordinary way — results never depend on which path
// ran.

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#define NO_IMPORT_ARRAY
#define PY_ARRAY_UNIQUE_SYMBOL fja_fastpath_ARRAY_API
#include <numpy/arrayobject.h>

#include <cctype>
#include <cmath>
#include <cstdint>
#include <limits>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace {

constexpr double kNaN = std::numeric_limits<double>::quiet_NaN();

enum PredKind : int8_t { P_NONE = -1, P_TRUE = 0, P_FALSE = 1, P_SIMPLE = 2, P_RAW = 3 };

struct Strings {
    std::unordered_map<std::string, int32_t> index;
    std::vector<std::string> values;
    int32_t intern(const std::string &s) {
        auto it = index.find(s);
        if (it != index.end()) return it->second;
        int32_t k = static_cast<int32_t>(values.size());
        index.emplace(s, k);
        values.push_back(s);
        return k;
    }
};

struct Tree {
    std::vector<int32_t> parent, id_s, score_s, default_s, pred_field, pred_value_s, depth;
    std::vector<double> score_d, record_count, pred_value_d;
    std::vector<int8_t> pred_kind, pred_op, default_pos;
    std::vector<int64_t> raw_start, raw_end;
    std::vector<int32_t> dist_node, dist_value_s;
    std::vector<double> dist_count, dist_prob, dist_conf;
    int32_t add_node(int32_t par, int32_t d) {
        parent.push_back(par);
        depth.push_back(d);
        id_s.push_back(-1);
        score_s.push_back(-1);
        default_s.push_back(-1);
        pred_field.push_back(-1);
        pred_value_s.push_back(-1);
        score_d.push_back(kNaN);
        record_count.push_back(kNaN);
        pred_value_d.push_back(kNaN);
        pred_kind.push_back(P_NONE);
        pred_op.push_back(-1);
        default_pos.push_back(-1);
        raw_start.push_back(-1);
        raw_end.push_back(-1);
        return static_cast<int32_t>(parent.size()) - 1;
    }
};

struct Attr {
    std::string_view name;  // local name
    std::string value;      // entity-decoded
};

struct Tag {
    std::string_view name;  // local name (namespace prefix stripped)
    bool end = false;       // </x>
    bool self_close = false;
    size_t start = 0, stop = 0;  // [start, stop) of the markup incl. '<' and '>'
    std::vector<Attr> attrs;
    const std::string *attr(std::string_view n) const {
        for (auto &a : attrs)
            if (a.name == n) return &a.value;
        return nullptr;
    }
};

bool is_name_char(char c) {
    return std::isalnum(static_cast<unsigned char>(c)) || c == '_' || c == '-' || c == '.' || c == ':';
}

std::string_view local_name(std::string_view q) {
    size_t p = q.rfind(':');
    return p == std::string_view::npos ? q : q.substr(p + 1);
}

void append_utf8(std::string &out, unsigned long cp) {
    if (cp < 0x80) {
        out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
        out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
        out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
        out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
        out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
        out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
        out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
        out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
}

// Decode XML entity references of an attribute value; false on a malformed reference.
bool decode(std::string_view in, std::string &out) {
    out.clear();
    out.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        char c = in[i];
        if (c != '&') {
            out.push_back(c);
            continue;
        }
        size_t semi = in.find(';', i);
        if (semi == std::string_view::npos) return false;
        std::string_view ent = in.substr(i + 1, semi - i - 1);
        if (ent == "lt") out.push_back('<');
        else if (ent == "gt") out.push_back('>');
        else if (ent == "amp") out.push_back('&');
        else if (ent == "quot") out.push_back('"');
        else if (ent == "apos") out.push_back('\'');
        else if (!ent.empty() && ent[0] == '#') {
            std::string num(ent.substr(1));
            char *end = nullptr;
            unsigned long cp = (!num.empty() && (num[0] == 'x' || num[0] == 'X'))
                                   ? std::strtoul(num.c_str() + 1, &end, 16)
                                   : std::strtoul(num.c_str(), &end, 10);
            if (!end || *end) return false;
            append_utf8(out, cp);
        } else {
            return false;
        }
        i = semi;
    }
    return true;
}

double to_double(const std::string &s) {
    if (s.empty()) return kNaN;
    const char *b = s.c_str();
    while (*b == ' ' || *b == '\t' || *b == '\n' || *b == '\r') ++b;
    char *end = nullptr;
    double v = std::strtod(b, &end);
    if (end == b) return kNaN;
    while (*end == ' ' || *end == '\t' || *end == '\n' || *end == '\r') ++end;
    return *end ? kNaN : v;
}

int8_t op_code(const std::string &op) {
    static const char *ops[] = {"equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan",
                                "greaterOrEqual", "isMissing", "isNotMissing"};
    for (int8_t k = 0; k < 8; ++k)
        if (op == ops[k]) return k;
    return -1;
}

class Scanner {
  public:
    Scanner(const char *buf, size_t n) : b_(buf), n_(n) {}

    // Next markup item at or after pos_: start/end tag into `t` (true), or false at end / error.
    // Text, comments, PIs, DOCTYPE and CDATA are skipped (copied by the caller through spans).
    bool next_tag(Tag &t) {
        while (pos_ < n_) {
            const char *lt = static_cast<const char *>(std::memchr(b_ + pos_, '<', n_ - pos_));
            if (!lt) {
                pos_ = n_;
                return false;
            }
            size_t i = static_cast<size_t>(lt - b_);
            if (starts(i, "<!--")) {
                if (!skip_to(i + 4, "-->")) return fail();
                continue;
            }
            if (starts(i, "<![CDATA[")) {
                if (!skip_to(i + 9, "]]>")) return fail();
                continue;
            }
            if (starts(i, "<?")) {
                if (!skip_to(i + 2, "?>")) return fail();
                continue;
            }
            if (starts(i, "<!")) {
                if (!skip_to(i + 2, ">")) return fail();
                continue;
            }
            return read_tag(i, t);
        }
        return false;
    }

    size_t pos() const { return pos_; }
    void seek(size_t p) { pos_ = p; }
    bool error() const { return error_; }

    // Skip the element whose start tag `t` was just read (nothing if it was self-closing).
    bool skip_element(const Tag &t) {
        if (t.self_close) return true;
        int depth = 1;
        Tag u;
        while (depth > 0) {
            if (!next_tag(u)) return fail();
            if (u.end) --depth;
            else if (!u.self_close) ++depth;
        }
        return true;
    }

  private:
    bool starts(size_t i, const char *s) const {
        size_t m = std::strlen(s);
        return i + m <= n_ && std::memcmp(b_ + i, s, m) == 0;
    }
    bool skip_to(size_t from, const char *s) {
        size_t m = std::strlen(s);
        const char *hit = static_cast<const char *>(memmem(b_ + from, n_ - from, s, m));
        if (!hit) return false;
        pos_ = static_cast<size_t>(hit - b_) + m;
        return true;
    }
    bool fail() {
        error_ = true;
        pos_ = n_;
        return false;
    }
    void ws(size_t &i) const {
        while (i < n_ && (b_[i] == ' ' || b_[i] == '\t' || b_[i] == '\n' || b_[i] == '\r')) ++i;
    }
    bool read_tag(size_t i, Tag &t) {
        t.start = i;
        t.end = false;
        t.self_close = false;
        t.attrs.clear();
        size_t k = i + 1;
        if (k < n_ && b_[k] == '/') {
            t.end = true;
            ++k;
        }
        size_t s = k;
        while (k < n_ && is_name_char(b_[k])) ++k;
        if (k == s) return fail();
        t.name = local_name(std::string_view(b_ + s, k - s));
        for (;;) {
            ws(k);
            if (k >= n_) return fail();
            if (b_[k] == '>') {
                ++k;
                break;
            }
            if (b_[k] == '/' && k + 1 < n_ && b_[k + 1] == '>') {
                t.self_close = true;
                k += 2;
                break;
            }
            if (t.end) return fail();
            size_t as = k;
            while (k < n_ && is_name_char(b_[k])) ++k;
            if (k == as) return fail();
            std::string_view an = local_name(std::string_view(b_ + as, k - as));
            ws(k);
            if (k >= n_ || b_[k] != '=') return fail();
            ++k;
            ws(k);
            if (k >= n_ || (b_[k] != '"' && b_[k] != '\'')) return fail();
            char q = b_[k++];
            const char *qe = static_cast<const char *>(std::memchr(b_ + k, q, n_ - k));
            if (!qe) return fail();
            Attr a;
            a.name = an;
            if (!decode(std::string_view(b_ + k, static_cast<size_t>(qe - (b_ + k))), a.value)) return fail();
            t.attrs.push_back(std::move(a));
            k = static_cast<size_t>(qe - b_) + 1;
        }
        t.stop = k;
        pos_ = k;
        return true;
    }

    const char *b_;
    size_t n_;
    size_t pos_ = 0;
    bool error_ = false;
};

// Parse the <Node> subtree whose start tag `root` was just read into `tr`. False on anything the
// flat form does not represent (the caller then falls back to the Python parser).
bool parse_tree(Scanner &sc, const Tag &root, Tree &tr, Strings &str) {
    struct Open {
        int32_t node;
    };
    std::vector<Open> stack;
    auto open_node = [&](const Tag &t, int32_t par) -> int32_t {
        int32_t d = par < 0 ? 0 : tr.depth[par] + 1;
        int32_t k = tr.add_node(par, d);
        if (auto v = t.attr("id")) tr.id_s[k] = str.intern(*v);
        if (auto v = t.attr("score")) {
            tr.score_s[k] = str.intern(*v);
            tr.score_d[k] = to_double(*v);
        }
        if (auto v = t.attr("recordCount")) tr.record_count[k] = to_double(*v);
        if (auto v = t.attr("defaultChild")) tr.default_s[k] = str.intern(*v);
        return k;
    };
    int32_t r = open_node(root, -1);
    if (root.self_close) return true;
    stack.push_back({r});
    Tag t;
    while (!stack.empty()) {
        if (!sc.next_tag(t)) return false;
        int32_t cur = stack.back().node;
        if (t.end) {
            if (t.name != "Node") return false;
            stack.pop_back();
            continue;
        }
        const std::string_view nm = t.name;
        if (nm == "Node") {
            int32_t k = open_node(t, cur);
            if (!t.self_close) stack.push_back({k});
        } else if (nm == "True" || nm == "False") {
            if (tr.pred_kind[cur] != P_NONE) return false;
            tr.pred_kind[cur] = nm == "True" ? P_TRUE : P_FALSE;
            if (!sc.skip_element(t)) return false;
        } else if (nm == "SimplePredicate") {
            if (tr.pred_kind[cur] != P_NONE) return false;
            const std::string *f = t.attr("field"), *op = t.attr("operator"), *v = t.attr("value");
            if (!f || !op) return false;
            tr.pred_kind[cur] = P_SIMPLE;
            tr.pred_field[cur] = str.intern(*f);
            tr.pred_op[cur] = op_code(*op);
            if (tr.pred_op[cur] < 0) return false;
            if (v) {
                tr.pred_value_s[cur] = str.intern(*v);
                tr.pred_value_d[cur] = to_double(*v);
            }
            if (!sc.skip_element(t)) return false;
        } else if (nm == "SimpleSetPredicate" || nm == "CompoundPredicate") {
            if (tr.pred_kind[cur] != P_NONE) return false;
            tr.pred_kind[cur] = P_RAW;
            tr.raw_start[cur] = static_cast<int64_t>(t.start);
            if (!sc.skip_element(t)) return false;
            tr.raw_end[cur] = static_cast<int64_t>(sc.pos());
        } else if (nm == "ScoreDistribution") {
            const std::string *v = t.attr("value");
            if (!v) return false;
            tr.dist_node.push_back(cur);
            tr.dist_value_s.push_back(str.intern(*v));
            const std::string *rc = t.attr("recordCount"), *pr = t.attr("probability"), *cf = t.attr("confidence");
            tr.dist_count.push_back(rc ? to_double(*rc) : 0.0);
            tr.dist_prob.push_back(pr ? to_double(*pr) : kNaN);
            tr.dist_conf.push_back(cf ? to_double(*cf) : kNaN);
            if (!sc.skip_element(t)) return false;
        } else if (nm == "Regression" || nm == "DecisionTree") {
            return false;  // embedded models: the Python parser reports them
        } else {
            if (!sc.skip_element(t)) return false;  // Extension, Partition, …
        }
    }
    // defaultChild -> child position (the child whose id equals it)
    const int32_t n = static_cast<int32_t>(tr.parent.size());
    std::vector<int32_t> seen(n, 0);
    for (int32_t k = 1; k < n; ++k) {
        int32_t p = tr.parent[k];
        int32_t pos = seen[p]++;
        if (tr.default_s[p] >= 0 && tr.id_s[k] == tr.default_s[p] && tr.default_pos[p] < 0)
            tr.default_pos[p] = static_cast<int8_t>(pos < 127 ? pos : 127);
    }
    return true;
}

template <typename T>
PyObject *to_array(const std::vector<T> &v, int typenum) {
    npy_intp dims[1] = {static_cast<npy_intp>(v.size())};
    PyObject *a = PyArray_SimpleNew(1, dims, typenum);
    if (a && !v.empty()) std::memcpy(PyArray_DATA(reinterpret_cast<PyArrayObject *>(a)), v.data(), v.size() * sizeof(T));
    return a;
}

bool put(PyObject *d, const char *k, PyObject *v) {
    if (!v) return false;
    int r = PyDict_SetItemString(d, k, v);
    Py_DECREF(v);
    return r == 0;
}

PyObject *tree_dict(const Tree &t) {
    PyObject *d = PyDict_New();
    if (!d) return nullptr;
    bool ok = put(d, "parent", to_array(t.parent, NPY_INT32)) && put(d, "depth", to_array(t.depth, NPY_INT32)) &&
              put(d, "id_s", to_array(t.id_s, NPY_INT32)) && put(d, "score_s", to_array(t.score_s, NPY_INT32)) &&
              put(d, "score_d", to_array(t.score_d, NPY_FLOAT64)) &&
              put(d, "record_count", to_array(t.record_count, NPY_FLOAT64)) &&
              put(d, "default_s", to_array(t.default_s, NPY_INT32)) &&
              put(d, "default_pos", to_array(t.default_pos, NPY_INT8)) &&
              put(d, "pred_kind", to_array(t.pred_kind, NPY_INT8)) &&
              put(d, "pred_field", to_array(t.pred_field, NPY_INT32)) &&
              put(d, "pred_op", to_array(t.pred_op, NPY_INT8)) &&
              put(d, "pred_value_s", to_array(t.pred_value_s, NPY_INT32)) &&
              put(d, "pred_value_d", to_array(t.pred_value_d, NPY_FLOAT64)) &&
              put(d, "raw_start", to_array(t.raw_start, NPY_INT64)) && put(d, "raw_end", to_array(t.raw_end, NPY_INT64)) &&
              put(d, "dist_node", to_array(t.dist_node, NPY_INT32)) &&
              put(d, "dist_value_s", to_array(t.dist_value_s, NPY_INT32)) &&
              put(d, "dist_count", to_array(t.dist_count, NPY_FLOAT64)) &&
              put(d, "dist_prob", to_array(t.dist_prob, NPY_FLOAT64)) &&
              put(d, "dist_conf", to_array(t.dist_conf, NPY_FLOAT64));
    if (!ok) {
        Py_DECREF(d);
        return nullptr;
    }
    return d;
}

}  // namespace

// scan_trees(doc: bytes-like) -> (skeleton: bytes, trees: list[dict], strings: list[str]) or None
PyObject *fja_scan_trees(PyObject *, PyObject *args) {
    Py_buffer view;
    if (!PyArg_ParseTuple(args, "y*", &view)) return nullptr;
    const char *buf = static_cast<const char *>(view.buf);
    const size_t n = static_cast<size_t>(view.len);
    std::vector<Tree> trees;
    Strings str;
    std::string skel;
    bool ok = true;
    Py_BEGIN_ALLOW_THREADS;
    skel.reserve(1 << 16);
    Scanner sc(buf, n);
    size_t copied = 0;  // source bytes up to here are in the skeleton
    Tag t;
    std::vector<bool> model_stack;  // per open element: is it a TreeModel awaiting its root Node
    while (sc.next_tag(t)) {
        if (t.end) {
            if (!model_stack.empty()) model_stack.pop_back();
            continue;
        }
        if (t.name == "Node" && !model_stack.empty() && model_stack.back()) {
            // the root Node of the innermost open TreeModel
            trees.emplace_back();
            if (!parse_tree(sc, t, trees.back(), str)) {
                ok = false;
                break;
            }
            skel.append(buf + copied, t.start - copied);
            skel.append("<Node fjaFlat=\"" + std::to_string(trees.size() - 1) + "\"/>");
            copied = sc.pos();
            model_stack.back() = false;
            continue;
        }
        if (!t.self_close) model_stack.push_back(t.name == "TreeModel");
    }
    if (sc.error()) ok = false;
    if (ok) skel.append(buf + copied, n - copied);
    Py_END_ALLOW_THREADS;
    PyBuffer_Release(&view);
    if (!ok || trees.empty()) Py_RETURN_NONE;
    PyObject *out_trees = PyList_New(static_cast<Py_ssize_t>(trees.size()));
    if (!out_trees) return nullptr;
    for (size_t i = 0; i < trees.size(); ++i) {
        PyObject *d = tree_dict(trees[i]);
        if (!d) {
            Py_DECREF(out_trees);
            return nullptr;
        }
        PyList_SET_ITEM(out_trees, static_cast<Py_ssize_t>(i), d);
    }
    PyObject *strings = PyList_New(static_cast<Py_ssize_t>(str.values.size()));
    if (!strings) {
        Py_DECREF(out_trees);
        return nullptr;
    }
    for (size_t i = 0; i < str.values.size(); ++i) {
        PyObject *s = PyUnicode_DecodeUTF8(str.values[i].data(), static_cast<Py_ssize_t>(str.values[i].size()),
                                           "replace");
        if (!s) {
            Py_DECREF(out_trees);
            Py_DECREF(strings);
            return nullptr;
        }
        PyList_SET_ITEM(strings, static_cast<Py_ssize_t>(i), s);
    }
    PyObject *sk = PyBytes_FromStringAndSize(skel.data(), static_cast<Py_ssize_t>(skel.size()));
    if (!sk) {
        Py_DECREF(out_trees);
        Py_DECREF(strings);
        return nullptr;
    }
    return Py_BuildValue("(NNN)", sk, out_trees, strings);
}
