// Streaming PMML tree reader: decision-tree bodies straight into flat arrays, no DOM.
//
// The reference loads models of "several hundreds of MegaBytes" (`README.md:239-242`) through
// JAXB into a full object graph (`S/api/PmmlModel.scala:53-58`); a malformed document fails the
// load and with it the job (`S/api/functions/EvaluationFunction.scala:45-48`). Nearly all of such
// a document is <Node> elements of TreeModels (random forests / GBDTs). This scanner makes one pass
// over the document bytes and
//
//   * parses every TreeModel's root <Node> subtree into per-tree flat arrays (preorder):
//     parent, children (CSR), id / score / defaultChild (interned strings, score also as a double),
//     recordCount, the node predicate (True / False / SimplePredicate field-operator-value with the
//     value also as a double; SimpleSetPredicate / CompoundPredicate as a byte span of the source for
//     the Python parser), ScoreDistributions (value, recordCount, probability, confidence);
//   * writes a *skeleton* copy of the document in which each such subtree is replaced by
//     <Node fjaFlat="k"/>. The skeleton (DataDictionary, MiningSchemas, Outputs, Targets, …) is
//     small and goes through the regular Python parser (expat), which attaches flat tree k to
//     TreeModel k.
//
// Fail-closed contract: the scanner never accepts a document the DOM path rejects, and never
// produces a different model from one it accepts. It therefore checks XML 1.0 well-formedness
// itself — UTF-8 and the XML Char range over the whole document, name grammar, matched end tags,
// quoted attribute values without '<', unique attributes, whitespace between attributes, entity /
// character references, comment / CDATA grammar, namespace prefixes in scope — and it *declines*
// (scan_trees returns None, the caller parses the ordinary way, whose verdict then stands) on
// anything it does not model exactly: embedded models, unknown child elements of a <Node>, a node
// without (or with two) predicates, numeric attributes that do not parse as Python floats,
// namespace declarations or prefixed attributes inside a tree body, DOCTYPEs, processing
// instructions inside a body, non-UTF-8 encodings. Declining is always safe; accepting torn markup
// is not. `tests/test_scan_fuzz.py` holds the scanner to that against ElementTree with a mutation
// corpus, also under ASan + UBSan.

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#define NO_IMPORT_ARRAY
#define PY_ARRAY_UNIQUE_SYMBOL fja_fastpath_ARRAY_API
#include <numpy/arrayobject.h>

#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
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
    std::string_view qname;  // as written (prefix kept)
    std::string value;       // entity-decoded, whitespace-normalised
};

struct Tag {
    std::string_view qname;  // as written
    std::string_view name;   // local name
    std::string_view prefix; // "" when unprefixed
    bool end = false;        // </x>
    bool self_close = false;
    bool has_ns_decl = false;   // carries xmlns / xmlns:p
    bool has_prefixed_attr = false;
    size_t start = 0, stop = 0;  // [start, stop) of the markup incl. '<' and '>'
    std::vector<Attr> attrs;
    const std::string *attr(std::string_view n) const {
        for (auto &a : attrs)
            if (a.qname == n) return &a.value;
        return nullptr;
    }
};

// ------------------------------------------------------------------------------ character level

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

inline bool is_name_start(char c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' || c == ':';
}
inline bool is_name_char(char c) {
    return is_name_start(c) || (c >= '0' && c <= '9') || c == '-' || c == '.';
}

inline bool is_xml_char(uint32_t cp) {
    return cp == 0x9 || cp == 0xA || cp == 0xD || (cp >= 0x20 && cp <= 0xD7FF) || (cp >= 0xE000 && cp <= 0xFFFD) ||
           (cp >= 0x10000 && cp <= 0x10FFFF);
}

// The whole document is well-formed UTF-8 and every character is an XML 1.0 Char (expat's first
// check). ASCII runs go 8 bytes at a time.
bool valid_utf8_xml_chars(const unsigned char *s, size_t n) {
    size_t i = 0;
    while (i < n) {
        if (i + 8 <= n) {
            uint64_t w;
            std::memcpy(&w, s + i, 8);
            // every byte in [0x20, 0x7F]: no high bit, and no byte below 0x20
            const uint64_t hi = w & 0x8080808080808080ULL;
            const uint64_t lo = (w - 0x2020202020202020ULL) & ~w & 0x8080808080808080ULL;
            if ((hi | lo) == 0) {
                i += 8;
                continue;
            }
        }
        const unsigned char c = s[i];
        if (c < 0x80) {
            if (c < 0x20 && c != 0x9 && c != 0xA && c != 0xD) return false;
            ++i;
            continue;
        }
        uint32_t cp;
        size_t len;
        if ((c & 0xE0) == 0xC0) {
            cp = c & 0x1F;
            len = 2;
        } else if ((c & 0xF0) == 0xE0) {
            cp = c & 0x0F;
            len = 3;
        } else if ((c & 0xF8) == 0xF0) {
            cp = c & 0x07;
            len = 4;
        } else {
            return false;
        }
        if (i + len > n) return false;
        for (size_t k = 1; k < len; ++k) {
            if ((s[i + k] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (s[i + k] & 0x3F);
        }
        // overlong forms and surrogates are not UTF-8
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000)) return false;
        if (cp >= 0xD800 && cp <= 0xDFFF) return false;
        if (!is_xml_char(cp)) return false;
        i += len;
    }
    return true;
}

void append_utf8(std::string &out, uint32_t cp) {
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

// One entity / character reference starting at in[i] == '&'. Appends its replacement text (if
// `out`) and returns the index of the terminating ';', or npos when the reference is malformed
// (undeclared entity, bad digits, a code point outside the Char range).
size_t reference(std::string_view in, size_t i, std::string *out) {
    const size_t semi = in.find(';', i + 1);
    if (semi == std::string_view::npos) return std::string_view::npos;
    const std::string_view ent = in.substr(i + 1, semi - i - 1);
    char rep = 0;
    if (ent == "lt") rep = '<';
    else if (ent == "gt") rep = '>';
    else if (ent == "amp") rep = '&';
    else if (ent == "quot") rep = '"';
    else if (ent == "apos") rep = '\'';
    if (rep) {
        if (out) out->push_back(rep);
        return semi;
    }
    if (ent.size() < 2 || ent[0] != '#') return std::string_view::npos;
    uint32_t cp = 0;
    if (ent[1] == 'x') {
        if (ent.size() < 3) return std::string_view::npos;
        for (size_t k = 2; k < ent.size(); ++k) {
            const char c = ent[k];
            uint32_t d;
            if (c >= '0' && c <= '9') d = static_cast<uint32_t>(c - '0');
            else if (c >= 'a' && c <= 'f') d = static_cast<uint32_t>(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') d = static_cast<uint32_t>(c - 'A' + 10);
            else return std::string_view::npos;
            cp = cp * 16 + d;
            if (cp > 0x10FFFF) return std::string_view::npos;
        }
    } else {
        for (size_t k = 1; k < ent.size(); ++k) {
            const char c = ent[k];
            if (c < '0' || c > '9') return std::string_view::npos;
            cp = cp * 10 + static_cast<uint32_t>(c - '0');
            if (cp > 0x10FFFF) return std::string_view::npos;
        }
    }
    if (!is_xml_char(cp)) return std::string_view::npos;
    if (out) append_utf8(*out, cp);
    return semi;
}

// Attribute value as the XML processor reports it: references replaced, literal white space
// normalised to ' ' (CR LF counts once). False on '<', a stray '&' or a malformed reference.
bool decode_attr(std::string_view in, std::string &out) {
    out.clear();
    out.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        const char c = in[i];
        if (c == '&') {
            i = reference(in, i, &out);
            if (i == std::string_view::npos) return false;
        } else if (c == '<') {
            return false;
        } else if (c == '\r') {
            out.push_back(' ');
            if (i + 1 < in.size() && in[i + 1] == '\n') ++i;
        } else if (c == '\n' || c == '\t') {
            out.push_back(' ');
        } else {
            out.push_back(c);
        }
    }
    return true;
}

// Character data between markup: every '&' starts a well-formed reference and "]]>" never occurs.
bool valid_text(std::string_view in) {
    for (size_t i = 0; i < in.size(); ++i) {
        const char c = in[i];
        if (c == '&') {
            i = reference(in, i, nullptr);
            if (i == std::string_view::npos) return false;
        } else if (c == ']' && i + 2 < in.size() && in[i + 1] == ']' && in[i + 2] == '>') {
            return false;
        }
    }
    return true;
}

// ------------------------------------------------------------------------------ numbers

// Python's float(str) for ASCII text: surrounding white space, an optional sign, then a decimal
// literal (digits may be grouped by single underscores) or inf / infinity / nan in any case.
// `ok` is false where Python raises ValueError. Strings with non-ASCII bytes are left to the
// Python side (flat.py patches them; Python also accepts Unicode digits and white space).
double py_float(const std::string &s, bool &ok) {
    ok = false;
    size_t b = 0, e = s.size();
    while (b < e && is_ws(s[b])) ++b;
    while (e > b && is_ws(s[e - 1])) --e;
    if (b == e) return kNaN;
    size_t i = b;
    bool neg = false;
    if (s[i] == '+' || s[i] == '-') {
        neg = s[i] == '-';
        ++i;
    }
    auto ieq = [&](const char *w) {
        const size_t m = std::strlen(w);
        if (e - i != m) return false;
        for (size_t k = 0; k < m; ++k)
            if ((s[i + k] | 0x20) != w[k]) return false;
        return true;
    };
    if (ieq("inf") || ieq("infinity")) {
        ok = true;
        return neg ? -std::numeric_limits<double>::infinity() : std::numeric_limits<double>::infinity();
    }
    if (ieq("nan")) {
        ok = true;
        return kNaN;
    }
    std::string clean;
    clean.reserve(e - b);
    if (neg) clean.push_back('-');
    // digitpart: digit (["_"] digit)*
    auto digits = [&](size_t &k) {
        size_t start = k;
        while (k < e) {
            if (s[k] >= '0' && s[k] <= '9') {
                clean.push_back(s[k]);
                ++k;
            } else if (s[k] == '_' && k > start && k + 1 < e && s[k - 1] >= '0' && s[k - 1] <= '9' &&
                       s[k + 1] >= '0' && s[k + 1] <= '9') {
                ++k;
            } else {
                break;
            }
        }
        return k > start;
    };
    bool int_part = digits(i);
    bool frac_part = false;
    if (i < e && s[i] == '.') {
        clean.push_back('.');
        ++i;
        frac_part = digits(i);
    }
    if (!int_part && !frac_part) return kNaN;
    if (i < e && (s[i] == 'e' || s[i] == 'E')) {
        clean.push_back('e');
        ++i;
        if (i < e && (s[i] == '+' || s[i] == '-')) clean.push_back(s[i++]);
        if (!digits(i)) return kNaN;
    }
    if (i != e) return kNaN;
    ok = true;
    return std::strtod(clean.c_str(), nullptr);
}

bool has_non_ascii(const std::string &s) {
    for (char c : s)
        if (static_cast<unsigned char>(c) >= 0x80) return true;
    return false;
}

// A numeric attribute the DOM path reads with float(): a value Python would reject (or one only
// Python can judge, non-ASCII) declines the scan.
bool numeric_attr(const std::string &s, double &v) {
    if (has_non_ascii(s)) return false;
    bool ok;
    v = py_float(s, ok);
    return ok;
}

// A string attribute that may also be numeric (score, split value): NaN where Python's float()
// fails. Non-ASCII strings stay NaN here and are settled in Python.
double maybe_number(const std::string &s) {
    if (has_non_ascii(s)) return kNaN;
    bool ok;
    double v = py_float(s, ok);
    return ok ? v : kNaN;
}

int8_t op_code(const std::string &op) {
    static const char *ops[] = {"equal", "notEqual", "lessThan", "lessOrEqual", "greaterThan",
                                "greaterOrEqual", "isMissing", "isNotMissing"};
    for (int8_t k = 0; k < 8; ++k)
        if (op == ops[k]) return k;
    return -1;
}

// ------------------------------------------------------------------------------ markup

class Scanner {
  public:
    Scanner(const char *buf, size_t n) : b_(buf), n_(n) {}

    // Next start / end tag into `t` (true), or false at the end of the document or on an error.
    // Character data, comments and CDATA sections are validated and skipped; processing
    // instructions are skipped outside tree bodies only; DOCTYPEs decline.
    bool next_tag(Tag &t) {
        while (pos_ < n_) {
            const char *lt = static_cast<const char *>(std::memchr(b_ + pos_, '<', n_ - pos_));
            const size_t i = lt ? static_cast<size_t>(lt - b_) : n_;
            if (!valid_text(std::string_view(b_ + pos_, i - pos_))) return fail();
            if (!lt) {
                pos_ = n_;
                return false;
            }
            if (starts(i, "<!--")) {
                // "--" only as part of the closing "-->"
                const char *dd = find(i + 4, "--");
                if (!dd || static_cast<size_t>(dd - b_) + 2 >= n_ || dd[2] != '>') return fail();
                pos_ = static_cast<size_t>(dd - b_) + 3;
                continue;
            }
            if (starts(i, "<![CDATA[")) {
                if (stack_.empty()) return fail();  // CDATA only inside an element
                const char *end = find(i + 9, "]]>");
                if (!end) return fail();
                pos_ = static_cast<size_t>(end - b_) + 3;
                continue;
            }
            if (starts(i, "<?")) {
                if (body_depth_ > 0) return fail();
                const char *end = find(i + 2, "?>");
                if (!end) return fail();
                pos_ = static_cast<size_t>(end - b_) + 2;
                continue;
            }
            if (starts(i, "<!")) return fail();  // DOCTYPE / stray markup declaration: decline
            return read_tag(i, t);
        }
        return false;
    }

    size_t pos() const { return pos_; }
    bool error() const { return error_; }
    size_t depth() const { return stack_.size(); }

    // Tree-body mode: stricter rules (no PIs, no namespace declarations, no prefixed attributes).
    void enter_body() { body_depth_ = stack_.size(); }
    void leave_body() { body_depth_ = 0; }
    // While a raw predicate is skipped every element must carry its root's prefix (flat.py
    // re-parses the span on its own, declaring only that prefix).
    void require_prefix(std::string_view p) {
        req_prefix_ = p;
        req_active_ = true;
    }
    void release_prefix() { req_active_ = false; }

    // Skip the element whose start tag `t` was just read (nothing if it was self-closing).
    bool skip_element(const Tag &t) {
        if (t.self_close) return true;
        const size_t target = stack_.size() - 1;
        Tag u;
        while (stack_.size() > target) {
            if (!next_tag(u)) return fail();
        }
        return true;
    }

    bool fail() {
        error_ = true;
        pos_ = n_;
        return false;
    }

  private:
    struct Frame {
        std::string_view qname;
        size_t ns_mark;  // prefixes_.size() before this element's declarations
    };

    bool starts(size_t i, const char *s) const {
        const size_t m = std::strlen(s);
        return i + m <= n_ && std::memcmp(b_ + i, s, m) == 0;
    }
    const char *find(size_t from, const char *s) const {
        const size_t m = std::strlen(s);
        if (from > n_) return nullptr;
        return static_cast<const char *>(memmem(b_ + from, n_ - from, s, m));
    }
    void ws(size_t &i) const {
        while (i < n_ && is_ws(b_[i])) ++i;
    }
    // XML Name at b_[k] (ASCII subset; anything else declines). Returns the end index or npos.
    size_t name_end(size_t k) const {
        if (k >= n_ || !is_name_start(b_[k])) return std::string_view::npos;
        ++k;
        while (k < n_ && is_name_char(b_[k])) ++k;
        return k;
    }
    // Split a QName; false for malformed prefixes ("a:", ":a", "a:b:c").
    static bool split_qname(std::string_view q, std::string_view &prefix, std::string_view &local) {
        const size_t p = q.find(':');
        if (p == std::string_view::npos) {
            prefix = std::string_view();
            local = q;
            return true;
        }
        if (p == 0 || p + 1 == q.size() || q.find(':', p + 1) != std::string_view::npos) return false;
        if (!is_name_start(q[p + 1]) || q[p + 1] == ':') return false;
        prefix = q.substr(0, p);
        local = q.substr(p + 1);
        return true;
    }
    bool prefix_bound(std::string_view p) const {
        if (p.empty() || p == "xml") return true;
        for (auto it = prefixes_.rbegin(); it != prefixes_.rend(); ++it)
            if (*it == p) return true;
        return false;
    }

    bool read_tag(size_t i, Tag &t) {
        t.start = i;
        t.end = false;
        t.self_close = false;
        t.has_ns_decl = false;
        t.has_prefixed_attr = false;
        t.attrs.clear();
        size_t k = i + 1;
        if (k < n_ && b_[k] == '/') {
            t.end = true;
            ++k;
        }
        const size_t s = k;
        k = name_end(k);
        if (k == std::string_view::npos) return fail();
        t.qname = std::string_view(b_ + s, k - s);
        if (!split_qname(t.qname, t.prefix, t.name)) return fail();
        if (t.end) {
            ws(k);
            if (k >= n_ || b_[k] != '>') return fail();
            ++k;
            if (stack_.empty() || stack_.back().qname != t.qname) return fail();
            prefixes_.resize(stack_.back().ns_mark);
            stack_.pop_back();
            t.stop = pos_ = k;
            return true;
        }
        const size_t ns_mark = prefixes_.size();
        for (;;) {
            const size_t before_ws = k;
            ws(k);
            if (k >= n_) return fail();
            if (b_[k] == '>') {
                ++k;
                break;
            }
            if (b_[k] == '/') {
                if (k + 1 >= n_ || b_[k + 1] != '>') return fail();
                t.self_close = true;
                k += 2;
                break;
            }
            if (k == before_ws) return fail();  // attributes are separated by white space
            const size_t as = k;
            k = name_end(k);
            if (k == std::string_view::npos) return fail();
            Attr a;
            a.qname = std::string_view(b_ + as, k - as);
            ws(k);
            if (k >= n_ || b_[k] != '=') return fail();
            ++k;
            ws(k);
            if (k >= n_ || (b_[k] != '"' && b_[k] != '\'')) return fail();
            const char q = b_[k++];
            const char *qe = static_cast<const char *>(std::memchr(b_ + k, q, n_ - k));
            if (!qe) return fail();
            if (!decode_attr(std::string_view(b_ + k, static_cast<size_t>(qe - (b_ + k))), a.value)) return fail();
            k = static_cast<size_t>(qe - b_) + 1;
            for (auto &o : t.attrs)
                if (o.qname == a.qname) return fail();  // duplicate attribute
            std::string_view ap, al;
            if (!split_qname(a.qname, ap, al)) return fail();
            if (a.qname == "xmlns" || ap == "xmlns") {
                t.has_ns_decl = true;
                if (ap == "xmlns") {
                    if (a.value.empty() || al == "xmlns") return fail();
                    prefixes_.push_back(al);
                }
            } else if (!ap.empty()) {
                t.has_prefixed_attr = true;
            }
            t.attrs.push_back(std::move(a));
        }
        t.stop = pos_ = k;
        if (stack_.size() >= kMaxDepth) return fail();
        if (!prefix_bound(t.prefix)) return fail();
        if (t.prefix == "xmlns") return fail();
        if (t.has_prefixed_attr) {
            // expanded-name uniqueness needs the namespace URIs: leave such documents to expat
            if (body_depth_ > 0) return fail();
            for (auto &a : t.attrs) {
                std::string_view ap, al;
                split_qname(a.qname, ap, al);
                if (ap != "xmlns" && !prefix_bound(ap)) return fail();
            }
        }
        if (body_depth_ > 0 && t.has_ns_decl) return fail();
        if (req_active_ && t.prefix != req_prefix_) return fail();
        if (t.self_close) {
            prefixes_.resize(ns_mark);
        } else {
            stack_.push_back({t.qname, ns_mark});
        }
        return true;
    }

    static constexpr size_t kMaxDepth = 1 << 16;
    const char *b_;
    size_t n_;
    size_t pos_ = 0;
    bool error_ = false;
    std::vector<Frame> stack_;
    std::vector<std::string_view> prefixes_;  // declared prefixes of the open elements, innermost last
    size_t body_depth_ = 0;                   // stack depth of a tree body's root (0: not in a body)
    std::string_view req_prefix_;
    bool req_active_ = false;
};

// Parse the <Node> subtree whose start tag `root` was just read into `tr`. False on anything the
// flat form does not represent exactly as the DOM parser would (the scan then declines).
bool parse_tree(Scanner &sc, const Tag &root, Tree &tr, Strings &str) {
    bool ok = true;
    auto open_node = [&](const Tag &t, int32_t par) -> int32_t {
        int32_t d = par < 0 ? 0 : tr.depth[par] + 1;
        int32_t k = tr.add_node(par, d);
        if (auto v = t.attr("id")) tr.id_s[k] = str.intern(*v);
        if (auto v = t.attr("score")) {
            tr.score_s[k] = str.intern(*v);
            tr.score_d[k] = maybe_number(*v);
        }
        if (auto v = t.attr("recordCount")) {
            double x = kNaN;
            if (!numeric_attr(*v, x)) ok = false;
            tr.record_count[k] = x;
        }
        if (auto v = t.attr("defaultChild")) tr.default_s[k] = str.intern(*v);
        return k;
    };
    const int32_t r = open_node(root, -1);
    if (!ok) return false;
    if (root.self_close) return tr.pred_kind[r] != P_NONE;  // a childless root has no predicate
    const size_t root_depth = sc.depth();  // the root <Node> is open at this depth
    std::vector<int32_t> stack{r};
    Tag t;
    while (!stack.empty()) {
        if (!sc.next_tag(t)) return false;
        const int32_t cur = stack.back();
        if (t.end) {
            // only <Node> elements are open here: the skipped ones close inside skip_element
            if (t.name != "Node") return false;
            if (tr.pred_kind[cur] == P_NONE) return false;  // the DOM parser raises "has no predicate"
            stack.pop_back();
            continue;
        }
        const std::string_view nm = t.name;
        if (nm == "Node") {
            int32_t k = open_node(t, cur);
            if (!ok) return false;
            if (t.self_close) return false;  // a leaf without predicate
            stack.push_back(k);
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
                tr.pred_value_d[cur] = maybe_number(*v);
            }
            if (!sc.skip_element(t)) return false;
        } else if (nm == "SimpleSetPredicate" || nm == "CompoundPredicate") {
            if (tr.pred_kind[cur] != P_NONE) return false;
            tr.pred_kind[cur] = P_RAW;
            tr.raw_start[cur] = static_cast<int64_t>(t.start);
            sc.require_prefix(t.prefix);
            const bool skipped = sc.skip_element(t);
            sc.release_prefix();
            if (!skipped) return false;
            tr.raw_end[cur] = static_cast<int64_t>(sc.pos());
        } else if (nm == "ScoreDistribution") {
            const std::string *v = t.attr("value");
            if (!v) return false;
            const std::string *rc = t.attr("recordCount"), *pr = t.attr("probability"), *cf = t.attr("confidence");
            double c = 0.0, p = kNaN, q = kNaN;
            if ((rc && !numeric_attr(*rc, c)) || (pr && !numeric_attr(*pr, p)) || (cf && !numeric_attr(*cf, q)))
                return false;
            tr.dist_node.push_back(cur);
            tr.dist_value_s.push_back(str.intern(*v));
            tr.dist_count.push_back(c);
            tr.dist_prob.push_back(p);
            tr.dist_conf.push_back(q);
            if (!sc.skip_element(t)) return false;
        } else if (nm == "Extension" || nm == "Partition") {
            if (!sc.skip_element(t)) return false;  // ignored by the DOM parser too
        } else {
            return false;  // embedded models, unknown elements: the DOM parser decides
        }
    }
    if (sc.depth() != root_depth - 1) return false;
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

// The XML declaration, if any, must say version 1.0 and (if it names one) the UTF-8 encoding.
bool acceptable_prolog(const char *b, size_t n) {
    size_t i = 0;
    if (n >= 3 && static_cast<unsigned char>(b[0]) == 0xEF && static_cast<unsigned char>(b[1]) == 0xBB &&
        static_cast<unsigned char>(b[2]) == 0xBF)
        i = 3;
    if (n - i < 6 || std::memcmp(b + i, "<?xml", 5) != 0 || !is_ws(b[i + 5])) return true;
    const char *end = static_cast<const char *>(memmem(b + i, n - i, "?>", 2));
    if (!end) return false;
    std::string decl(b + i, static_cast<size_t>(end - (b + i)));
    for (auto &c : decl) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    auto value_of = [&](const char *key, std::string &out) {
        size_t p = decl.find(key);
        if (p == std::string::npos) return false;
        p += std::strlen(key);
        while (p < decl.size() && (is_ws(decl[p]) || decl[p] == '=')) ++p;
        if (p >= decl.size() || (decl[p] != '"' && decl[p] != '\'')) return false;
        const char q = decl[p++];
        const size_t e = decl.find(q, p);
        if (e == std::string::npos) return false;
        out = decl.substr(p, e - p);
        return true;
    };
    std::string v;
    if (!value_of("version", v) || v != "1.0") return false;
    if (decl.find("encoding") != std::string::npos) {
        if (!value_of("encoding", v) || (v != "utf-8" && v != "utf8")) return false;
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

// The whole scan, free of Python objects (runs with the GIL released).
bool scan(const char *buf, size_t n, std::vector<Tree> &trees, Strings &str, std::string &skel) {
    if (!acceptable_prolog(buf, n)) return false;
    if (!valid_utf8_xml_chars(reinterpret_cast<const unsigned char *>(buf), n)) return false;
    skel.reserve(1 << 16);
    Scanner sc(buf, n);
    size_t copied = 0;  // source bytes up to here are in the skeleton
    Tag t;
    // per open element: is it a TreeModel still awaiting its root Node
    std::vector<bool> model_stack;
    while (sc.next_tag(t)) {
        if (t.end) {
            if (model_stack.empty()) return false;
            model_stack.pop_back();
            continue;
        }
        if (t.name == "Node" && !model_stack.empty() && model_stack.back()) {
            // the root Node of the innermost open TreeModel (the DOM parser's _child(el, "Node"))
            if (t.has_ns_decl || t.has_prefixed_attr) return false;
            trees.emplace_back();
            sc.enter_body();
            const bool ok = parse_tree(sc, t, trees.back(), str);
            sc.leave_body();
            if (!ok) return false;
            skel.append(buf + copied, t.start - copied);
            skel.append("<Node fjaFlat=\"" + std::to_string(trees.size() - 1) + "\"/>");
            copied = sc.pos();
            model_stack.back() = false;
            continue;
        }
        if (!t.self_close) model_stack.push_back(t.name == "TreeModel");
    }
    if (sc.error() || sc.depth() != 0) return false;
    skel.append(buf + copied, n - copied);
    return true;
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
    bool ok;
    Py_BEGIN_ALLOW_THREADS;
    ok = scan(buf, n, trees, str, skel);
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
        // valid UTF-8 (checked above), so strict decoding cannot fail
        PyObject *s = PyUnicode_DecodeUTF8(str.values[i].data(), static_cast<Py_ssize_t>(str.values[i].size()),
                                           "strict");
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
