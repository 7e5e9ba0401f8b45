// Native record ingest: delimited text records -> the engine's [rows, fields] fp32 matrix.
//
// The reference receives records as JVM objects one at a time (Flink sources, `S/package.scala:76-79`);
// at MI355X rates (hundreds of millions of records/s per node) host ingest, not the GPU, is the
// bound, so text parsing runs here in C++ on all cores, writing straight into the
// (pinned) host buffer the H2D stage ships:
//  * pass 1 splits the buffer into per-thread line ranges (memchr for '\n'), pass 2 parses every
//    range into its row slice in place — no intermediate objects, no per-record allocation;
//  * numeric fields are parsed in ONE pass where they are plain decimals (SWAR digit runs, 8 bytes
//    per step, no per-digit branch; no token split or trim), then a Clinger fast path for plain decimals (<= 19 significant digits, exponent
//    within +-22: the decimal is exact in double, so one double operation rounds it correctly; the
//    double -> fp32 rounding is exact unless that double sits on an fp32 midpoint, which falls
//    back), otherwise std::from_chars (locale-free, exact round-to-nearest fp32); empty fields and
//    the configured missing tokens become NaN (PMML missing); unparsable numerics become NaN and are
//    counted;
//  * categorical (string) fields: per-column dictionaries map the token to the PMML vocabulary code
//    (`pmml/fields.py::FieldSchema`), unknown tokens to -1 (an invalid code: the kernels' FieldPrep
//    code-range check applies invalidValueTreatment);
//  * a column map selects / reorders input columns into the model's active-field order;
//  * the parse passes run on a persistent worker pool (threads are created once, on first use,
//    and parked on a condition variable between calls — no thread creation per batch).
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#define INGEST_API extern "C" __attribute__((visibility("default")))

namespace {

struct Vocab {
  std::vector<std::unordered_map<std::string, float>> cols;
};

struct Spec {
  char delim = ',';
  int n_in = 0;                      // columns per input line
  std::vector<int> target;           // input column -> output column (-1: skip)
  std::vector<int> kind;             // output column: 0 numeric, 1 categorical
  std::vector<std::string> missing;  // tokens that mean "missing"
  const Vocab* vocab = nullptr;
  bool fast = true;                  // single-pass numeric fields (off when a missing token is numeric)
};

inline std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t' || s.front() == '"')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r' || s.back() == '"')) s.remove_suffix(1);
  return s;
}

inline bool is_missing(const Spec& sp, std::string_view tok) {
  if (tok.empty()) return true;
  for (const auto& m : sp.missing)
    if (tok == m) return true;
  return false;
}

constexpr double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Decimal w * 10^exp10 -> fp32 when exact in one double operation (Clinger: w < 2^53, |exp10| <=
// 22) and the double does not sit on an fp32 rounding midpoint; false -> the caller falls back to
// std::from_chars.
inline bool finish_decimal(uint64_t w, int exp10, bool neg, float* out) {
  if (w > (uint64_t{1} << 53) || exp10 < -22 || exp10 > 22) return false;
  double d = static_cast<double>(w);
  d = exp10 < 0 ? d / kPow10[-exp10] : d * kPow10[exp10];
  // double -> float is exact unless d lies on a float rounding midpoint (then the decimal may be
  // on either side of it: let from_chars decide)
  uint64_t bits;
  std::memcpy(&bits, &d, 8);
  const int be = static_cast<int>((bits >> 52) & 0x7FF);
  if (be != 0 && be >= 1023 - 126) {  // normal float range: 29 dropped mantissa bits
    if ((bits & ((uint64_t{1} << 29) - 1)) == (uint64_t{1} << 28)) return false;
  } else if (d != 0.0) {
    return false;  // subnormal / underflow region: from_chars
  }
  const float f = static_cast<float>(d);
  *out = neg ? -f : f;
  return true;
}

// [+-]digits[.digits][(e|E)[+-]digits] starting at s; scanning stops at the first other byte.
// Returns the end of the number (s when there is none) and the decimal's parts; *ok = false when
// the number has more than 19 significant digits or a malformed exponent.
inline const char* scan_decimal(const char* s, const char* e, uint64_t* w_out, int* exp_out, bool* neg_out,
                                bool* ok) {
  const char* start = s;
  bool neg = false;
  if (s < e && (*s == '-' || *s == '+')) neg = *s++ == '-';
  uint64_t w = 0;
  int digits = 0, exp10 = 0;
  bool any = false;
  while (s < e && static_cast<unsigned>(*s - '0') < 10u) {
    if (w != 0 || *s != '0') ++digits;
    w = w * 10u + static_cast<unsigned>(*s - '0');
    ++s;
    any = true;
  }
  if (s < e && *s == '.') {
    ++s;
    while (s < e && static_cast<unsigned>(*s - '0') < 10u) {
      if (w != 0 || *s != '0') ++digits;
      w = w * 10u + static_cast<unsigned>(*s - '0');
      --exp10;
      ++s;
      any = true;
    }
  }
  *ok = any && digits <= 19;
  if (!any) return start;
  if (s < e && (*s == 'e' || *s == 'E')) {
    ++s;
    bool eneg = false;
    if (s < e && (*s == '-' || *s == '+')) eneg = *s++ == '-';
    int ev = 0, ed = 0;
    while (s < e && static_cast<unsigned>(*s - '0') < 10u && ed < 6) {
      ev = ev * 10 + (*s - '0');
      ++s;
      ++ed;
    }
    if (ed == 0) *ok = false;
    exp10 += eneg ? -ev : ev;
  }
  *w_out = w;
  *exp_out = exp10;
  *neg_out = neg;
  return s;
}

// SWAR digit runs (8 bytes per step, no per-digit branch). n_digits8: how many of the 8 bytes at
// p, from the first, are ASCII digits (x = byte ^ '0' is 0..9 exactly for digits; x + 0x76 sets bit
// 7 for x >= 10 — a carry out of a non-digit byte only reaches bytes after the first non-digit).
inline int n_digits8(uint64_t v) {
  const uint64_t x = v ^ 0x3030303030303030ULL;
  const uint64_t nd = ((x + 0x7676767676767676ULL) | x) & 0x8080808080808080ULL;
  return nd ? (__builtin_ctzll(nd) >> 3) : 8;
}

// Value of the first n (1..8) digit bytes of v (first character in the lowest byte).
inline uint64_t digits8_value(uint64_t v, int n) {
  uint64_t x = (v ^ 0x3030303030303030ULL) << (8 * (8 - n));  // keep n digits, zeros before them
  x = (x * 10) + (x >> 8);                                     // pairs
  x = (((x & 0x000000FF000000FFULL) * (100 + (1000000ULL << 32))) +
       (((x >> 16) & 0x000000FF000000FFULL) * (1 + (10000ULL << 32)))) >> 32;
  return x;
}

constexpr uint64_t kPow10u[9] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000, 100000000};

// scan_decimal with SWAR digit runs; needs 16 readable bytes at s (bend: end of the buffer). The
// digit count guard is on all digits (leading zeros included): > 19 -> *ok = false (the caller's
// scalar path decides).
inline const char* scan_decimal_swar(const char* s, const char* e, const char* bend, uint64_t* w_out,
                                     int* exp_out, bool* neg_out, bool* ok) {
  const char* start = s;
  bool neg = false;
  if (s < e && (*s == '-' || *s == '+')) neg = *s++ == '-';
  uint64_t w = 0;
  int total = 0, exp10 = 0;
  for (;;) {  // integer digits
    if (s + 8 > bend) { *ok = false; return start; }
    uint64_t v;
    std::memcpy(&v, s, 8);
    const int n = n_digits8(v);
    if (n == 0) break;
    w = w * kPow10u[n] + digits8_value(v, n);
    s += n;
    total += n;
    if (n < 8 || total > 19) break;
  }
  if (s < e && *s == '.') {
    ++s;
    for (;;) {
      if (s + 8 > bend) { *ok = false; return start; }
      uint64_t v;
      std::memcpy(&v, s, 8);
      const int n = n_digits8(v);
      if (n == 0) break;
      w = w * kPow10u[n] + digits8_value(v, n);
      s += n;
      total += n;
      exp10 -= n;
      if (n < 8 || total > 19) break;
    }
  }
  if (s > e) { *ok = false; return start; }  // a digit run may not cross the field's line end
  *ok = total > 0 && total <= 19;
  if (total == 0) return start;
  if (s < e && (*s == 'e' || *s == 'E')) {
    ++s;
    bool eneg = false;
    if (s < e && (*s == '-' || *s == '+')) eneg = *s++ == '-';
    int ev = 0, ed = 0;
    while (s < e && static_cast<unsigned>(*s - '0') < 10u && ed < 6) {
      ev = ev * 10 + (*s - '0');
      ++s;
      ++ed;
    }
    if (ed == 0) *ok = false;
    exp10 += eneg ? -ev : ev;
  }
  *w_out = w;
  *exp_out = exp10;
  *neg_out = neg;
  return s;
}

// Clinger fast path over a whole (trimmed) token. Returns false when the token is not of that
// form or is outside the exact range (the caller then uses std::from_chars).
inline bool fast_decimal(const char* s, const char* e, float* out) {
  uint64_t w = 0;
  int exp10 = 0;
  bool neg = false, ok = false;
  const char* q = scan_decimal(s, e, &w, &exp10, &neg, &ok);
  if (!ok || q != e) return false;
  return finish_decimal(w, exp10, neg, out);
}

// Single-pass numeric field at p: the number must run up to the delimiter / end of line (an
// optional '\r' before the end of the line). On success *next = the delimiter or line end and the
// fp32 value is written; otherwise the caller takes the general path (token split, trim, missing
// tokens, from_chars) for this field.
inline bool fast_field(const char* p, const char* le, const char* bend, char delim, float* out, const char** next) {
  uint64_t w = 0;
  int exp10 = 0;
  bool neg = false, ok = false;
  const char* q = scan_decimal_swar(p, le, bend, &w, &exp10, &neg, &ok);
  if (!ok) q = scan_decimal(p, le, &w, &exp10, &neg, &ok);
  if (!ok) return false;
  if (q < le && *q != delim && !(*q == '\r' && q + 1 == le)) return false;
  if (!finish_decimal(w, exp10, neg, out)) return false;
  *next = q;
  return true;
}

// Parse lines [b, e) into rows out[0..]; returns rows written; bad numeric tokens counted.
size_t parse_range(const Spec& sp, const char* b, const char* e, const char* bend, float* out, int n_out,
                   size_t max_rows, size_t* bad) {
  size_t r = 0;
  const float nan = std::nanf("");
  while (b < e && r < max_rows) {
    const char* nl = static_cast<const char*>(memchr(b, '\n', (size_t)(e - b)));
    const char* le = nl ? nl : e;
    if (le > b && !(le - b == 1 && *b == '\r')) {
      float* row = out + r * (size_t)n_out;
      for (int c = 0; c < n_out; ++c) row[c] = nan;
      const char* p = b;
      for (int c = 0; c < sp.n_in && p <= le; ++c) {
        const int oc = sp.target[c];
        if (sp.fast && oc >= 0 && sp.kind[oc] == 0) {
          const char* nx;
          if (fast_field(p, le, bend, sp.delim, &row[oc], &nx)) {  // one pass: no token split / trim
            if (nx >= le || *nx != sp.delim) break;
            p = nx + 1;
            continue;
          }
        }
        const char* q = static_cast<const char*>(memchr(p, sp.delim, (size_t)(le - p)));
        const char* te = q ? q : le;
        if (oc >= 0) {
          std::string_view tok = trim(std::string_view(p, (size_t)(te - p)));
          if (!is_missing(sp, tok)) {
            if (sp.kind[oc] == 0) {
              float v;
              const char* s = tok.data();
              const char* te2 = tok.data() + tok.size();
              if (fast_decimal(s, te2, &v)) {
                row[oc] = v;
              } else {
                if (*s == '+') ++s;
                auto res = std::from_chars(s, te2, v);
                if (res.ec == std::errc() && res.ptr == te2) {
                  row[oc] = v;
                } else if (tok == "inf" || tok == "Infinity" || tok == "+inf") {
                  row[oc] = INFINITY;
                } else if (tok == "-inf" || tok == "-Infinity") {
                  row[oc] = -INFINITY;
                } else {
                  ++*bad;
                }
              }
            } else {
              const auto& m = sp.vocab->cols[oc];
              auto it = m.find(std::string(tok));
              row[oc] = it == m.end() ? -1.0f : it->second;
            }
          }
        }
        if (!q) break;
        p = q + 1;
      }
      ++r;
    }
    b = nl ? nl + 1 : e;
  }
  return r;
}

// Persistent fork-join pool: run(T, fn) executes fn(0..T-1) across the workers and the caller and
// returns when all are done. One job at a time (callers serialise on job_mu_).
class Pool {
 public:
  static Pool& instance() {
    static Pool p;
    return p;
  }

  void run(int T, const std::function<void(int)>& fn) {
    if (T <= 1) {
      if (T == 1) fn(0);
      return;
    }
    std::lock_guard<std::mutex> job_lock(job_mu_);
    grow(T - 1);
    uint64_t g;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_tasks_ = T;
      next_ = 0;
      remaining_ = T;
      g = ++gen_;
    }
    cv_.notify_all();
    work(g);  // the caller takes tasks too
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return remaining_ == 0; });
    fn_ = nullptr;
  }

  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  void grow(int n) {
    while ((int)workers_.size() < std::min(n, 63)) workers_.emplace_back([this] { loop(); });
  }

  // Claim tasks of job generation g under the lock: a worker that wakes late can never run a
  // finished job's function (the job cannot complete while one of its tasks is claimed).
  void work(uint64_t g) {
    for (;;) {
      const std::function<void(int)>* fn;
      int t;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (gen_ != g || fn_ == nullptr || next_ >= n_tasks_) return;
        t = next_++;
        fn = fn_;
      }
      (*fn)(t);
      std::lock_guard<std::mutex> lk(mu_);
      if (--remaining_ == 0) done_cv_.notify_all();
    }
  }

  void loop() {
    uint64_t seen;
    {
      std::lock_guard<std::mutex> lk(mu_);
      seen = gen_;
    }
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work(seen);
    }
  }

  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_tasks_ = 0, remaining_ = 0, next_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

size_t count_lines(const char* b, const char* e) {
  size_t n = 0;
  while (b < e) {
    const char* nl = static_cast<const char*>(memchr(b, '\n', (size_t)(e - b)));
    const char* le = nl ? nl : e;
    if (le > b && !(le - b == 1 && *b == '\r')) ++n;
    b = nl ? nl + 1 : e;
  }
  return n;
}

}  // namespace

INGEST_API void* ingest_vocab_new(int n_cols) {
  auto* v = new Vocab();
  v->cols.resize((size_t)std::max(0, n_cols));
  return v;
}

INGEST_API void ingest_vocab_free(void* h) { delete static_cast<Vocab*>(h); }

INGEST_API int ingest_vocab_add(void* h, int col, const char* s, int len, float code) {
  auto* v = static_cast<Vocab*>(h);
  if (col < 0 || (size_t)col >= v->cols.size()) return -1;
  v->cols[(size_t)col][std::string(s, (size_t)len)] = code;
  return 0;
}

// Parse complete lines of `buf` (a trailing partial line is left unconsumed).
//   target[n_in]: output column per input column (-1 skip); kind[n_out]: 0 numeric, 1 categorical;
//   missing: '\0'-separated list of missing tokens (n_missing entries).
// Returns rows written (<= max_rows); *consumed = bytes of buf covered; *bad = unparsable numerics.
INGEST_API long long ingest_parse(const char* buf, size_t len, char delim, int n_in, const int* target, int n_out,
                                  const int* kind, const char* missing, int n_missing, void* vocab, float* out,
                                  size_t max_rows, int n_threads, size_t* consumed, size_t* bad) {
  Spec sp;
  sp.delim = delim;
  sp.n_in = n_in;
  sp.target.assign(target, target + n_in);
  sp.kind.assign(kind, kind + n_out);
  for (int i = 0, off = 0; i < n_missing; ++i) {
    sp.missing.emplace_back(missing + off);
    off += (int)sp.missing.back().size() + 1;
  }
  sp.vocab = static_cast<const Vocab*>(vocab);
  for (const auto& m : sp.missing) {  // "-999" as a missing token must not take the number path
    uint64_t w;
    int ex;
    bool ng, ok;
    const std::string_view t = trim(m);
    if (!t.empty() && scan_decimal(t.data(), t.data() + t.size(), &w, &ex, &ng, &ok) != t.data()) sp.fast = false;
  }
  for (int c = 0; c < n_in; ++c)
    if (sp.target[c] >= n_out) return -2;
  for (int c = 0; c < n_out; ++c)
    if (sp.kind[c] == 1 && (!sp.vocab || (size_t)c >= sp.vocab->cols.size())) return -3;
  // complete lines only
  const char* end = buf + len;
  while (end > buf && end[-1] != '\n') --end;
  *consumed = (size_t)(end - buf);
  *bad = 0;
  if (end == buf) return 0;
  int T = std::max(1, std::min(n_threads, 64));
  const size_t total = (size_t)(end - buf);
  if (total < (size_t)T * 65536) T = std::max<int>(1, (int)(total / 65536));
  std::vector<const char*> cut((size_t)T + 1);
  cut[0] = buf;
  cut[(size_t)T] = end;
  for (int t = 1; t < T; ++t) {
    const char* p = buf + total * (size_t)t / (size_t)T;
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    cut[(size_t)t] = nl ? nl + 1 : end;
    if (cut[(size_t)t] < cut[(size_t)t - 1]) cut[(size_t)t] = cut[(size_t)t - 1];
  }
  std::vector<size_t> lines((size_t)T, 0), start((size_t)T + 1, 0), bads((size_t)T, 0);
  Pool& pool = Pool::instance();
  pool.run(T, [&](int t) { lines[(size_t)t] = count_lines(cut[(size_t)t], cut[(size_t)t + 1]); });
  for (int t = 0; t < T; ++t) start[(size_t)t + 1] = start[(size_t)t] + lines[(size_t)t];
  const size_t rows = std::min(start[(size_t)T], max_rows);
  pool.run(T, [&](int t) {
    if (start[(size_t)t] >= rows) return;
    const size_t cap = std::min(lines[(size_t)t], rows - start[(size_t)t]);
    parse_range(sp, cut[(size_t)t], cut[(size_t)t + 1], buf + len, out + start[(size_t)t] * (size_t)n_out, n_out,
                cap, &bads[(size_t)t]);
  });
  if (rows < start[(size_t)T]) {
    // stopped at max_rows: report the bytes actually covered (lines before the cap)
    size_t seen = 0;
    const char* p = buf;
    while (p < end && seen < rows) {
      const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
      const char* le = nl ? nl : end;
      if (le > p && !(le - p == 1 && *p == '\r')) ++seen;
      p = nl ? nl + 1 : end;
    }
    *consumed = (size_t)(p - buf);
  }
  for (size_t b : bads) *bad += b;
  return (long long)rows;
}
