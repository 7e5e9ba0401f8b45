// Host sanitizer harness for the native ingest ("-fsanitize=address for the C++ host
// extension"). Built by tests/test_native_ingest.py with
//   g++ -std=c++17 -g -O1 -fsanitize=address,undefined -fno-omit-frame-pointer -pthread
// and run as a plain executable (no Python in the process, so ASan needs no preload). Exercises the
// edge cases that touch buffer boundaries: no trailing newline, CRLF, blank lines, short / long rows,
// overlong tokens, missing tokens, vocabulary lookups, max_rows caps and multi-threaded splits.
#include "ingest.cpp"

#include <cstdio>
#include <cstdlib>
#include <memory>

static int failures = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

struct Harness {
  std::vector<int> target{0, 1, -1, 2};  // input col 2 is skipped
  std::vector<int> kind{0, 0, 1};        // output col 2 is categorical
  std::string missing = std::string("NA") + '\0' + "?" + '\0';
  void* vocab = ingest_vocab_new(3);
  Harness() {
    ingest_vocab_add(vocab, 2, "red", 3, 0.f);
    ingest_vocab_add(vocab, 2, "green", 5, 1.f);
  }
  ~Harness() { ingest_vocab_free(vocab); }
  long long run(const std::string& text, std::vector<float>& out, size_t max_rows, int threads, size_t* consumed,
                size_t* bad) {
    // exact-size heap copy: ASan flags any read past the caller's buffer
    std::unique_ptr<char[]> buf(new char[text.size() ? text.size() : 1]);
    std::memcpy(buf.get(), text.data(), text.size());
    return ingest_parse(buf.get(), text.size(), ',', 4, target.data(), 3, kind.data(), missing.data(), 2, vocab,
                        out.data(), max_rows, threads, consumed, bad);
  }
};

int main() {
  Harness h;
  size_t consumed = 0, bad = 0;
  {  // basic rows, CRLF, blank lines, missing tokens, unknown category, trailing partial line
    std::string t = "1.5,2,x,red\r\n\nNA,?,y,green\n3,4e2,z,blue\n5,6,w,re";
    std::vector<float> out(4 * 3, -7.f);
    long long n = h.run(t, out, 4, 1, &consumed, &bad);
    CHECK(n == 3);
    CHECK(consumed == t.rfind('\n') + 1);
    CHECK(out[0] == 1.5f && out[1] == 2.f && out[2] == 0.f);
    CHECK(std::isnan(out[3]) && std::isnan(out[4]) && out[5] == 1.f);
    CHECK(out[6] == 3.f && out[7] == 400.f && out[8] == -1.f);
    CHECK(out[9] == -7.f);  // untouched beyond the returned rows
  }
  {  // short and long rows, garbage numerics, overlong token
    std::string longtok(5000, '9');
    std::string t = "1\n1,2,3,green,extra,cols\nabc,1e999999," + longtok + ",red\n";
    std::vector<float> out(3 * 3, 0.f);
    long long n = h.run(t, out, 3, 1, &consumed, &bad);
    CHECK(n == 3);
    CHECK(out[0] == 1.f && std::isnan(out[1]) && std::isnan(out[2]));
    CHECK(out[3] == 1.f && out[4] == 2.f && out[5] == 1.f);
    CHECK(std::isnan(out[6]));
    CHECK(bad >= 1);
  }
  {  // empty input / no complete line
    std::vector<float> out(3, 0.f);
    CHECK(h.run("", out, 1, 4, &consumed, &bad) == 0 && consumed == 0);
    CHECK(h.run("1,2,3,red", out, 1, 4, &consumed, &bad) == 0 && consumed == 0);
  }
  {  // multi-threaded split (> 64 KiB per thread) with a max_rows cap inside a later thread's range
    std::string t;
    const int rows = 40000;
    for (int i = 0; i < rows; ++i) t += std::to_string(i) + "," + std::to_string(i * 0.5) + ",q," + (i % 2 ? "red\n" : "green\n");
    for (size_t cap : {(size_t)rows, (size_t)rows - 1234, (size_t)17}) {
      std::vector<float> out(cap * 3, 0.f);
      long long n = h.run(t, out, cap, 8, &consumed, &bad);
      CHECK(n == (long long)cap);
      CHECK(bad == 0);
      bool ok = true;
      for (size_t r = 0; r < cap; ++r)
        ok = ok && out[r * 3] == (float)r && out[r * 3 + 2] == (r % 2 ? 0.f : 1.f);
      CHECK(ok);
      if (cap == (size_t)rows) CHECK(consumed == t.size());
      else CHECK(consumed < t.size() && t[consumed - 1] == '\n');
    }
  }
  {  // bad column maps are rejected before any write
    std::vector<int> tgt{0, 5};
    std::vector<float> out(3, 0.f);
    CHECK(ingest_parse("1,2\n", 4, ',', 2, tgt.data(), 3, h.kind.data(), h.missing.data(), 2, h.vocab, out.data(), 1,
                       1, &consumed, &bad) == -2);
    CHECK(ingest_parse("1,2\n", 4, ',', 2, h.target.data(), 3, h.kind.data(), h.missing.data(), 2, nullptr, out.data(),
                       1, 1, &consumed, &bad) == -3);
  }
  std::printf("ingest selftest: %s (%d failures)\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
