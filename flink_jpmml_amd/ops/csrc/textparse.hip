// Delimited text records parsed on the GPU: raw CSV bytes in HBM -> the engine's [rows, F] fp32
// matrix (the text ingest of the reference's socket / file jobs, `E/CheckpointEvaluate.scala:80-82`).
//
// Host parsing tops out near 7 GB/s on 16 cores (`native/csrc/ingest.cpp`, ~20 M records/s of
// 32-field CSV) — 20x below what one MI355X scores. Here the host only reads file bytes into
// pinned memory; they cross PCIe once and the GPU finds the records and parses the fields:
//
//   row_start_count / row_start_write  (3-phase compaction, 4 KiB tiles): a row starts at byte s
//     when s follows a '\n' (or is 0) and the line is not empty ("\n" or "\r\n" lines carry no
//     record, as on the host). Phase 1 counts per tile, phase 2 (row_start_scan, one workgroup)
//     turns the counts into tile offsets, phase 3 writes every row start in order.
//   parse_rows: one lane per record walks its line (~350 bytes for 32 fields): split at the
//     delimiter, trim ' ' '\t' '"' (and a final '\r'), empty / configured missing tokens -> NaN,
//     plain decimals (<= 19 significant digits, |exp10| <= 22) -> fp32 exactly as
//     ingest.cpp::finish_decimal does (one correctly rounded double operation; the double -> fp32
//     step is exact unless the double sits on an fp32 midpoint). Anything else (midpoints,
//     subnormals, inf / nan spellings, > 19 digits, junk) flags the record: the host re-parses
//     those few lines with the exact host parser and patches the rows, so results are
//     bit-identical to ingest.cpp for every input.

#include <algorithm>

#include "common.h"

namespace {

constexpr int TP_TB = 256;
constexpr int TP_TILE = TP_TB * 16;  // bytes per workgroup tile (16 per lane)
constexpr int TP_MAX_MISSING = 8;
constexpr int TP_MISSING_LEN = 16;

struct TextParseArgs {
  const uint8_t* buf;     // chunk bytes (ends with '\n')
  long long n_bytes;
  const long long* starts;  // row starts
  int n_rows;
  int n_cols;             // columns per input line
  const int* colmap;      // input column -> output column (-1: skip); n_cols entries
  int F;                  // output columns
  char delim;
  int n_missing;
  const char* missing;    // n_missing x TP_MISSING_LEN, NUL-padded
  float* X;               // [n_rows, F]
  int* flagged;           // [max_flagged] row indices needing the host parser
  int max_flagged;
  int* n_flagged;         // device counter
};

__device__ __forceinline__ bool is_row_start(const uint8_t* b, long long n, long long s) {
  if (s >= n) return false;
  if (s > 0 && b[s - 1] != '\n') return false;
  const uint8_t c = b[s];
  if (c == '\n') return false;
  if (c == '\r' && s + 1 < n && b[s + 1] == '\n') return false;
  return true;
}

// per-lane bitmask of row starts among its 16 bytes
__device__ __forceinline__ unsigned lane_starts(const uint8_t* b, long long n, long long s0) {
  unsigned m = 0;
  uint8_t v[18];
  // bytes s0-1 .. s0+16 (neighbours for the boundary tests)
#pragma unroll
  for (int j = 0; j < 18; ++j) {
    const long long p = s0 - 1 + j;
    v[j] = (p >= 0 && p < n) ? b[p] : (uint8_t)'\n';
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const long long s = s0 + j;
    const bool prev_nl = (s == 0) || v[j] == '\n';
    const uint8_t c = v[j + 1];
    const bool empty = c == '\n' || (c == '\r' && v[j + 2] == '\n');
    if (s < n && prev_nl && !empty) m |= 1u << j;
  }
  return m;
}

__global__ __launch_bounds__(TP_TB) void row_start_count(const uint8_t* __restrict__ b, long long n,
                                                         int* __restrict__ tile_counts) {
  __shared__ int wsum[TP_TB / 64];
  const long long s0 = (long long)blockIdx.x * TP_TILE + 16 * threadIdx.x;
  int c = __popc(lane_starts(b, n, s0));
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < TP_TB / 64; ++w) t += wsum[w];
    tile_counts[blockIdx.x] = t;
  }
}

// exclusive scan of tile_counts (in place) + the total in tile_counts[n_tiles]; one workgroup
__global__ __launch_bounds__(1024) void row_start_scan(int* __restrict__ tile_counts, int n_tiles) {
  __shared__ int part[1024];
  const int per = (n_tiles + 1023) / 1024;
  const int a = threadIdx.x * per, e = min(n_tiles, a + per);
  int s = 0;
  for (int i = a; i < e; ++i) s += tile_counts[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int i = a; i < e; ++i) {
    const int c = tile_counts[i];
    tile_counts[i] = run;
    run += c;
  }
  if (threadIdx.x == 1023) tile_counts[n_tiles] = part[1023];
}

__global__ __launch_bounds__(TP_TB) void row_start_write(const uint8_t* __restrict__ b, long long n,
                                                         const int* __restrict__ tile_offsets,
                                                         long long* __restrict__ starts) {
  __shared__ int wsum[TP_TB / 64];
  const long long s0 = (long long)blockIdx.x * TP_TILE + 16 * threadIdx.x;
  const unsigned m = lane_starts(b, n, s0);
  const int c = __popc(m);
  // exclusive prefix of c within the wave, then across the workgroup's waves
  int incl = c;
  const int lane = threadIdx.x & 63;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[threadIdx.x >> 6] = incl;
  __syncthreads();
  int base = tile_offsets[blockIdx.x];
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) base += wsum[w];
  int k = base + incl - c;
  unsigned mm = m;
  while (mm) {
    const int j = __ffs(mm) - 1;
    mm &= mm - 1;
    starts[k++] = s0 + j;
  }
}

__device__ __forceinline__ bool is_space(uint8_t c) { return c == ' ' || c == '\t' || c == '"'; }

constexpr double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                             1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// The token [p, e) (trimmed) as ingest.cpp's fast path: true + *out on success.
__device__ bool fast_token(const uint8_t* p, const uint8_t* e, float* out) {
  const uint8_t* s = p;
  bool neg = false;
  if (s < e && (*s == '-' || *s == '+')) neg = *s++ == '-';
  unsigned long long w = 0;
  int digits = 0, exp10 = 0;
  bool any = false;
  while (s < e && (unsigned)(*s - '0') < 10u) {
    if (w != 0 || *s != '0') ++digits;
    w = w * 10u + (unsigned)(*s - '0');
    ++s;
    any = true;
  }
  if (s < e && *s == '.') {
    ++s;
    while (s < e && (unsigned)(*s - '0') < 10u) {
      if (w != 0 || *s != '0') ++digits;
      w = w * 10u + (unsigned)(*s - '0');
      --exp10;
      ++s;
      any = true;
    }
  }
  if (!any || digits > 19) return false;
  if (s < e && (*s == 'e' || *s == 'E')) {
    ++s;
    bool eneg = false;
    if (s < e && (*s == '-' || *s == '+')) eneg = *s++ == '-';
    int ev = 0, ed = 0;
    while (s < e && (unsigned)(*s - '0') < 10u && ed < 6) {
      ev = ev * 10 + (*s - '0');
      ++s;
      ++ed;
    }
    if (ed == 0) return false;
    exp10 += eneg ? -ev : ev;
  }
  if (s != e) return false;
  // finish_decimal
  if (w > (1ull << 53) || exp10 < -22 || exp10 > 22) return false;
  double d = (double)w;
  d = exp10 < 0 ? d / kP10[-exp10] : d * kP10[exp10];
  const unsigned long long bits = __double_as_longlong(d);
  const int be = (int)((bits >> 52) & 0x7FF);
  if (be != 0 && be >= 1023 - 126) {
    if ((bits & ((1ull << 29) - 1)) == (1ull << 28)) return false;
  } else if (d != 0.0) {
    return false;
  }
  const float f = (float)d;
  *out = neg ? -f : f;
  return true;
}

// One record: the line starting at p (it ends at the next '\n' before bend). Field values land in
// out[oc] (out pre-filled with NaN); returns true when a token needs the host parser. colmap and
// missing may live in LDS or global memory, as may the line itself.
__device__ __forceinline__ bool parse_record(const uint8_t* p, const uint8_t* bend, int n_cols, const int* colmap,
                                             char delim, int n_missing, const char* missing, float* out) {
  // line end: the next '\n' (the chunk ends with one)
  const uint8_t* le = p;
  while (le < bend && *le != '\n') ++le;
  bool bad = false;
  for (int c = 0; c < n_cols && p <= le; ++c) {
    const uint8_t* te = p;
    while (te < le && *te != (uint8_t)delim) ++te;
    const int oc = colmap[c];
    if (oc >= 0) {
      const uint8_t* s = p;
      const uint8_t* e = te;
      while (s < e && is_space(*s)) ++s;
      while (e > s && (is_space(e[-1]) || e[-1] == '\r')) --e;
      bool miss = s == e;
      for (int m = 0; !miss && m < n_missing; ++m) {
        const char* tok = missing + m * TP_MISSING_LEN;
        int k = 0;
        while (k < TP_MISSING_LEN && tok[k] && s + k < e && s[k] == (uint8_t)tok[k]) ++k;
        miss = (k == TP_MISSING_LEN || !tok[k]) && s + k == e;
      }
      if (!miss) {
        float v;
        if (fast_token(s, e, &v)) out[oc] = v;
        else bad = true;
      }
    }
    if (te >= le) break;
    p = te + 1;
  }
  return bad;
}

__device__ __forceinline__ void flag_row(const TextParseArgs& a, int r) {
  const int k = atomicAdd(a.n_flagged, 1);
  if (k < a.max_flagged) a.flagged[k] = r;
}

// Global-memory variant: one lane per record reading its line byte by byte from HBM (every load
// instruction touches 64 different lines). Kept for workgroups whose byte span exceeds the LDS
// staging capacity of parse_rows_lds (very long lines).
__global__ __launch_bounds__(TP_TB) void parse_rows(TextParseArgs a) {
  const int r = blockIdx.x * TP_TB + threadIdx.x;
  if (r >= a.n_rows) return;
  float* row = a.X + (size_t)r * a.F;
  const float nan = __builtin_nanf("");
  for (int c = 0; c < a.F; ++c) row[c] = nan;
  if (parse_record(a.buf + a.starts[r], a.buf + a.n_bytes, a.n_cols, a.colmap, a.delim, a.n_missing, a.missing, row))
    flag_row(a, r);
}

// LDS-staged variant. The records of a workgroup are one contiguous byte span of the chunk
// [starts[r0], starts[r0 + PR_TB]): the workgroup copies it into LDS with coalesced 16-byte loads,
// every lane then parses its record out of LDS (byte reads at LDS latency, no per-byte TA
// traffic), and the [PR_TB, F] result tile — contiguous in X — leaves with coalesced stores.
// Output rows are padded to F + 1 floats in LDS so the per-lane column writes do not collide in
// one bank. A span beyond `cap` bytes (lines much longer than the chunk's average) takes the
// global-memory path for that workgroup.
constexpr int PR_TB = 128;
constexpr int PR_MAX_COLS = 256;

__global__ __launch_bounds__(PR_TB) void parse_rows_lds(TextParseArgs a, int cap) {
  extern __shared__ __align__(16) uint8_t lds[];
  __shared__ int colmap_l[PR_MAX_COLS];
  __shared__ char missing_l[TP_MAX_MISSING * TP_MISSING_LEN];
  const int tid = threadIdx.x;
  const int F = a.F, FP = a.F + 1;
  float* out = reinterpret_cast<float*>(lds);
  uint8_t* text = lds + (size_t)PR_TB * FP * 4;
  const int r0 = blockIdx.x * PR_TB;
  const int nr = min(PR_TB, a.n_rows - r0);
  const long long s_lo = a.starts[r0];
  const long long s_hi = r0 + nr < a.n_rows ? a.starts[r0 + nr] : a.n_bytes;
  const long long a_lo = s_lo & ~15ll;
  const long long span = s_hi - a_lo;
  const float nan = __builtin_nanf("");
  if (span > cap) {  // global-memory path for this workgroup
    if (tid < nr) {
      const int r = r0 + tid;
      float* row = a.X + (size_t)r * F;
      for (int c = 0; c < F; ++c) row[c] = nan;
      if (parse_record(a.buf + a.starts[r], a.buf + a.n_bytes, a.n_cols, a.colmap, a.delim, a.n_missing, a.missing,
                       row))
        flag_row(a, r);
    }
    return;
  }
  for (int c = tid; c < a.n_cols; c += PR_TB) colmap_l[c] = a.colmap[c];
  for (int i = tid; i < a.n_missing * TP_MISSING_LEN; i += PR_TB) missing_l[i] = a.missing[i];
  for (int i = tid; i < PR_TB * FP; i += PR_TB) out[i] = nan;
  // stage [a_lo, s_hi): whole 16-byte words inside the chunk, the tail byte by byte
  const long long full_end = min(s_hi + 15, a.n_bytes) & ~15ll;  // 16-byte words fully inside the chunk
  const int n16 = (int)((full_end - a_lo) >> 4);
  const uint4* src = reinterpret_cast<const uint4*>(a.buf + a_lo);
  uint4* dst = reinterpret_cast<uint4*>(text);
  for (int i = tid; i < n16; i += PR_TB) dst[i] = src[i];
  for (long long p = full_end + tid; p < s_hi; p += PR_TB) text[p - a_lo] = a.buf[p];
  __syncthreads();
  if (tid < nr) {
    const int r = r0 + tid;
    if (parse_record(text + (a.starts[r] - a_lo), text + span, a.n_cols, colmap_l, a.delim, a.n_missing, missing_l,
                     out + tid * FP))
      flag_row(a, r);
  }
  __syncthreads();
  // the tile is X[r0 : r0 + nr] — one contiguous run of nr * F floats
  float* xo = a.X + (size_t)r0 * F;
  const int total = nr * F;
  for (int i = tid; i < total; i += PR_TB) {
    const int rr = i / F;
    xo[i] = out[rr * FP + (i - rr * F)];
  }
}

}  // namespace

PMML_API int pmml_textparse_args_size() { return (int)sizeof(TextParseArgs); }

// Row starts of a chunk: tile_counts needs ceil(n_bytes / 4096) + 1 ints; the total row count
// lands in tile_counts[n_tiles]. Call pmml_text_rows_write afterwards (the host sizes the output
// from the total) to fill `starts`.
PMML_API int pmml_text_rows_count(hipStream_t stream, const uint8_t* buf, long long n_bytes, int* tile_counts) {
  if (n_bytes <= 0) return 0;
  const long long tiles = (n_bytes + TP_TILE - 1) / TP_TILE;
  if (tiles > 0x7FFFFFFFLL) return -2;
  hipLaunchKernelGGL(row_start_count, dim3((unsigned)tiles), dim3(TP_TB), 0, stream, buf, n_bytes, tile_counts);
  hipLaunchKernelGGL(row_start_scan, dim3(1), dim3(1024), 0, stream, tile_counts, (int)tiles);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

PMML_API int pmml_text_rows_write(hipStream_t stream, const uint8_t* buf, long long n_bytes, const int* tile_offsets,
                                  long long* starts) {
  if (n_bytes <= 0) return 0;
  const long long tiles = (n_bytes + TP_TILE - 1) / TP_TILE;
  hipLaunchKernelGGL(row_start_write, dim3((unsigned)tiles), dim3(TP_TB), 0, stream, buf, n_bytes, tile_offsets,
                     starts);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

PMML_API int pmml_text_parse(hipStream_t stream, const TextParseArgs* args) {
  const TextParseArgs& a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.F < 1 || a.n_cols < 1 || a.n_missing < 0 || a.n_missing > TP_MAX_MISSING) return -2;
  // LDS staging capacity: 1.25x the chunk's average bytes per workgroup (so two workgroups share a
  // CU for 32-field rows); a workgroup over it parses from global memory.
  const long long avg = a.n_bytes / a.n_rows + 1;
  const long long out_bytes = (long long)PR_TB * (a.F + 1) * 4;
  long long cap = ((avg * PR_TB * 5 / 4 + 256) + 15) & ~15ll;
  cap = std::max(cap, 4096ll);
  const long long lds_max = 160 * 1024 - 2048;  // minus the static tables
  const bool lds_ok = a.n_cols <= PR_MAX_COLS && ((reinterpret_cast<uintptr_t>(a.buf) & 15) == 0) &&
                      out_bytes + 4096 + 16 <= lds_max;
  if (!lds_ok) {
    hipLaunchKernelGGL(parse_rows, dim3((a.n_rows + TP_TB - 1) / TP_TB), dim3(TP_TB), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -7;
  }
  cap = std::min(cap, lds_max - out_bytes - 16);
  const size_t lds = (size_t)(out_bytes + cap + 16);
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(parse_rows_lds),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(parse_rows_lds, dim3((a.n_rows + PR_TB - 1) / PR_TB), dim3(PR_TB), lds, stream, a, (int)cap);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
