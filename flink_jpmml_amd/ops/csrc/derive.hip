// Derived fields (PMML TransformationDictionary / LocalTransformations) on the device.
//
// A DerivedField's expression tree (Apply / FieldRef / Constant / NormContinuous / NormDiscrete /
// Discretize / MapValues) is lowered on the host (runtime/derive.py) into a postfix program over
// a per-row fp64 value stack. One workgroup owns DTB rows:
//  * the raw input tile is staged into LDS as [col][DTB] with the MiningField preparation fused
//    (stage_rows_T: missing replacement, validity + invalidValueTreatment, outliers); rows the
//    preparation rejects are flagged;
//  * every lane runs the same instruction stream (the program is uniform, so control flow never
//    diverges — only value selects differ per lane); the stack lives in LDS lane-major
//    ([slot][DTB] doubles: conflict-free, no scratch); derived results are appended to the tile as
//    new columns so later derived fields can reference earlier ones;
//  * the columns the model reads (out_cols) are written back row-major ([rows, n_sel],
//    coalesced): the augmented, already-prepared input matrix of the model kernel that runs next.
// Program arithmetic is fp64 like the host oracle (pmml/fields.py::eval_expression); stored
// columns are rounded to fp32 (every model kernel consumes fp32 features).
#include "common.h"

namespace {

constexpr int DTB = 128;     // rows per workgroup
constexpr int DSTACK = 16;   // value-stack depth (checked on the host)

struct DInsn {
  int op, a, b, c;
  double x, y;
};
static_assert(sizeof(DInsn) == 32, "DInsn mirrors runtime/derive.py");

struct DeriveArgs {
  const float* X;
  int n_rows, n_in, ldx, n_tile;  // n_tile = n_in + number of derived columns
  const FieldPrep* prep;          // [n_in] or null
  const DInsn* prog;
  const double* pool;
  const int* out_cols;            // [n_sel] tile columns written to `out`
  int n_insn, n_sel;
  float* out;                     // [n_rows, n_sel]
  uint8_t* row_ok;                // [n_rows]
};

enum : int {
  D_LOAD = 0, D_CONST = 1, D_MAPMISS = 2, D_REMAP = 3, D_NORMCONT = 4, D_NORMDISC = 5, D_DISCRETIZE = 6,
  D_MAPVALUES = 7, D_APPLY = 8, D_STORE = 9,
};

// Apply function ids (mirror of runtime/derive.py::APPLY_FN)
enum : int {
  F_ADD = 0, F_SUB, F_MUL, F_DIV, F_POW, F_MOD, F_HYPOT, F_ATAN2,      // binary arithmetic
  F_EQ = 10, F_NE, F_LT, F_LE, F_GT, F_GE, F_THRESHOLD,                 // comparisons -> 0/1
  F_LOG10 = 20, F_LN, F_SQRT, F_ABS, F_EXP, F_FLOOR, F_CEIL, F_ROUND, F_RINT, F_SIN, F_COS, F_TAN, F_ASIN,
  F_ACOS, F_ATAN, F_SINH, F_COSH, F_TANH, F_EXPM1, F_LN1P, F_NOT,      // unary
  F_ERF, F_SNCDF, F_SNPDF, F_SNIDF,                                    // unary, PMML 4.4 (41-44)
  F_MIN = 50, F_MAX, F_SUM, F_AVG, F_PRODUCT, F_MEDIAN, F_AND, F_OR,   // n-ary
  F_ISMISSING = 60, F_ISNOTMISSING, F_IF,                              // no mapMissingTo / defaultValue
};

__device__ __forceinline__ bool isnan_d(double v) { return v != v; }

__device__ __forceinline__ double unary(int fn, double v) {
  switch (fn) {
    case F_LOG10: return log10(v);
    case F_LN: return log(v);
    case F_SQRT: return sqrt(v);
    case F_ABS: return fabs(v);
    case F_EXP: return exp(v);
    case F_FLOOR: return floor(v);
    case F_CEIL: return ceil(v);
    case F_ROUND: return floor(v + 0.5);
    case F_RINT: return rint(v);
    case F_SIN: return sin(v);
    case F_COS: return cos(v);
    case F_TAN: return tan(v);
    case F_ASIN: return asin(v);
    case F_ACOS: return acos(v);
    case F_ATAN: return atan(v);
    case F_SINH: return sinh(v);
    case F_COSH: return cosh(v);
    case F_TANH: return tanh(v);
    case F_EXPM1: return expm1(v);
    case F_LN1P: return log1p(v);
    case F_NOT: return v == 0.0 ? 1.0 : 0.0;
    case F_ERF: return erf(v);
    case F_SNCDF: return normcdf(v);
    case F_SNPDF: return exp(-0.5 * v * v) * 0.3989422804014327;  // 1 / sqrt(2 pi)
    case F_SNIDF: return normcdfinv(v);
    default: return __builtin_nan("");
  }
}

__device__ __forceinline__ double binary(int fn, double a, double b) {
  switch (fn) {
    case F_ADD: return a + b;
    case F_SUB: return a - b;
    case F_MUL: return a * b;
    case F_DIV: return a / b;
    case F_POW: return pow(a, b);
    case F_MOD: {  // numpy.mod: the result takes the sign of the divisor (a zero result too: -0.0
                   // for b < 0, which atan2 / a division downstream can see)
      double r = fmod(a, b);
      if (r == 0.0) return copysign(0.0, b);
      if ((r < 0.0) != (b < 0.0)) r += b;
      return r;
    }
    case F_HYPOT: return hypot(a, b);
    case F_ATAN2: return atan2(a, b);
    case F_EQ: return a == b ? 1.0 : 0.0;
    case F_NE: return a != b ? 1.0 : 0.0;
    case F_LT: return a < b ? 1.0 : 0.0;
    case F_LE: return a <= b ? 1.0 : 0.0;
    case F_GT: return a > b ? 1.0 : 0.0;
    case F_GE: return a >= b ? 1.0 : 0.0;
    case F_THRESHOLD: return a > b ? 1.0 : 0.0;
    default: return __builtin_nan("");
  }
}

// closure bit 0: left bound open, bit 1: right bound open (absent bounds are +-inf, closed)
__device__ __forceinline__ bool in_interval(double v, double lo, double hi, int closure) {
  const bool lo_ok = (closure & 1) ? (v > lo) : (v >= lo);
  const bool hi_ok = (closure & 2) ? (v < hi) : (v <= hi);
  return lo_ok && hi_ok;
}

__global__ __launch_bounds__(DTB) void derive_kernel(DeriveArgs a) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  double* stk = reinterpret_cast<double*>(smem_raw);                 // [DSTACK][DTB]
  float* tile = reinterpret_cast<float*>(stk + DSTACK * DTB);        // [n_tile][DTB]
  int* bad = reinterpret_cast<int*>(tile + a.n_tile * DTB);          // [DTB]
  const int tid = threadIdx.x;
  const int row0 = blockIdx.x * DTB;
  stage_rows_T<DTB>(a.X, a.n_rows, a.n_in, a.ldx, a.prep, tile, bad, row0);

#define S(i) stk[(i) * DTB + tid]
  int sp = 0;
  for (int pc = 0; pc < a.n_insn; ++pc) {
    const DInsn in = a.prog[pc];
    switch (in.op) {
      case D_LOAD: S(sp) = (double)tile[in.a * DTB + tid]; ++sp; break;
      case D_CONST: S(sp) = in.x; ++sp; break;
      case D_MAPMISS: {
        const double v = S(sp - 1);
        if (isnan_d(v)) S(sp - 1) = in.x;
        break;
      }
      case D_REMAP: {  // string code of one vocabulary -> code of another
        const double v = S(sp - 1);
        double r = __builtin_nan("");
        if (!isnan_d(v) && v >= 0.0 && v < (double)in.b) r = a.pool[in.a + (int)v];
        S(sp - 1) = r;
        break;
      }
      case D_NORMCONT: {  // piecewise-linear LinearNorm interpolation (pool: orig[b], norm[b])
        const double v = S(sp - 1);
        const double* orig = a.pool + in.a;
        const double* nrm = orig + in.b;
        const int n = in.b;
        double r;
        if (isnan_d(v)) {
          r = in.x;  // mapMissingTo (NaN when absent)
        } else {
          int seg = 0;
          for (int k = 1; k < n - 1; ++k) seg += (v >= orig[k]) ? 1 : 0;
          r = nrm[seg] + (v - orig[seg]) * (nrm[seg + 1] - nrm[seg]) / (orig[seg + 1] - orig[seg]);
          const bool lo = v < orig[0], hi = v > orig[n - 1];
          if (in.c == 1 && (lo || hi)) r = __builtin_nan("");
          if (in.c == 2) r = lo ? nrm[0] : (hi ? nrm[n - 1] : r);
        }
        S(sp - 1) = r;
        break;
      }
      case D_NORMDISC: {
        const double v = S(sp - 1);
        S(sp - 1) = isnan_d(v) ? in.y : (v == in.x ? 1.0 : 0.0);
        break;
      }
      case D_DISCRETIZE: {  // pool: [lo, hi, closure, value] per bin
        const double v = S(sp - 1);
        double r = in.y;  // defaultValue for present, unmatched values
        if (isnan_d(v)) {
          r = in.x;
        } else {
          const double* bins = a.pool + in.a;
          for (int k = 0; k < in.b; ++k) {
            if (in_interval(v, bins[4 * k], bins[4 * k + 1], (int)bins[4 * k + 2])) {
              r = bins[4 * k + 3];
              break;
            }
          }
        }
        S(sp - 1) = r;
        break;
      }
      case D_MAPVALUES: {  // c keys on the stack; pool rows: [key_0..key_{c-1}, out] x b
        const int k = in.c;
        bool anymiss = false;
        for (int j = 0; j < k; ++j) anymiss = anymiss || isnan_d(S(sp - k + j));
        double r = anymiss ? in.x : in.y;
        if (!anymiss) {
          const double* rows = a.pool + in.a;
          for (int i = 0; i < in.b; ++i) {
            bool m = true;
            for (int j = 0; j < k; ++j) m = m && (S(sp - k + j) == rows[i * (k + 1) + j]);
            if (m) {
              r = rows[i * (k + 1) + k];
              break;
            }
          }
        }
        sp -= k;
        S(sp) = r;
        ++sp;
        break;
      }
      case D_APPLY: {
        const int fn = in.a, n = in.b;
        const int base = sp - n;
        double r;
        bool miss = false;
        if (fn == F_ISMISSING || fn == F_ISNOTMISSING) {
          const bool m = isnan_d(S(base));
          r = ((fn == F_ISMISSING) == m) ? 1.0 : 0.0;
          sp = base;
          S(sp) = r;
          ++sp;
          break;
        }
        if (fn == F_IF) {
          const double cond = S(base);
          r = __builtin_nan("");
          if (cond == 1.0 && n > 1) r = S(base + 1);
          if (cond == 0.0 && n > 2) r = S(base + 2);
          sp = base;
          S(sp) = r;
          ++sp;
          break;
        }
        if (fn >= F_MIN && fn <= F_MEDIAN) {  // nan-aware reductions: missing only if every arg is
          int cnt = 0;
          double acc = (fn == F_PRODUCT) ? 1.0 : 0.0;
          double mn = __builtin_inf(), mx = -__builtin_inf();
          for (int j = 0; j < n; ++j) {
            const double v = S(base + j);
            if (isnan_d(v)) continue;
            ++cnt;
            mn = fmin(mn, v);
            mx = fmax(mx, v);
            if (fn == F_PRODUCT) acc *= v; else acc += v;
          }
          miss = cnt == 0;
          if (fn == F_MIN) r = mn;
          else if (fn == F_MAX) r = mx;
          else if (fn == F_SUM || fn == F_PRODUCT) r = acc;
          else if (fn == F_AVG) r = acc / (double)cnt;
          else {  // median: compact + insertion-sort the present values in place (our stack slots)
            int m = 0;
            for (int j = 0; j < n; ++j) {
              const double v = S(base + j);
              if (!isnan_d(v)) { S(base + m) = v; ++m; }
            }
            for (int i = 1; i < m; ++i) {
              const double v = S(base + i);
              int j = i - 1;
              while (j >= 0 && S(base + j) > v) { S(base + j + 1) = S(base + j); --j; }
              S(base + j + 1) = v;
            }
            r = (m == 0) ? __builtin_nan("")
                         : ((m & 1) ? S(base + m / 2) : 0.5 * (S(base + m / 2 - 1) + S(base + m / 2)));
          }
        } else {
          for (int j = 0; j < n; ++j) miss = miss || isnan_d(S(base + j));
          if (fn == F_AND || fn == F_OR) {
            bool acc = (fn == F_AND);
            for (int j = 0; j < n; ++j) {
              const bool t = S(base + j) != 0.0;
              acc = (fn == F_AND) ? (acc && t) : (acc || t);
            }
            r = acc ? 1.0 : 0.0;
          } else if (fn >= F_LOG10) {
            r = unary(fn, S(base));
          } else {
            r = binary(fn, S(base), S(base + 1));
          }
        }
        if (miss) r = in.x;                                 // mapMissingTo (NaN when absent)
        else if (isnan_d(r) && !isnan_d(in.y)) r = in.y;    // defaultValue
        sp = base;
        S(sp) = r;
        ++sp;
        break;
      }
      case D_STORE: {
        double v = S(sp - 1);
        --sp;
        if (in.c == 2 && !isnan_d(v)) v = trunc(v);  // integer
        tile[in.a * DTB + tid] = (float)v;
        break;
      }
      default: break;
    }
  }
#undef S
  __syncthreads();
  const int n_sel = a.n_sel;
  const int total = DTB * n_sel;
  for (int e = tid; e < total; e += DTB) {
    const int r = e / n_sel;
    const int c = e - r * n_sel;
    const int row = row0 + r;
    if (row < a.n_rows) a.out[(size_t)row * n_sel + c] = tile[a.out_cols[c] * DTB + r];
  }
  const int row = row0 + tid;
  if (row < a.n_rows) a.row_ok[row] = bad[tid] ? 0 : 1;
}

__global__ __launch_bounds__(256) void mask_invalid_kernel(float* score, uint8_t* valid, const uint8_t* row_ok,
                                                           float* score2, uint8_t* valid2, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n || row_ok[i]) return;
  score[i] = __builtin_nanf("");
  valid[i] = 0;
  if (score2) {
    score2[i] = __builtin_nanf("");
    valid2[i] = 0;
  }
}

}  // namespace

PMML_API int pmml_derive_args_size() { return (int)sizeof(DeriveArgs); }
PMML_API int pmml_derive_rows_per_block() { return DTB; }
PMML_API int pmml_derive_stack_depth() { return DSTACK; }

PMML_API int pmml_derive_launch(hipStream_t stream, const DeriveArgs* args) {
  const DeriveArgs a = *args;
  if (a.n_rows <= 0) return 0;
  if (a.n_tile < a.n_in || a.n_in <= 0 || a.n_sel <= 0) return -2;
  const size_t lds = (size_t)DSTACK * DTB * 8 + (size_t)a.n_tile * DTB * 4 + DTB * 4;
  if (lds > 160 * 1024) return -5;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(derive_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(derive_kernel, dim3((a.n_rows + DTB - 1) / DTB), dim3(DTB), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

// Rows the field preparation rejected -> EmptyScore (score NaN, valid 0), for model kernels that
// take no per-row validity input.
PMML_API int pmml_mask_invalid(hipStream_t stream, float* score, uint8_t* valid, const uint8_t* row_ok,
                               float* score2, uint8_t* valid2, int n) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mask_invalid_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, score, valid, row_ok,
                     score2, valid2, n);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
