// Host NeuralNetwork layer of the float64 oracle (linked into `_fastpath`).
//
// JPMML computes every neuron as bias + w_0 x_0 + w_1 x_1 + ... in connection order, one rounding
// per product and per sum (`S/api/PmmlModel.scala:159-160`; Java has no implicit FMA). The numpy
// oracle (`models/neural.py::forward`) reproduces that with one vector operation per CONNECTION —
// a million numpy calls for a 1024 x 1024 layer. This is the same arithmetic in C++, vectorised
// across the layer's neurons: when every neuron of a layer reads the same sources in the same
// order, z[r, j] = (((b_j + W[0, j] x[r, s_0]) + W[1, j] x[r, s_1]) + ...), bit-identical to the
// numpy loop (the build passes -ffp-contract=off: no fused multiply-add).
//
//   seq_affine(A f64 [n, k], order int32 [m], W f64 [m, out], b f64 [out], out f64 [n, out])
//       order[t] = column of A read by term t (every neuron's t-th connection), W[t, j] its weight.

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace {

struct View {
    Py_buffer b{};
    bool ok = false;
    ~View() {
        if (ok) PyBuffer_Release(&b);
    }
    bool get(PyObject *o, char type, Py_ssize_t itemsize, bool writable, const char *what) {
        if (PyObject_GetBuffer(o, &b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT | (writable ? PyBUF_WRITABLE : 0)) != 0)
            return false;
        ok = true;
        const char *f = b.format ? b.format : "B";
        if (*f == '<' || *f == '=' || *f == '@') ++f;
        if (b.itemsize != itemsize || f[0] != type || f[1] != '\0') {
            PyErr_Format(PyExc_TypeError, "seq_affine: %s must be a C-contiguous '%c' buffer", what, type);
            return false;
        }
        return true;
    }
    Py_ssize_t n() const { return b.len / b.itemsize; }
};

// The blocked loop (rows in blocks of RB: each weight row W[t] is read once per block while the
// block's partial sums stay in L2; the per-neuron term order is unchanged). Instantiated for the
// baseline ISA and for AVX-512 (8 neurons per instruction; -ffp-contract=off keeps the product and
// the sum separately rounded there too).
#define FJA_SEQ_AFFINE_BODY                                                                              \
    constexpr Py_ssize_t RB = 32;                                                                        \
    for (Py_ssize_t r0 = 0; r0 < n; r0 += RB) {                                                          \
        const Py_ssize_t r1 = r0 + RB < n ? r0 + RB : n;                                                 \
        for (Py_ssize_t r = r0; r < r1; ++r) std::memcpy(z + r * out, bias, sizeof(double) * (size_t)out); \
        for (Py_ssize_t t = 0; t < m; ++t) {                                                             \
            const double *wt = w + t * out;                                                              \
            const int32_t col = ord[t];                                                                  \
            for (Py_ssize_t r = r0; r < r1; ++r) {                                                       \
                const double x = a[r * k + col];                                                         \
                double *zr = z + r * out;                                                                \
                for (Py_ssize_t j = 0; j < out; ++j) {                                                   \
                    const double p = wt[j] * x;                                                          \
                    zr[j] = zr[j] + p;                                                                   \
                }                                                                                        \
            }                                                                                            \
        }                                                                                                \
    }

void affine_base(const double *a, Py_ssize_t n, Py_ssize_t k, const int32_t *ord, Py_ssize_t m, const double *w,
                 const double *bias, Py_ssize_t out, double *z) {
    FJA_SEQ_AFFINE_BODY
}

#if defined(__x86_64__)
// Register-blocked AVX-512 form: 8 rows x 8 neurons of partial sums live in zmm registers across
// the whole term loop (one weight vector load feeds 8 rows), separate mul and add instructions —
// the same two roundings per term, in the same order, as the loop above.
__attribute__((target("avx512f"))) void affine_avx512(const double *a, Py_ssize_t n, Py_ssize_t k,
                                                      const int32_t *ord, Py_ssize_t m, const double *w,
                                                      const double *bias, Py_ssize_t out, double *z) {
    constexpr int R = 8;
    Py_ssize_t r0 = 0;
    for (; r0 + R <= n; r0 += R) {
        for (Py_ssize_t j0 = 0; j0 < out; j0 += 8) {
            const Py_ssize_t rem = out - j0;
            const __mmask8 mk = rem >= 8 ? static_cast<__mmask8>(0xFF) : static_cast<__mmask8>((1u << rem) - 1u);
            const __m512d b0 = _mm512_maskz_loadu_pd(mk, bias + j0);
            __m512d acc[R];
            for (int rr = 0; rr < R; ++rr) acc[rr] = b0;
            const double *ar = a + r0 * k;
            for (Py_ssize_t t = 0; t < m; ++t) {
                const __m512d wv = _mm512_maskz_loadu_pd(mk, w + t * out + j0);
                const int32_t col = ord[t];
#pragma GCC unroll 8
                for (int rr = 0; rr < R; ++rr)
                    acc[rr] = _mm512_add_pd(acc[rr], _mm512_mul_pd(wv, _mm512_set1_pd(ar[rr * k + col])));
            }
            for (int rr = 0; rr < R; ++rr) _mm512_mask_storeu_pd(z + (r0 + rr) * out + j0, mk, acc[rr]);
        }
    }
    if (r0 < n) affine_base(a + r0 * k, n - r0, k, ord, m, w, bias, out, z + r0 * out);
}
#endif

PyObject *seq_affine(PyObject *, PyObject *args) {
    PyObject *oa, *oo, *ow, *ob, *oz;
    Py_ssize_t k;
    if (!PyArg_ParseTuple(args, "OnOOOO", &oa, &k, &oo, &ow, &ob, &oz)) return nullptr;
    View A, order, W, b, Z;
    if (!A.get(oa, 'd', 8, false, "A") || !order.get(oo, 'i', 4, false, "order") || !W.get(ow, 'd', 8, false, "W") ||
        !b.get(ob, 'd', 8, false, "b") || !Z.get(oz, 'd', 8, true, "out"))
        return nullptr;
    const Py_ssize_t out = b.n(), m = order.n();
    if (k < 1 || A.n() % k || W.n() != m * out) {
        PyErr_SetString(PyExc_ValueError, "seq_affine: shape mismatch");
        return nullptr;
    }
    const Py_ssize_t n = A.n() / k;
    if (Z.n() != n * out) {
        PyErr_SetString(PyExc_ValueError, "seq_affine: output shape mismatch");
        return nullptr;
    }
    const int32_t *ord = static_cast<const int32_t *>(order.b.buf);
    for (Py_ssize_t t = 0; t < m; ++t)
        if (ord[t] < 0 || ord[t] >= k) {
            PyErr_SetString(PyExc_ValueError, "seq_affine: source column out of range");
            return nullptr;
        }
    const double *a = static_cast<const double *>(A.b.buf);
    const double *w = static_cast<const double *>(W.b.buf);
    const double *bias = static_cast<const double *>(b.b.buf);
    double *z = static_cast<double *>(Z.b.buf);
#if defined(__x86_64__)
    const bool avx = __builtin_cpu_supports("avx512f");
#else
    const bool avx = false;
#endif
    Py_BEGIN_ALLOW_THREADS
#if defined(__x86_64__)
    if (avx)
        affine_avx512(a, n, k, ord, m, w, bias, out, z);
    else
#endif
        affine_base(a, n, k, ord, m, w, bias, out, z);
    Py_END_ALLOW_THREADS
    Py_RETURN_NONE;
}

}  // namespace

PyObject *fja_seq_affine(PyObject *self, PyObject *args) { return seq_affine(self, args); }
