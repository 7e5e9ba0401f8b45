// Per-record fast path of the stream runtime (CPython C API + NumPy C API, built with g++).
//
// The reference scores one record at a time: every event is a FlinkML vector and every result a
// `Prediction(Score(x))` object (`S/package.scala:76-82,138-142`, `S/models/prediction/Prediction.scala:72`).
// The MI355X engine keeps that API but scores micro-batches on the GPU, so the per-record cost that
// remains is purely host-side object traffic:
//
//   * pack_dense      — a list of DenseVector objects -> one [n, width] float64 matrix. Reads each
//                       vector's `data` slot through the slot's member offset (no attribute lookup)
//                       and memcpy's its contiguous float64 payload.
//   * make_predictions — scores/valid arrays -> list of Prediction(Score(x)) / the shared
//                       EmptyScore prediction. Objects are allocated with tp_alloc and their slots
//                       filled directly (the Python __init__s only assign those same slots).
//   * scan_trees      — the streaming TreeModel reader of large PMML documents (pmml_scan.cpp).
//   * forest_leaves / forest_values / forest_sums / forest_votes — the float64 oracle's tree walk in C++
//     (tree_walk.cpp).
//   * seq_affine      — the oracle's NeuralNetwork layer sums in connection order (nn_host.cpp).
//
// Both return None / -1 when an input does not have the exact expected shape; the Python caller
// then takes its general (slower, element-wise) path — results are identical either way.

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#define PY_ARRAY_UNIQUE_SYMBOL fja_fastpath_ARRAY_API
#include <numpy/arrayobject.h>

#include <cstdint>
#include <cstring>
#include <vector>

PyObject *fja_scan_trees(PyObject *, PyObject *args);     // pmml_scan.cpp
PyObject *fja_forest_compile(PyObject *, PyObject *args); // tree_walk.cpp
PyObject *fja_set_walk_threads(PyObject *, PyObject *args); // tree_walk.cpp
PyObject *fja_forest_leaves(PyObject *, PyObject *args);  // tree_walk.cpp
PyObject *fja_forest_values(PyObject *, PyObject *args);  // tree_walk.cpp
PyObject *fja_forest_sums(PyObject *, PyObject *args);    // tree_walk.cpp
PyObject *fja_forest_votes(PyObject *, PyObject *args);   // tree_walk.cpp
PyObject *fja_seq_affine(PyObject *, PyObject *args);     // nn_host.cpp

namespace {

// Byte offset of the __slots__ member `name` of heap type `tp` (-1 if it is not a slot).
Py_ssize_t slot_offset(PyTypeObject *tp, const char *name) {
    PyObject *descr = PyObject_GetAttrString(reinterpret_cast<PyObject *>(tp), name);
    if (!descr) {
        PyErr_Clear();
        return -1;
    }
    Py_ssize_t off = -1;
    if (Py_IS_TYPE(descr, &PyMemberDescr_Type)) {
        PyMemberDef *m = reinterpret_cast<PyMemberDescrObject *>(descr)->d_member;
        if (m->type == T_OBJECT_EX || m->type == T_OBJECT) off = m->offset;
    }
    Py_DECREF(descr);
    return off;
}

// pack_dense(vectors: list, dense_type: type, width: int, out: ndarray[float64, n*width]) -> int
// Returns n on success, -1 if some element is not an exact `dense_type` whose `data` slot holds a
// C-contiguous float64 1-D array of `width` values (nothing is guaranteed about `out` then).
PyObject *pack_dense(PyObject *, PyObject *args) {
    PyObject *seq, *type_obj, *out_obj;
    Py_ssize_t width;
    if (!PyArg_ParseTuple(args, "O!OnO", &PyList_Type, &seq, &type_obj, &width, &out_obj)) return nullptr;
    if (!PyType_Check(type_obj) || !PyArray_Check(out_obj)) {
        PyErr_SetString(PyExc_TypeError, "pack_dense(list, type, int, ndarray)");
        return nullptr;
    }
    PyTypeObject *tp = reinterpret_cast<PyTypeObject *>(type_obj);
    PyArrayObject *out = reinterpret_cast<PyArrayObject *>(out_obj);
    const Py_ssize_t n = PyList_GET_SIZE(seq);
    if (width < 0) {
        PyErr_SetString(PyExc_ValueError, "pack_dense: negative width");
        return nullptr;
    }
    if (PyArray_TYPE(out) != NPY_DOUBLE || !PyArray_IS_C_CONTIGUOUS(out) || PyArray_SIZE(out) < n * width) {
        PyErr_SetString(PyExc_ValueError, "pack_dense: out must be a C-contiguous float64 array of n*width");
        return nullptr;
    }
    const Py_ssize_t off = slot_offset(tp, "data");
    if (off < 0) return PyLong_FromLong(-1);
    double *dst = static_cast<double *>(PyArray_DATA(out));
    const size_t row_bytes = static_cast<size_t>(width) * sizeof(double);
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *v = PyList_GET_ITEM(seq, i);
        if (Py_TYPE(v) != tp) return PyLong_FromLong(-1);
        PyObject *data = *reinterpret_cast<PyObject **>(reinterpret_cast<char *>(v) + off);
        if (!data || !PyArray_Check(data)) return PyLong_FromLong(-1);
        PyArrayObject *a = reinterpret_cast<PyArrayObject *>(data);
        if (PyArray_TYPE(a) != NPY_DOUBLE || PyArray_NDIM(a) != 1 || PyArray_DIM(a, 0) != width ||
            !PyArray_IS_C_CONTIGUOUS(a))
            return PyLong_FromLong(-1);
        std::memcpy(dst + i * width, PyArray_DATA(a), row_bytes);
    }
    return PyLong_FromSsize_t(n);
}

// make_predictions(scores: float32[n], valid: bool/uint8[n], prediction_type, score_type, empty) -> list
PyObject *make_predictions(PyObject *, PyObject *args) {
    PyObject *s_obj, *v_obj, *ptype_obj, *stype_obj, *empty;
    if (!PyArg_ParseTuple(args, "OOOOO", &s_obj, &v_obj, &ptype_obj, &stype_obj, &empty)) return nullptr;
    if (!PyArray_Check(s_obj) || !PyArray_Check(v_obj) || !PyType_Check(ptype_obj) || !PyType_Check(stype_obj)) {
        PyErr_SetString(PyExc_TypeError, "make_predictions(ndarray, ndarray, type, type, object)");
        return nullptr;
    }
    PyArrayObject *sa = reinterpret_cast<PyArrayObject *>(s_obj);
    PyArrayObject *va = reinterpret_cast<PyArrayObject *>(v_obj);
    if (PyArray_TYPE(sa) != NPY_FLOAT || !PyArray_IS_C_CONTIGUOUS(sa) || PyArray_ITEMSIZE(va) != 1 ||
        !PyArray_IS_C_CONTIGUOUS(va) || PyArray_SIZE(va) != PyArray_SIZE(sa)) {
        Py_RETURN_NONE;
    }
    PyTypeObject *ptype = reinterpret_cast<PyTypeObject *>(ptype_obj);
    PyTypeObject *stype = reinterpret_cast<PyTypeObject *>(stype_obj);
    const Py_ssize_t p_val = slot_offset(ptype, "value"), p_out = slot_offset(ptype, "outputs");
    const Py_ssize_t s_val = slot_offset(stype, "value");
    if (p_val < 0 || p_out < 0 || s_val < 0) Py_RETURN_NONE;
    const Py_ssize_t n = PyArray_SIZE(sa);
    const float *s = static_cast<const float *>(PyArray_DATA(sa));
    const unsigned char *ok = static_cast<const unsigned char *>(PyArray_DATA(va));
    PyObject *list = PyList_New(n);
    if (!list) return nullptr;
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (!ok[i]) {
            Py_INCREF(empty);
            PyList_SET_ITEM(list, i, empty);
            continue;
        }
        PyObject *f = PyFloat_FromDouble(static_cast<double>(s[i]));
        PyObject *score = f ? stype->tp_alloc(stype, 0) : nullptr;
        PyObject *pred = score ? ptype->tp_alloc(ptype, 0) : nullptr;
        if (!pred) {
            Py_XDECREF(f);
            Py_XDECREF(score);
            Py_DECREF(list);
            return nullptr;
        }
        *reinterpret_cast<PyObject **>(reinterpret_cast<char *>(score) + s_val) = f;  // steals f
        *reinterpret_cast<PyObject **>(reinterpret_cast<char *>(pred) + p_val) = score;  // steals score
        Py_INCREF(Py_None);
        *reinterpret_cast<PyObject **>(reinterpret_cast<char *>(pred) + p_out) = Py_None;
        PyList_SET_ITEM(list, i, pred);
    }
    return list;
}

// group_ids(ids: list | ndarray[object]) -> (codes: int32[n], keys: list)
// Dictionary-encodes a per-row model-id column in first-appearance order (the mixed-model batch of
// the dynamic operator, `S/package.scala:111-114`, keyed by id string). Rows usually repeat a few
// id objects: a 256-entry direct-mapped cache on the object pointer answers most rows without
// hashing; misses fall back to a dict keyed by the (equal-comparing) id values.
PyObject *group_ids(PyObject *, PyObject *args) {
    PyObject *seq;
    if (!PyArg_ParseTuple(args, "O", &seq)) return nullptr;
    PyObject *fast = nullptr;
    PyObject **items;
    Py_ssize_t n;
    if (PyArray_Check(seq)) {
        PyArrayObject *a = reinterpret_cast<PyArrayObject *>(seq);
        if (PyArray_TYPE(a) != NPY_OBJECT || PyArray_NDIM(a) != 1 || !PyArray_IS_C_CONTIGUOUS(a)) {
            PyErr_SetString(PyExc_TypeError, "group_ids: a 1-D contiguous object array or a list");
            return nullptr;
        }
        items = static_cast<PyObject **>(PyArray_DATA(a));
        n = PyArray_DIM(a, 0);
    } else {
        fast = PySequence_Fast(seq, "group_ids: a sequence of ids");
        if (!fast) return nullptr;
        items = PySequence_Fast_ITEMS(fast);
        n = PySequence_Fast_GET_SIZE(fast);
    }
    npy_intp dims[1] = {static_cast<npy_intp>(n)};
    PyObject *codes_obj = PyArray_SimpleNew(1, dims, NPY_INT32);
    PyObject *keys = PyList_New(0);
    PyObject *index = PyDict_New();
    if (!codes_obj || !keys || !index) {
        Py_XDECREF(codes_obj);
        Py_XDECREF(keys);
        Py_XDECREF(index);
        Py_XDECREF(fast);
        return nullptr;
    }
    int32_t *codes = static_cast<int32_t *>(PyArray_DATA(reinterpret_cast<PyArrayObject *>(codes_obj)));
    PyObject *cache_obj[256] = {nullptr};
    int32_t cache_code[256];
    bool ok = true;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *o = items[i];
        const size_t h = (reinterpret_cast<uintptr_t>(o) >> 4) & 255;
        if (cache_obj[h] == o) {
            codes[i] = cache_code[h];
            continue;
        }
        PyObject *c = PyDict_GetItemWithError(index, o);  // borrowed
        int32_t code;
        if (c) {
            code = static_cast<int32_t>(PyLong_AsLong(c));
        } else {
            if (PyErr_Occurred()) {
                ok = false;
                break;
            }
            code = static_cast<int32_t>(PyList_GET_SIZE(keys));
            PyObject *v = PyLong_FromLong(code);
            if (!v || PyDict_SetItem(index, o, v) < 0 || PyList_Append(keys, o) < 0) {
                Py_XDECREF(v);
                ok = false;
                break;
            }
            Py_DECREF(v);
        }
        // the dict holds a reference to an equal key, and `items` keeps `o` alive for the loop
        cache_obj[h] = o;
        cache_code[h] = code;
        codes[i] = code;
    }
    Py_DECREF(index);
    Py_XDECREF(fast);
    if (!ok) {
        Py_DECREF(codes_obj);
        Py_DECREF(keys);
        return nullptr;
    }
    return Py_BuildValue("(NN)", codes_obj, keys);
}

// counting_sort(codes: int32[n], k: int) -> (perm: int32[n], counts: int64[k])
// Stable grouping permutation: rows of code 0 first (in row order), then code 1, ... One pass to
// count, one to place; the GIL is released. Codes outside [0, k) raise ValueError.
PyObject *counting_sort(PyObject *, PyObject *args) {
    PyObject *c_obj;
    Py_ssize_t k;
    if (!PyArg_ParseTuple(args, "On", &c_obj, &k)) return nullptr;
    if (!PyArray_Check(c_obj)) {
        PyErr_SetString(PyExc_TypeError, "counting_sort(int32 ndarray, int)");
        return nullptr;
    }
    PyArrayObject *ca = reinterpret_cast<PyArrayObject *>(c_obj);
    if (PyArray_TYPE(ca) != NPY_INT32 || PyArray_NDIM(ca) != 1 || !PyArray_IS_C_CONTIGUOUS(ca) || k < 0 ||
        k > (1 << 24)) {
        PyErr_SetString(PyExc_ValueError, "counting_sort: contiguous 1-D int32 codes and 0 <= k <= 2^24");
        return nullptr;
    }
    const npy_intp n = PyArray_DIM(ca, 0);
    npy_intp dn[1] = {n}, dk[1] = {static_cast<npy_intp>(k)};
    PyObject *perm_obj = PyArray_SimpleNew(1, dn, NPY_INT32);
    PyObject *cnt_obj = PyArray_ZEROS(1, dk, NPY_INT64, 0);
    if (!perm_obj || !cnt_obj) {
        Py_XDECREF(perm_obj);
        Py_XDECREF(cnt_obj);
        return nullptr;
    }
    const int32_t *codes = static_cast<const int32_t *>(PyArray_DATA(ca));
    int32_t *perm = static_cast<int32_t *>(PyArray_DATA(reinterpret_cast<PyArrayObject *>(perm_obj)));
    int64_t *cnt = static_cast<int64_t *>(PyArray_DATA(reinterpret_cast<PyArrayObject *>(cnt_obj)));
    bool ok = n <= 0x7FFFFFFF;
    Py_BEGIN_ALLOW_THREADS;
    for (npy_intp i = 0; ok && i < n; ++i) {
        const int32_t c = codes[i];
        if (c < 0 || c >= k) ok = false;
        else ++cnt[c];
    }
    if (ok) {
        std::vector<int64_t> next(static_cast<size_t>(k) + 1, 0);
        for (Py_ssize_t j = 0; j < k; ++j) next[j + 1] = next[j] + cnt[j];
        for (npy_intp i = 0; i < n; ++i) perm[next[codes[i]]++] = static_cast<int32_t>(i);
    }
    Py_END_ALLOW_THREADS;
    if (!ok) {
        Py_DECREF(perm_obj);
        Py_DECREF(cnt_obj);
        PyErr_SetString(PyExc_ValueError, "counting_sort: code outside [0, k) or more than 2^31 rows");
        return nullptr;
    }
    return Py_BuildValue("(NN)", perm_obj, cnt_obj);
}

PyMethodDef methods[] = {
    {"group_ids", group_ids, METH_VARARGS, "Dictionary-encode a model-id column (first-appearance order)."},
    {"counting_sort", counting_sort, METH_VARARGS, "Stable grouping permutation of int32 codes."},
    {"pack_dense", pack_dense, METH_VARARGS, "Pack a list of DenseVector objects into a float64 matrix."},
    {"make_predictions", make_predictions, METH_VARARGS, "Prediction objects for a scored batch."},
    {"scan_trees", fja_scan_trees, METH_VARARGS, "Streaming TreeModel reader: (skeleton, flat trees, strings)."},
    {"set_walk_threads", fja_set_walk_threads, METH_VARARGS, "Worker threads of the host tree walk (default 1)."},
    {"forest_compile", fja_forest_compile, METH_VARARGS, "Oracle tree walk: compile a program once (capsule)."},
    {"forest_leaves", fja_forest_leaves, METH_VARARGS, "Oracle tree walk: scoring node per tree and row."},
    {"forest_values", fja_forest_values, METH_VARARGS, "Oracle tree walk: leaf value per row and tree."},
    {"forest_sums", fja_forest_sums, METH_VARARGS, "Oracle tree walk: numpy-pairwise ensemble sum per row."},
    {"forest_votes", fja_forest_votes, METH_VARARGS, "Oracle tree walk: (weighted) majority vote shares per row."},
    {"seq_affine", fja_seq_affine, METH_VARARGS, "Oracle NeuralNetwork layer: bias + sum in connection order."},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fastpath", "Per-record fast path of the stream runtime.", -1,
                      methods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__fastpath(void) {
    import_array();
    return PyModule_Create(&module);
}
