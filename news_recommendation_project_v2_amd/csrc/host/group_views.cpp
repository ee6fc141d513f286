// Host side of the drop-in API's return format: get_final_second_attention_score
// (data_model_helper.py:416-443) returns `grouped_scores`, an object array with
// one 1-D array per impression (group_items, data_utils.py:400-411:
// np.array([items[s:e] for ...], dtype=object)).  At MIND-large-dev size that is
// 376 k Python-level slices, 59-63 ms of the call's 87-91 ms (bench
// extra.api_end_to_end_ms, round 6) while the GPU work is 9.7 ms.  This CPython
// extension builds the same object array in C: every element a 1-D view of
// `items` (the same dtype, memory and base object as items[s:e]), created with
// the NumPy C API in one pass, no Python frames per element.
//
//   _nrhost.group_views(items: 1-D C-contiguous ndarray, counts: 1-D int64 ndarray)
//       -> ndarray[object] of len(counts) views
//
// Semantics kept by the caller (data_utils.group_items): equal counts
// everywhere (np.array would build a 2-D object array), n == 0, or a `func`
// still take the NumPy path, so the result is always what the reference's
// expression returns.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>

#include <stdint.h>

#ifndef NRX_BUILD_HASH
#define NRX_BUILD_HASH "unknown"
#endif
// the content hash build() compares against the source (read from the file's bytes)
extern "C" __attribute__((used)) const char nrx_build_hash[] = "nrx-build-hash:" NRX_BUILD_HASH;

static PyObject* group_views(PyObject*, PyObject* args) {
  PyObject *items_o = nullptr, *counts_o = nullptr;
  if (!PyArg_ParseTuple(args, "OO", &items_o, &counts_o)) return nullptr;
  if (!PyArray_Check(items_o) || !PyArray_Check(counts_o)) {
    PyErr_SetString(PyExc_TypeError, "group_views: items and counts must be ndarrays");
    return nullptr;
  }
  PyArrayObject* items = (PyArrayObject*)items_o;
  PyArrayObject* counts = (PyArrayObject*)counts_o;
  if (PyArray_NDIM(items) != 1 || !PyArray_IS_C_CONTIGUOUS(items) || PyArray_NDIM(counts) != 1 ||
      PyArray_TYPE(counts) != NPY_INT64 || !PyArray_IS_C_CONTIGUOUS(counts)) {
    PyErr_SetString(PyExc_ValueError, "group_views: 1-D C-contiguous items and int64 counts expected");
    return nullptr;
  }
  const npy_intp n = PyArray_DIM(counts, 0), len = PyArray_DIM(items, 0);
  const int64_t* c = (const int64_t*)PyArray_DATA(counts);
  int64_t total = 0;
  for (npy_intp i = 0; i < n; ++i) {
    if (c[i] < 0) {
      PyErr_SetString(PyExc_ValueError, "group_views: negative count");
      return nullptr;
    }
    total += c[i];
  }
  if (total > (int64_t)len) {
    PyErr_SetString(PyExc_ValueError, "group_views: counts sum past the items");
    return nullptr;
  }
  npy_intp dims[1] = {n};
  PyArrayObject* out = (PyArrayObject*)PyArray_SimpleNew(1, dims, NPY_OBJECT);
  if (!out) return nullptr;
  PyObject** slot = (PyObject**)PyArray_DATA(out);
  PyArray_Descr* descr = PyArray_DESCR(items);
  const npy_intp isz = PyArray_ITEMSIZE(items);
  char* base = (char*)PyArray_DATA(items);
  const int flags = PyArray_FLAGS(items) & (NPY_ARRAY_WRITEABLE | NPY_ARRAY_ALIGNED);
  int64_t off = 0;
  for (npy_intp i = 0; i < n; ++i) {
    npy_intp d[1] = {(npy_intp)c[i]};
    npy_intp st[1] = {isz};
    Py_INCREF(descr);  // stolen by NewFromDescr
    PyObject* v = PyArray_NewFromDescr(&PyArray_Type, descr, 1, d, st, base + off * isz,
                                       flags | NPY_ARRAY_C_CONTIGUOUS | NPY_ARRAY_F_CONTIGUOUS, nullptr);
    if (!v) {
      Py_DECREF(out);
      return nullptr;
    }
    Py_INCREF(items_o);
    if (PyArray_SetBaseObject((PyArrayObject*)v, items_o) < 0) {  // steals the reference
      Py_DECREF(v);
      Py_DECREF(out);
      return nullptr;
    }
    Py_XDECREF(slot[i]);  // PyArray_SimpleNew(NPY_OBJECT) fills with None
    slot[i] = v;
    off += c[i];
  }
  return (PyObject*)out;
}

static PyMethodDef kMethods[] = {
    {"group_views", group_views, METH_VARARGS, "object array of per-group 1-D views of items"},
    {nullptr, nullptr, 0, nullptr}};

static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_nrhost", "native host helpers of the drop-in API", -1,
                                     kMethods};

PyMODINIT_FUNC PyInit__nrhost(void) {
  import_array();
  return PyModule_Create(&kModule);
}
