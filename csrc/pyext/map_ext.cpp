// mp4x._native._mp4x_map — one native pass that turns a Dict[key, Tensor] into the operands of
// the device map collectives (ids + rows), for ``allreduceMap`` & co on GPU tensors
// (mp4x/parallel/sparse.py ``_map_tensors``; reference: ProcessCommSlave.allreduceMap,
// J/comm/ProcessCommSlave.java:2053-2088, which walks the map entry by entry).
//
// Why native: with 200k float[64] values per rank (BASELINE config 4) the Python form spends its
// time on per-value attribute calls — dictionary lookup 27 ms, ``_base`` 44 ms, ``numel`` 36 ms,
// ``is_contiguous`` 27 ms, ``storage_offset`` 25 ms on this container's CPU — each a torch
// method dispatch of 100+ ns.  Here one ``PyDict_Next`` walk does the key lookup (the str hash is
// cached in the key object) and reads the same tensor facts straight off ``at::Tensor``.
//
// pack(map, key2id, base, ids, rows) -> (n_missing, rows_ok)
//   map     dict whose values are tensors
//   key2id  dict key -> int id (the communicator's KeyDictionary)
//   base    None, or the contiguous tensor every value is expected to be a whole row of, a row
//           being numel(first value) elements (base viewed as [numel / d, d])
//   ids     writable int64 buffer of len(map): the key's id, -1 where the key has no id yet
//   rows    writable int64 buffer of len(map): the value's row index in ``base`` (when rows_ok)
// rows_ok is False as soon as one value is not a whole contiguous row of ``base`` (other
// storage, other dtype or numel, not contiguous, misaligned or out of range); ids are always complete.
//
// pack(map, key2id, base, ids, rows, hint_keys, hint_ids, make_hint) -> (n_missing, rows_ok, hits, keys)
//   the position hint of a fresh dict built from the same key objects as an earlier one (the
//   GBDT / feature-count pattern: a new dict per call, same feature-name strings, same order):
//   hint_keys  None or a tuple of the key objects of an earlier complete walk, in its order
//   hint_ids   None or an int64 buffer of their ids (same length)
//   make_hint  True: also return this walk's keys as a tuple (the next call's hint_keys)
//   A key that IS the hint's key object at its position takes the hinted id with no dictionary
//   probe — a pointer compare instead of a cache-missing lookup in a dictionary of ~1M keys
//   (ids never change once given, and the tuple keeps the objects alive, so identity is exact).
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>

namespace {

struct OutBuf {
  Py_buffer v{};
  bool ok = false;
  ~OutBuf() {
    if (ok) PyBuffer_Release(&v);
  }
};

bool get_i64(PyObject* o, OutBuf* b, Py_ssize_t n, const char* what) {
  if (PyObject_GetBuffer(o, &b->v, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return false;
  b->ok = true;
  const char* f = b->v.format;
  if (f && (*f == '@' || *f == '=' || *f == '<')) ++f;
  if (b->v.itemsize != 8 || !f || !(f[0] == 'l' || f[0] == 'q') || f[1] || b->v.len != n * 8) {
    PyErr_Format(PyExc_ValueError, "%s must be a writable int64 buffer of %zd elements", what, n);
    return false;
  }
  return true;
}

PyObject* pack(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 5 && na != 8) {
    PyErr_Format(PyExc_TypeError, "pack expects 5 or 8 arguments, got %zd", na);
    return nullptr;
  }
  PyObject* map = a[0];
  PyObject* key2id = a[1];
  if (!PyDict_Check(map) || !PyDict_Check(key2id)) {
    PyErr_SetString(PyExc_TypeError, "pack: map and key2id must be dicts");
    return nullptr;
  }
  const Py_ssize_t n = PyDict_GET_SIZE(map);
  OutBuf ib, rb;
  if (!get_i64(a[3], &ib, n, "ids") || !get_i64(a[4], &rb, n, "rows")) return nullptr;
  auto* ids = static_cast<int64_t*>(ib.v.buf);
  auto* rows = static_cast<int64_t*>(rb.v.buf);

  // the base tensor's facts (rows are checked against these)
  bool rows_ok = false;
  const c10::StorageImpl* storage = nullptr;
  int64_t base_off = 0, d = 0, nrows = 0;
  caffe2::TypeMeta dtype;
  if (a[2] != Py_None) {
    if (!THPVariable_Check(a[2])) {
      PyErr_SetString(PyExc_TypeError, "pack: base must be a tensor or None");
      return nullptr;
    }
    const at::Tensor& b = THPVariable_Unpack(a[2]);
    // rows are d = numel(first value) elements: base viewed as [numel / d, d]
    PyObject* first = nullptr;
    Py_ssize_t p0 = 0;
    PyObject* k0;
    if (PyDict_Next(map, &p0, &k0, &first) && THPVariable_Check(first) && b.defined() && b.is_contiguous()) {
      d = THPVariable_Unpack(first).numel();
      if (d > 0 && b.numel() > 0 && b.numel() % d == 0) {
        storage = b.storage().unsafeGetStorageImpl();
        base_off = b.storage_offset();
        nrows = b.numel() / d;
        dtype = b.dtype();
        rows_ok = true;
      }
    }
  }

  // the optional position hint + the keys tuple this walk hands back
  PyObject* hk = nullptr;
  const int64_t* hid = nullptr;
  Py_ssize_t nh = 0;
  OutBuf hb;
  PyObject* keys_out = nullptr;
  if (na == 8) {
    if (a[5] != Py_None && a[6] != Py_None) {
      if (!PyTuple_Check(a[5])) {
        PyErr_SetString(PyExc_TypeError, "pack: hint_keys must be a tuple or None");
        return nullptr;
      }
      nh = PyTuple_GET_SIZE(a[5]);
      if (PyObject_GetBuffer(a[6], &hb.v, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return nullptr;
      hb.ok = true;
      if (hb.v.itemsize != 8 || hb.v.len != nh * 8) {
        PyErr_SetString(PyExc_ValueError, "pack: hint_ids must be an int64 buffer as long as hint_keys");
        return nullptr;
      }
      hk = a[5];
      hid = static_cast<const int64_t*>(hb.v.buf);
    }
    if (PyObject_IsTrue(a[7]) && !(keys_out = PyTuple_New(n))) return nullptr;
  }

  Py_ssize_t pos = 0, i = 0;
  PyObject *k, *v;
  int64_t missing = 0, hits = 0;
  while (PyDict_Next(map, &pos, &k, &v)) {
    if (i >= n) break;                                     // a key's __eq__ grew the map
    if (keys_out) {
      Py_INCREF(k);
      PyTuple_SET_ITEM(keys_out, i, k);
    }
    if (i < nh && PyTuple_GET_ITEM(hk, i) == k) {          // same key object at this position
      ids[i] = hid[i];
      ++hits;
      goto row;
    }
    {
    PyObject* id = PyDict_GetItemWithError(key2id, k);   // borrowed
    if (id) {
      const long long x = PyLong_AsLongLong(id);
      if (x == -1 && PyErr_Occurred()) {
        Py_XDECREF(keys_out);
        return nullptr;
      }
      ids[i] = x;
    } else {
      if (PyErr_Occurred()) {                             // unhashable key etc.
        Py_XDECREF(keys_out);
        return nullptr;
      }
      ids[i] = -1;
      ++missing;
    }
    }
  row:
    if (rows_ok) {
      if (!THPVariable_Check(v)) {
        rows_ok = false;
      } else {
        // TensorImpl fields only: no Storage handle copy (two atomic refcount ops per value)
        const c10::TensorImpl* t = THPVariable_Unpack(v).unsafeGetTensorImpl();
        const int64_t off = t->storage_offset() - base_off;
        if (!t->has_storage() || t->unsafe_storage().unsafeGetStorageImpl() != storage || t->numel() != d ||
            t->dtype() != dtype || !t->is_contiguous() || off < 0 || off % d != 0 || off / d >= nrows) {
          rows_ok = false;
        } else {
          rows[i] = off / d;
        }
      }
    }
    ++i;
  }
  if (i != n) {
    Py_XDECREF(keys_out);
    PyErr_SetString(PyExc_RuntimeError, "pack: map changed size during the walk");
    return nullptr;
  }
  if (na == 5) return Py_BuildValue("(LO)", static_cast<long long>(missing), rows_ok ? Py_True : Py_False);
  return Py_BuildValue("(LOLN)", static_cast<long long>(missing), rows_ok ? Py_True : Py_False,
                       static_cast<long long>(hits), keys_out ? keys_out : (Py_INCREF(Py_None), Py_None));
}

// dict_version(d) -> int: CPython's per-dict modification tag (PEP 509, ``ma_version_tag``).
// Every insert, delete or value replacement gives the dict a new, globally unique tag, so an
// equal tag means the same dict with the same key -> value objects: the walk's result for it
// (ids, rows) still holds, and the device Map API skips the walk for a map passed again as is.
PyObject* dict_version(PyObject*, PyObject* d) {
  if (!PyDict_Check(d)) {
    PyErr_SetString(PyExc_TypeError, "dict_version(dict)");
    return nullptr;
  }
  return PyLong_FromUnsignedLongLong(reinterpret_cast<PyDictObject*>(d)->ma_version_tag);
}

PyMethodDef kMethods[] = {
    {"pack", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(pack)), METH_FASTCALL,
     "pack(map, key2id, base, ids, rows[, hint_keys, hint_ids, make_hint]) -> (n_missing, rows_ok[, hits, keys])"},
    {"dict_version", reinterpret_cast<PyCFunction>(dict_version), METH_O, "dict_version(d) -> PEP 509 tag"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_mp4x_map", "native Dict[key, Tensor] -> ids/rows pass", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__mp4x_map() { return PyModule_Create(&kModule); }
