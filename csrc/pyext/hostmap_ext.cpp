// mp4x._native._mp4x_hostmap — native passes of the HOST map collectives (values on the CPU:
// Python scalars, numpy rows, objects).  Plain CPython API, no torch: a host-only job never pays
// for importing libtorch.
//
// partition(map, p): the owner split every host ``*Map`` collective starts with
// (ProcessCommSlave.allreduceMap / reduceMap / broadcastMap, J/comm/ProcessCommSlave.java:2053-2088,
// 1490-1516, 842-883).  The Python rule hashes each key through ``str.encode('utf-16-be')`` and a
// Python-level loop (~3.7 us per key); here it is one dict walk reading the str's PEP 393 buffer.
// stack_rows(values, out): the value-row copy of the map codecs without np.stack's per-value checks.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>

#include <cstdint>
#include <cstring>

namespace {

// java.lang.String.hashCode of a str: 31-polynomial over its UTF-16 code units, int32 wrap
// (code points above U+FFFF count as their surrogate pair, as in Java).
template <typename CH>
uint32_t java_hash(const CH* s, Py_ssize_t n) {
  uint32_t h = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    const uint32_t c = s[i];
    if (sizeof(CH) == 4 && c > 0xFFFF) {
      const uint32_t u = c - 0x10000;
      h = 31 * h + (0xD800 + (u >> 10));
      h = 31 * h + (0xDC00 + (u & 0x3FF));
    } else {
      h = 31 * h + c;
    }
  }
  return h;
}

// partition(map, p) -> [p dicts] | None
// The host map collectives' owner rule ``key.hashCode() % p`` with Java's signed remainder and
// negatives wrapped (mp4x/utils/hashing.py owner_of; reference ProcessCommSlave.java:2059-2072),
// insertion order kept within each part.  None when a key is not a str (the Python rule decides).
PyObject* partition(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 2 || !PyDict_Check(a[0])) {
    PyErr_SetString(PyExc_TypeError, "partition(map: dict, p: int)");
    return nullptr;
  }
  const long p = PyLong_AsLong(a[1]);
  if (p <= 0) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "partition: p must be > 0");
    return nullptr;
  }
  PyObject* map = a[0];
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(map, &pos, &k, &v))
    if (!PyUnicode_CheckExact(k) || PyUnicode_READY(k) != 0) Py_RETURN_NONE;
  PyObject* parts = PyList_New(p);
  if (!parts) return nullptr;
  for (long r = 0; r < p; ++r) {
    PyObject* d = PyDict_New();
    if (!d) {
      Py_DECREF(parts);
      return nullptr;
    }
    PyList_SET_ITEM(parts, r, d);
  }
  pos = 0;
  while (PyDict_Next(map, &pos, &k, &v)) {
    const Py_ssize_t n = PyUnicode_GET_LENGTH(k);
    const void* data = PyUnicode_DATA(k);
    uint32_t h;
    switch (PyUnicode_KIND(k)) {
      case PyUnicode_1BYTE_KIND: h = java_hash(static_cast<const Py_UCS1*>(data), n); break;
      case PyUnicode_2BYTE_KIND: h = java_hash(static_cast<const Py_UCS2*>(data), n); break;
      default: h = java_hash(static_cast<const Py_UCS4*>(data), n); break;
    }
    const int64_t hs = static_cast<int32_t>(h);
    int64_t idx = (hs < 0 ? -hs : hs) % p;
    if (hs < 0 && idx != 0) idx = p - idx;
    if (PyDict_SetItem(PyList_GET_ITEM(parts, idx), k, v) != 0) {
      Py_DECREF(parts);
      return nullptr;
    }
  }
  return parts;
}

// owner_ids(keys: list, p, out) -> bool
// The same owner rule as ``partition`` for a key LIST, written as int32 into ``out`` (a writable
// C-contiguous int32 buffer of len(keys)): the columnar host map path (mp4x/parallel/hostmap.py)
// splits keys and value rows with one stable argsort of these ids instead of building p dicts.
// False when a key is not a str (the caller applies the Python rule).
PyObject* owner_ids(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 3 || !PyList_Check(a[0])) {
    PyErr_SetString(PyExc_TypeError, "owner_ids(keys: list, p: int, out)");
    return nullptr;
  }
  const long p = PyLong_AsLong(a[1]);
  if (p <= 0) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "owner_ids: p must be > 0");
    return nullptr;
  }
  Py_buffer ob;
  if (PyObject_GetBuffer(a[2], &ob, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  const Py_ssize_t n = PyList_GET_SIZE(a[0]);
  if (ob.len != n * (Py_ssize_t)sizeof(int32_t)) {
    PyBuffer_Release(&ob);
    PyErr_SetString(PyExc_ValueError, "owner_ids: out must hold len(keys) int32");
    return nullptr;
  }
  int32_t* out = static_cast<int32_t*>(ob.buf);
  bool ok = true;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* k = PyList_GET_ITEM(a[0], i);
    if (!PyUnicode_CheckExact(k) || PyUnicode_READY(k) != 0) {
      ok = false;
      break;
    }
    const Py_ssize_t len = PyUnicode_GET_LENGTH(k);
    const void* data = PyUnicode_DATA(k);
    uint32_t h;
    switch (PyUnicode_KIND(k)) {
      case PyUnicode_1BYTE_KIND: h = java_hash(static_cast<const Py_UCS1*>(data), len); break;
      case PyUnicode_2BYTE_KIND: h = java_hash(static_cast<const Py_UCS2*>(data), len); break;
      default: h = java_hash(static_cast<const Py_UCS4*>(data), len); break;
    }
    const int64_t hs = static_cast<int32_t>(h);
    int64_t idx = (hs < 0 ? -hs : hs) % p;
    if (hs < 0 && idx != 0) idx = p - idx;
    out[i] = static_cast<int32_t>(idx);
  }
  PyBuffer_Release(&ob);
  if (ok) Py_RETURN_TRUE;
  Py_RETURN_FALSE;
}

// stack_rows(values: list, out) -> bool
// np.stack for the map codecs (mp4x/parallel/wire.py): copy each value's bytes into row i of the
// C-contiguous ``out`` through the buffer protocol.  False (nothing promised about ``out``) as
// soon as a value is not a C-contiguous buffer of exactly one row with out's item format; the
// caller then takes np.stack.  np.stack spends ~1.3 us per value on array checks and shape sets.
PyObject* stack_rows(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 2 || !PyList_Check(a[0])) {
    PyErr_SetString(PyExc_TypeError, "stack_rows(values: list, out)");
    return nullptr;
  }
  Py_buffer ob;
  if (PyObject_GetBuffer(a[1], &ob, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return nullptr;
  const Py_ssize_t n = PyList_GET_SIZE(a[0]);
  bool ok = n > 0 && ob.len % n == 0 && ob.format != nullptr;
  const Py_ssize_t row = ok ? ob.len / n : 0;
  char* dst = static_cast<char*>(ob.buf);
  // numpy rows (the common case): read the array struct directly — type number, contiguity and
  // byte size — instead of a buffer-protocol round trip per row (~10x cheaper per value)
  const int out_type = PyArray_Check(a[1]) ? PyArray_TYPE(reinterpret_cast<PyArrayObject*>(a[1])) : -1;
  for (Py_ssize_t i = 0; ok && i < n; ++i) {
    PyObject* it = PyList_GET_ITEM(a[0], i);
    if (out_type >= 0 && PyArray_CheckExact(it)) {
      PyArrayObject* arr = reinterpret_cast<PyArrayObject*>(it);
      if (PyArray_TYPE(arr) == out_type && PyArray_NBYTES(arr) == row && PyArray_IS_C_CONTIGUOUS(arr) &&
          PyArray_ISNOTSWAPPED(arr)) {
        std::memcpy(dst + i * row, PyArray_DATA(arr), row);
        continue;
      }
    }
    Py_buffer vb;
    if (PyObject_GetBuffer(it, &vb, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
      PyErr_Clear();
      ok = false;
      break;
    }
    ok = vb.len == row && vb.itemsize == ob.itemsize && vb.format != nullptr && std::strcmp(vb.format, ob.format) == 0;
    if (ok) std::memcpy(dst + i * row, vb.buf, row);
    PyBuffer_Release(&vb);
  }
  PyBuffer_Release(&ob);
  if (ok) Py_RETURN_TRUE;
  Py_RETURN_FALSE;
}

// learn_keys(key2id: dict, id2key: list, proposals) -> int
// One key-dictionary sync round (mp4x/parallel/sparse.py KeyDictionary.learn_round): walk every
// rank's block of proposed keys in rank order and give each key not in ``key2id`` yet the next id
// (= len(id2key)), appending it to ``id2key``.  ONE dict operation per key (PyDict_SetDefault:
// a single probe that inserts or finds) instead of the union dict + membership test + insert of
// the Python form.  Blocks may be None.  Returns the number of new keys, or (number, new dict) when
// it numbered a large first round into a presized dict the caller must use instead of key2id.
PyObject* learn_keys(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 3 || !PyDict_CheckExact(a[0]) || !PyList_CheckExact(a[1])) {
    PyErr_SetString(PyExc_TypeError, "learn_keys(key2id: dict, id2key: list, proposals)");
    return nullptr;
  }
  PyObject* d = a[0];
  PyObject* ids = a[1];
  const Py_ssize_t base = PyList_GET_SIZE(ids);
  // A large round into an EMPTY dictionary (a map collective's first call: ~1M keys) grows the
  // dict through ~17 resizes that rehash every entry; presizing it to the proposals' total avoids
  // them.  The caller then swaps the returned dict in (learn_keys returns (count, dict)).
  PyObject* fresh = nullptr;
  if (PyDict_GET_SIZE(d) == 0 && PyList_CheckExact(a[2])) {
    Py_ssize_t total = 0;
    for (Py_ssize_t b = 0; b < PyList_GET_SIZE(a[2]); ++b) {
      PyObject* blk = PyList_GET_ITEM(a[2], b);
      if (blk != Py_None && PyList_CheckExact(blk)) total += PyList_GET_SIZE(blk);
    }
    if (total > (1 << 16)) {
      fresh = _PyDict_NewPresized(total);
      if (!fresh) return nullptr;
      d = fresh;
    }
  }
  Py_ssize_t next = base;
  PyObject* it = PyObject_GetIter(a[2]);
  if (!it) return nullptr;
  PyObject* blk;
  while ((blk = PyIter_Next(it)) != nullptr) {
    if (blk == Py_None) {
      Py_DECREF(blk);
      continue;
    }
    PyObject* seq = PySequence_Fast(blk, "learn_keys: every proposal block must be a sequence or None");
    Py_DECREF(blk);
    if (!seq) break;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    PyObject** items = PySequence_Fast_ITEMS(seq);
    bool ok = true;
    PyObject* id = nullptr;                                    // the next id, made once per insert
    for (Py_ssize_t i = 0; i < n && ok; ++i) {
      if (!id && !(id = PyLong_FromSsize_t(next))) {
        ok = false;
        break;
      }
      PyObject* got = PyDict_SetDefault(d, items[i], id);     // borrowed
      if (!got) {
        ok = false;
      } else if (got == id) {                                  // inserted: a new key
        if (PyList_Append(ids, items[i]) != 0) ok = false;
        ++next;
        Py_DECREF(id);                                         // the dict holds it now
        id = nullptr;
      }                                                        // known key: the id object is reused
    }
    Py_XDECREF(id);
    Py_DECREF(seq);
    if (!ok) break;
  }
  Py_DECREF(it);
  if (PyErr_Occurred()) {
    Py_XDECREF(fresh);
    return nullptr;
  }
  if (fresh) return Py_BuildValue("(nN)", next - base, fresh);
  return PyLong_FromSsize_t(next - base);
}

PyMethodDef kMethods[] = {
    {"partition", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(partition)), METH_FASTCALL,
     "partition(map, p) -> [p dicts] by Java String.hashCode % p, or None for non-str keys"},
    {"owner_ids", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(owner_ids)), METH_FASTCALL,
     "owner_ids(keys, p, out) -> bool: out[i] = Java String.hashCode(keys[i]) % p (int32)"},
    {"stack_rows", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(stack_rows)), METH_FASTCALL,
     "stack_rows(values, out) -> bool: row i of out = bytes of values[i]"},
    {"learn_keys", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(learn_keys)), METH_FASTCALL,
     "learn_keys(key2id, id2key, proposals) -> int: number the keys not in key2id yet, in order"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_mp4x_hostmap", "native passes of the host map collectives", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__mp4x_hostmap() {
  import_array();
  return PyModule_Create(&kModule);
}
