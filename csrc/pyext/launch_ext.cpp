// _mp4x_launch: the per-call launch of the IPC allreduce kernels without ctypes.
//
// A small device allreduce is host-bound (profiles/r4/latency/): ctypes converts each of the 15
// arguments of mp4x_ipc_allreduce_ex through its argtypes on every call (~2 us of a ~12 us call).
// This extension parses them with METH_FASTCALL and calls the SAME exported function of
// libmp4x_hip.so through a pointer handed over once (``bind``: the address ctypes resolved in the
// already-loaded library, so release / debug builds and the torch HIP runtime are the ones in use).
// No HIP headers, no link against the HIP library.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>

namespace {

// mp4x_ipc_allreduce_ex2 (the slot arguments last; 0 / 0 = the single-buffer form)
using AllreduceEx = int (*)(int algo, int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs, int rank,
                            int p, int64_t nbytes, const void* src, void* out, uint32_t epoch, int blocks,
                            const uint32_t* epoch_dev, float scale, void* stream, int64_t slot_base,
                            int64_t slot_vecs);

AllreduceEx g_allreduce_ex = nullptr;

// mp4x_ipc_fast_allreduce(state, algo, dtype, op, buf, nbytes, blocks, scale, stream): the latency
// tier's whole per-call path (error words, capture check, epoch, launch) in libmp4x_hip.so.
using FastAllreduce = int (*)(const void* state, int algo, int dtype, int op, void* buf, int64_t nbytes, int blocks,
                              float scale, void* stream);
FastAllreduce g_fast = nullptr;

// mp4x_ipc_fast_plan(state, stage, nstage, pull, npull, src_off, out_off, base, grid_len, buf_vecs,
// blocks, stream): the same one-call path for a memoised copy plan.
using FastPlan = int (*)(const void* state, const int64_t* stage, int nstage, const int64_t* pull, int npull,
                         int64_t src_off, int64_t out_off, void* base, int64_t grid_len, int64_t buf_vecs, int blocks,
                         void* stream);
FastPlan g_fast_plan = nullptr;

// mp4x_ipc_fast_rs(state, dtype, op, seg_lo, seg_hi, src_off, out_off, base, blocks, stream): the
// same for a memoised fused reduce-scatter.
using FastRs = int (*)(const void* state, int dtype, int op, const int64_t* seg_lo, const int64_t* seg_hi,
                       int64_t src_off, int64_t out_off, void* base, int blocks, void* stream);
FastRs g_fast_rs = nullptr;

void* as_ptr(PyObject* o) {   // int address, or None -> NULL
  if (o == Py_None) return nullptr;
  return PyLong_AsVoidPtr(o);
}

PyObject* bind(PyObject*, PyObject* addr) {
  void* f = PyLong_AsVoidPtr(addr);
  if (!f && PyErr_Occurred()) return nullptr;
  g_allreduce_ex = reinterpret_cast<AllreduceEx>(f);
  Py_RETURN_NONE;
}

// allreduce_ex(algo, dtype, op, data_pp, sig_pp, rank, p, nbytes, src, out, epoch, blocks,
//              epoch_dev, scale, stream) -> rc     (pointers as int addresses or None)
PyObject* allreduce_ex(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 15 && na != 17) {
    PyErr_SetString(PyExc_TypeError, "allreduce_ex takes 15 arguments (+ slot_base, slot_vecs)");
    return nullptr;
  }
  if (!g_allreduce_ex) {
    PyErr_SetString(PyExc_RuntimeError, "_mp4x_launch: bind() was not called");
    return nullptr;
  }
  const int algo = (int)PyLong_AsLong(a[0]);
  const int dtype = (int)PyLong_AsLong(a[1]);
  const int op = (int)PyLong_AsLong(a[2]);
  void* const* data = static_cast<void* const*>(as_ptr(a[3]));
  void* const* sig = static_cast<void* const*>(as_ptr(a[4]));
  const int rank = (int)PyLong_AsLong(a[5]);
  const int p = (int)PyLong_AsLong(a[6]);
  const int64_t nbytes = PyLong_AsLongLong(a[7]);
  const void* src = as_ptr(a[8]);
  void* out = as_ptr(a[9]);
  const uint32_t epoch = (uint32_t)PyLong_AsUnsignedLong(a[10]);
  const int blocks = (int)PyLong_AsLong(a[11]);
  const uint32_t* edev = static_cast<const uint32_t*>(as_ptr(a[12]));
  const float scale = (float)PyFloat_AsDouble(a[13]);
  void* stream = as_ptr(a[14]);
  const int64_t slot_base = na == 17 ? PyLong_AsLongLong(a[15]) : 0;
  const int64_t slot_vecs = na == 17 ? PyLong_AsLongLong(a[16]) : 0;
  if (PyErr_Occurred()) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_allreduce_ex(algo, dtype, op, data, sig, rank, p, nbytes, src, out, epoch, blocks, edev, scale, stream,
                      slot_base, slot_vecs);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

PyObject* bind_fast(PyObject*, PyObject* addr) {
  void* f = PyLong_AsVoidPtr(addr);
  if (!f && PyErr_Occurred()) return nullptr;
  g_fast = reinterpret_cast<FastAllreduce>(f);
  Py_RETURN_NONE;
}

// fast_allreduce(entry, stream[, base]) -> rc.  `entry` is the engine's memoised launch tuple
// (state address, algo, dtype, op, buffer address — or its offset from `base` when base is given —,
// nbytes, blocks, scale); rc 1003 / 1004 / MP4X_E_BADARG = not launched (an earlier collective
// failed / the stream is capturing / an unaligned buffer): the caller takes the full path.
PyObject* fast_allreduce(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if ((na != 2 && na != 3) || !PyTuple_Check(a[0]) || PyTuple_GET_SIZE(a[0]) < 8) {
    PyErr_SetString(PyExc_TypeError, "fast_allreduce(entry: tuple of 8, stream[, base])");
    return nullptr;
  }
  if (!g_fast) {
    PyErr_SetString(PyExc_RuntimeError, "_mp4x_launch: bind_fast() was not called");
    return nullptr;
  }
  PyObject* const* t = &PyTuple_GET_ITEM(a[0], 0);
  const void* state = PyLong_AsVoidPtr(t[0]);
  const int algo = (int)PyLong_AsLong(t[1]);
  const int dtype = (int)PyLong_AsLong(t[2]);
  const int op = (int)PyLong_AsLong(t[3]);
  char* buf = static_cast<char*>(PyLong_AsVoidPtr(t[4]));
  if (na == 3) buf = static_cast<char*>(PyLong_AsVoidPtr(a[2])) + PyLong_AsLongLong(t[4]);
  const int64_t nbytes = PyLong_AsLongLong(t[5]);
  const int blocks = (int)PyLong_AsLong(t[6]);
  const float scale = (float)PyFloat_AsDouble(t[7]);
  void* stream = as_ptr(a[1]);
  if (PyErr_Occurred()) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_fast(state, algo, dtype, op, buf, nbytes, blocks, scale, stream);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

PyObject* bind_fast_plan(PyObject*, PyObject* addr) {
  void* f = PyLong_AsVoidPtr(addr);
  if (!f && PyErr_Occurred()) return nullptr;
  g_fast_plan = reinterpret_cast<FastPlan>(f);
  Py_RETURN_NONE;
}

// fast_plan(entry, stream, base) -> rc.  `entry`: the engine's memoised copy plan (state address,
// stage array address, nstage, pull array address, npull, src_off, out_off, grid_len, buf_vecs,
// blocks, ...); rc != 0 = not launched (an earlier collective failed / capturing / unaligned): the
// caller takes the full path.
PyObject* fast_plan(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 3 || !PyTuple_Check(a[0]) || PyTuple_GET_SIZE(a[0]) < 10) {
    PyErr_SetString(PyExc_TypeError, "fast_plan(entry: tuple of >= 10, stream, base)");
    return nullptr;
  }
  if (!g_fast_plan) {
    PyErr_SetString(PyExc_RuntimeError, "_mp4x_launch: bind_fast_plan() was not called");
    return nullptr;
  }
  PyObject* const* t = &PyTuple_GET_ITEM(a[0], 0);
  const void* state = PyLong_AsVoidPtr(t[0]);
  const int64_t* stage = static_cast<const int64_t*>(PyLong_AsVoidPtr(t[1]));
  const int nstage = (int)PyLong_AsLong(t[2]);
  const int64_t* pull = static_cast<const int64_t*>(PyLong_AsVoidPtr(t[3]));
  const int npull = (int)PyLong_AsLong(t[4]);
  const int64_t src_off = PyLong_AsLongLong(t[5]);
  const int64_t out_off = PyLong_AsLongLong(t[6]);
  const int64_t grid_len = PyLong_AsLongLong(t[7]);
  const int64_t buf_vecs = PyLong_AsLongLong(t[8]);
  const int blocks = (int)PyLong_AsLong(t[9]);
  void* stream = as_ptr(a[1]);
  void* base = PyLong_AsVoidPtr(a[2]);
  if (PyErr_Occurred()) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_fast_plan(state, stage, nstage, pull, npull, src_off, out_off, base, grid_len, buf_vecs, blocks, stream);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

PyObject* bind_fast_rs(PyObject*, PyObject* addr) {
  void* f = PyLong_AsVoidPtr(addr);
  if (!f && PyErr_Occurred()) return nullptr;
  g_fast_rs = reinterpret_cast<FastRs>(f);
  Py_RETURN_NONE;
}

// fast_rs(entry, stream, base) -> rc.  `entry`: the engine's memoised reduce-scatter (state
// address, dtype, op, seg_lo array address, seg_hi array address, src_off, out_off, blocks, ...).
PyObject* fast_rs(PyObject*, PyObject* const* a, Py_ssize_t na) {
  if (na != 3 || !PyTuple_Check(a[0]) || PyTuple_GET_SIZE(a[0]) < 8) {
    PyErr_SetString(PyExc_TypeError, "fast_rs(entry: tuple of >= 8, stream, base)");
    return nullptr;
  }
  if (!g_fast_rs) {
    PyErr_SetString(PyExc_RuntimeError, "_mp4x_launch: bind_fast_rs() was not called");
    return nullptr;
  }
  PyObject* const* t = &PyTuple_GET_ITEM(a[0], 0);
  const void* state = PyLong_AsVoidPtr(t[0]);
  const int dtype = (int)PyLong_AsLong(t[1]);
  const int op = (int)PyLong_AsLong(t[2]);
  const int64_t* lo = static_cast<const int64_t*>(PyLong_AsVoidPtr(t[3]));
  const int64_t* hi = static_cast<const int64_t*>(PyLong_AsVoidPtr(t[4]));
  const int64_t src_off = PyLong_AsLongLong(t[5]);
  const int64_t out_off = PyLong_AsLongLong(t[6]);
  const int blocks = (int)PyLong_AsLong(t[7]);
  void* stream = as_ptr(a[1]);
  void* base = PyLong_AsVoidPtr(a[2]);
  if (PyErr_Occurred()) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_fast_rs(state, dtype, op, lo, hi, src_off, out_off, base, blocks, stream);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

PyMethodDef kMethods[] = {
    {"bind_fast_rs", bind_fast_rs, METH_O, "bind_fast_rs(address of mp4x_ipc_fast_rs in libmp4x_hip.so)"},
    {"fast_rs", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(fast_rs)), METH_FASTCALL,
     "fast_rs(entry, stream, base) -> rc"},
    {"bind_fast_plan", bind_fast_plan, METH_O, "bind_fast_plan(address of mp4x_ipc_fast_plan in libmp4x_hip.so)"},
    {"fast_plan", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(fast_plan)), METH_FASTCALL,
     "fast_plan(entry, stream, base) -> rc"},
    {"bind_fast", bind_fast, METH_O, "bind_fast(address of mp4x_ipc_fast_allreduce in the loaded libmp4x_hip.so)"},
    {"fast_allreduce", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(fast_allreduce)), METH_FASTCALL,
     "fast_allreduce(entry, stream) -> rc"},
    {"bind", bind, METH_O, "bind(address of mp4x_ipc_allreduce_ex2 in the loaded libmp4x_hip.so)"},
    {"allreduce_ex", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(allreduce_ex)), METH_FASTCALL,
     "allreduce_ex(algo, dtype, op, data_pp, sig_pp, rank, p, nbytes, src, out, epoch, blocks, epoch_dev, scale, "
     "stream) -> rc"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_mp4x_launch", "ctypes-free launch of the IPC allreduce kernels", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__mp4x_launch(void) { return PyModule_Create(&kModule); }
