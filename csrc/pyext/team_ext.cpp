// mp4x._native._mp4x_team — CPython binding of the native thread team (csrc/host/host_ops.cpp
// ``mp4x_team_*``) for ThreadCommSlave's host-array collectives.
//
// Why a C extension and not ctypes: a 2-thread float[1024] allreduce (BASELINE config 1) moves
// 4 KB; the cost is the Python around it.  Through ctypes each call paid ~2 us of argument
// conversion plus ~2 us for ``ndarray.ctypes.data``, per thread, serialised by the GIL.  Here the
// array goes through the buffer protocol (its format, rank, contiguity and length checked in C)
// and the call is one METH_FASTCALL entry that releases the GIL around the team collective.
//
// Return value: 0 done; a negative native code (barrier timeout / abort) or MP4X_E_*; or
// kNotEligible (the buffer is not a 1-D C-contiguous array of the dtype) -> the caller takes its
// generic path; kOutOfRange ([f, t) does not fit the array) -> the caller raises.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>

extern "C" {
int mp4x_team_barrier(void* h, int tid);
int mp4x_team_reduce(void* h, int tid, void* buf, int64_t f, int64_t t, int dtype, int op, int root);
int mp4x_team_bcast(void* h, int tid, void* buf, int64_t f, int64_t t, int elem_bytes, int root);
int mp4x_team_allreduce(void* h, int tid, void* buf, int64_t f, int64_t t, int dtype, int op);
}

namespace {

constexpr int kNotEligible = -100;
constexpr int kOutOfRange = -101;

// dtype codes of enum mp4x_dtype (csrc/include/mp4x/ops.h): F64 F32 I64 I32 I16 I8
bool format_matches(const char* fmt, int dtype, Py_ssize_t itemsize) {
  if (!fmt) return false;
  if (*fmt == '@' || *fmt == '=' || *fmt == '<') ++fmt;
  if (!fmt[0] || fmt[1]) return false;
  const char c = fmt[0];
  switch (dtype) {
    case 0: return c == 'd';
    case 1: return c == 'f';
    case 2: return (c == 'l' || c == 'q') && itemsize == 8;
    case 3: return (c == 'i' || c == 'l') && itemsize == 4;
    case 4: return c == 'h';
    case 5: return c == 'b';
    default: return false;
  }
}

struct Args {
  void* team;
  int tid;
  Py_buffer view;
  int64_t f, t;
  bool have_view = false;
};

// (team, tid, arr, f, t, dtype) common prefix; returns 0, or a code to hand back to Python, or -1
// with a Python error set.
int parse(PyObject* const* a, Py_ssize_t n, Py_ssize_t want, Args* out, int dtype_at, int* dtype) {
  if (n != want) {
    PyErr_Format(PyExc_TypeError, "expected %zd arguments, got %zd", want, n);
    return -1;
  }
  out->team = PyLong_AsVoidPtr(a[0]);
  out->tid = (int)PyLong_AsLong(a[1]);
  out->f = PyLong_AsLongLong(a[3]);
  out->t = PyLong_AsLongLong(a[4]);
  *dtype = (int)PyLong_AsLong(a[dtype_at]);
  if (PyErr_Occurred()) return -1;
  if (PyObject_GetBuffer(a[2], &out->view, PyBUF_WRITABLE | PyBUF_FORMAT | PyBUF_C_CONTIGUOUS) != 0) {
    PyErr_Clear();
    return kNotEligible;
  }
  out->have_view = true;
  if (out->view.ndim != 1 || !format_matches(out->view.format, *dtype, out->view.itemsize)) return kNotEligible;
  if (out->f < 0 || out->t < out->f || out->t > out->view.shape[0]) return kOutOfRange;
  return 0;
}

PyObject* finish(Args* a, int rc) {
  if (a->have_view) PyBuffer_Release(&a->view);
  if (rc == -1 && PyErr_Occurred()) return nullptr;
  return PyLong_FromLong(rc);
}

PyObject* py_allreduce(PyObject*, PyObject* const* a, Py_ssize_t n) {  // (team, tid, arr, f, t, dtype, op)
  Args x;
  int dtype;
  int rc = parse(a, n, 7, &x, 5, &dtype);
  if (rc == 0) {
    const int op = (int)PyLong_AsLong(a[6]);
    if (PyErr_Occurred()) return finish(&x, -1);
    Py_BEGIN_ALLOW_THREADS
    rc = mp4x_team_allreduce(x.team, x.tid, x.view.buf, x.f, x.t, dtype, op);
    Py_END_ALLOW_THREADS
  }
  return finish(&x, rc);
}

PyObject* py_reduce(PyObject*, PyObject* const* a, Py_ssize_t n) {  // (team, tid, arr, f, t, dtype, op, root)
  Args x;
  int dtype;
  int rc = parse(a, n, 8, &x, 5, &dtype);
  if (rc == 0) {
    const int op = (int)PyLong_AsLong(a[6]);
    const int root = (int)PyLong_AsLong(a[7]);
    if (PyErr_Occurred()) return finish(&x, -1);
    Py_BEGIN_ALLOW_THREADS
    rc = mp4x_team_reduce(x.team, x.tid, x.view.buf, x.f, x.t, dtype, op, root);
    Py_END_ALLOW_THREADS
  }
  return finish(&x, rc);
}

PyObject* py_bcast(PyObject*, PyObject* const* a, Py_ssize_t n) {  // (team, tid, arr, f, t, dtype, root)
  Args x;
  int dtype;
  int rc = parse(a, n, 7, &x, 5, &dtype);
  if (rc == 0) {
    const int root = (int)PyLong_AsLong(a[6]);
    if (PyErr_Occurred()) return finish(&x, -1);
    const int es = (int)x.view.itemsize;
    Py_BEGIN_ALLOW_THREADS
    rc = mp4x_team_bcast(x.team, x.tid, x.view.buf, x.f, x.t, es, root);
    Py_END_ALLOW_THREADS
  }
  return finish(&x, rc);
}

PyObject* py_barrier(PyObject*, PyObject* const* a, Py_ssize_t n) {  // (team, tid)
  if (n != 2) {
    PyErr_SetString(PyExc_TypeError, "barrier(team, tid)");
    return nullptr;
  }
  void* team = PyLong_AsVoidPtr(a[0]);
  const int tid = (int)PyLong_AsLong(a[1]);
  if (PyErr_Occurred()) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = mp4x_team_barrier(team, tid);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

PyMethodDef kMethods[] = {
    {"allreduce", (PyCFunction)(void (*)(void))py_allreduce, METH_FASTCALL, "team allreduce of arr[f:t]"},
    {"reduce", (PyCFunction)(void (*)(void))py_reduce, METH_FASTCALL, "team reduce of arr[f:t] into root"},
    {"bcast", (PyCFunction)(void (*)(void))py_bcast, METH_FASTCALL, "root's arr[f:t] to every thread"},
    {"barrier", (PyCFunction)(void (*)(void))py_barrier, METH_FASTCALL, "team barrier"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_mp4x_team", "native thread-team collectives", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__mp4x_team(void) {
  PyObject* m = PyModule_Create(&kModule);
  if (m) {
    PyModule_AddIntConstant(m, "NOT_ELIGIBLE", kNotEligible);
    PyModule_AddIntConstant(m, "OUT_OF_RANGE", kOutOfRange);
  }
  return m;
}
