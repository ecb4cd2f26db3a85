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

using AllreduceEx = int (*)(int algo, int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs, int rank,
                            int p, int64_t nbytes, const void* src, void* out, uint32_t epoch, int blocks,
                            const uint32_t* epoch_dev, float scale, void* stream);

AllreduceEx g_allreduce_ex = nullptr;

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
  if (na != 15) {
    PyErr_SetString(PyExc_TypeError, "allreduce_ex takes 15 arguments");
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
  if (PyErr_Occurred()) return nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_allreduce_ex(algo, dtype, op, data, sig, rank, p, nbytes, src, out, epoch, blocks, edev, scale, stream);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

PyMethodDef kMethods[] = {
    {"bind", bind, METH_O, "bind(address of mp4x_ipc_allreduce_ex in the loaded libmp4x_hip.so)"},
    {"allreduce_ex", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(allreduce_ex)), METH_FASTCALL,
     "allreduce_ex(algo, dtype, op, data_pp, sig_pp, rank, p, nbytes, src, out, epoch, blocks, epoch_dev, scale, "
     "stream) -> rc"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_mp4x_launch", "ctypes-free launch of the IPC allreduce kernels", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__mp4x_launch(void) { return PyModule_Create(&kModule); }
