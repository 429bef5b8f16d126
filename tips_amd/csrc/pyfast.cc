// pyfast.cc — tips_amd._fast: the per-tensor host work of a gradient-list call, in C++.
//
// Not part of the C-ABI (include/tips_hip.h has no torch types): this is the Python mirror's
// plumbing, the step between a Python list of torch tensors and tips_fused_allreduce_flat's plain
// pointer and count arrays. The reference walks its gradient list in Python, one op per gradient
// (tips/tensorflow/__init__.py:212-222); here the list is one library call, and for 1000 gradients
// reading each tensor's data pointer, dtype and shape through Python attribute calls cost more host
// time (~0.2 ms) than the fused allreduce's device work. THPVariable_Unpack reads them in tens of
// nanoseconds per tensor.
//
//   dev_list(seq, ptrs_addr, numels_addr[, on_device=1[, cap]]) -> (scalar_type, device_index,
//                                                                  shape_hash) | None
//       every item a dense, contiguous device (HIP) tensor - or, with on_device=0, CPU tensor - of
//       one dtype on one device: writes its
//       data pointer and element count into the int64 arrays at the two addresses (n entries each,
//       allocated by the caller) and returns the dtype (c10::ScalarType as int), the device index
//       and a 64-bit FNV-1a hash of every tensor's (ndim, sizes); None as soon as one item is not
//       such a tensor (the caller takes its general path), and None without writing anything when
//       cap is given and the sequence does not hold exactly cap items (the arrays' size).
//   max_refcount(seq) -> int: the largest reference count of the items (a flat output set is free
//       again when no view of it is referenced outside the library's own lists).
#include <Python.h>

#include <cstdint>

#include <torch/csrc/autograd/python_variable.h>

namespace {

inline uint64_t fnv(uint64_t h, uint64_t v) { return (h ^ v) * 1099511628211ull; }

PyObject* dev_list(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs < 3 || nargs > 5) {
    PyErr_SetString(PyExc_TypeError, "dev_list(seq, ptrs_addr, numels_addr[, on_device=1[, cap]])");
    return nullptr;
  }
  PyObject* seq = PySequence_Fast(args[0], "dev_list: a sequence of tensors");
  if (!seq) return nullptr;
  const unsigned long long pa = PyLong_AsUnsignedLongLong(args[1]);
  const unsigned long long na = PyLong_AsUnsignedLongLong(args[2]);
  const bool on_device = nargs < 4 || PyObject_IsTrue(args[3]) == 1;
  const long long cap = nargs < 5 ? -1 : PyLong_AsLongLong(args[4]);
  if (PyErr_Occurred()) {
    Py_DECREF(seq);
    return nullptr;
  }
  int64_t* ptrs = reinterpret_cast<int64_t*>(pa);
  int64_t* numels = reinterpret_cast<int64_t*>(na);
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  if (cap >= 0 && n != cap) {  // (a sequence whose len() and items disagree: never past the arrays)
    Py_DECREF(seq);
    Py_RETURN_NONE;
  }
  PyObject** items = PySequence_Fast_ITEMS(seq);
  int st = -1, dev = -1;
  uint64_t h = 1469598103934665603ull;
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject* o = items[i];
    if (!THPVariable_Check(o)) {
      Py_DECREF(seq);
      Py_RETURN_NONE;
    }
    const at::Tensor& t = THPVariable_Unpack(o);
    if (!t.defined() || t.layout() != c10::kStrided || !(on_device ? t.is_cuda() : t.is_cpu()) || !t.is_contiguous()) {
      Py_DECREF(seq);
      Py_RETURN_NONE;
    }
    const int s = (int)t.scalar_type();
    const int d = (int)t.get_device();
    if (i == 0) {
      st = s;
      dev = d;
    } else if (s != st || d != dev) {
      Py_DECREF(seq);
      Py_RETURN_NONE;
    }
    ptrs[i] = reinterpret_cast<int64_t>(t.data_ptr());
    numels[i] = t.numel();
    const auto sz = t.sizes();
    h = fnv(h, (uint64_t)sz.size());
    for (int64_t v : sz) h = fnv(h, (uint64_t)v);
  }
  Py_DECREF(seq);
  return Py_BuildValue("(iiK)", st, dev, (unsigned long long)h);
}

PyObject* max_refcount(PyObject*, PyObject* arg) {
  PyObject* seq = PySequence_Fast(arg, "max_refcount: a sequence");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject** items = PySequence_Fast_ITEMS(seq);
  Py_ssize_t m = 0;
  for (Py_ssize_t i = 0; i < n; i++)
    if (Py_REFCNT(items[i]) > m) m = Py_REFCNT(items[i]);
  Py_DECREF(seq);
  return PyLong_FromSsize_t(m);
}

PyMethodDef kMethods[] = {
    {"dev_list", (PyCFunction)(void (*)(void))dev_list, METH_FASTCALL,
     "dev_list(seq, ptrs_addr, numels_addr[, on_device[, cap]]) -> (scalar_type, device, shape_hash) or None"},
    {"max_refcount", max_refcount, METH_O, "max_refcount(seq) -> the largest reference count of the items"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fast", "tips_amd host-side list helpers", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__fast(void) { return PyModule_Create(&kModule); }
