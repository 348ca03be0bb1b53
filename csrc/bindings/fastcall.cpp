// Direct CPython (METH_FASTCALL) entry points for the per-batch hot ops, bypassing the torch.ops dispatcher.
//
// A metric ``update`` on MI355X is launch-bound for the headline shapes (the 8192 x 1000 bf16 confusion-matrix kernel
// runs in ~5 us), and on the GPU host a boxed ``torch.ops.tm_amd.*`` call costs ~5.5 us of CPU before the kernel is
// even enqueued (IValue boxing of every argument + dispatch-key computation), against ~3.8 us for a trivial ATen op.
// These wrappers unpack the PyObjects straight into at::Tensor / scalars and call the same C++ launchers that the
// dispatcher registrations use (one implementation, two front doors; the torch.ops path remains for TorchScript,
// torch.compile and anything that needs the dispatcher).  Built as ``torchmetrics_amd/_C/_fastcall.so`` linked
// against ``libtm_amd.so``.
#include <Python.h>
#include <torch/csrc/autograd/python_variable.h>

#include <ATen/ATen.h>
#include <c10/util/Optional.h>

#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace tm_amd {
void mc_update(const at::Tensor& preds, const at::Tensor& target, at::Tensor out, at::Tensor flag, int64_t num_classes,
               int64_t ignore_index, bool has_ignore, int64_t mode, bool samplewise);
void mc_stats_finalize(at::Tensor ws, int64_t num_classes, bool micro, bool accumulate, at::Tensor tp, at::Tensor fp,
                       at::Tensor tn, at::Tensor fn);
void bin_update(const at::Tensor& preds, const at::Tensor& target, at::Tensor ws, at::Tensor flag, at::Tensor not_prob,
                int64_t num_labels, double threshold, int64_t ignore_index, bool has_ignore, bool samplewise,
                bool prob_check_all);
void bin_stats_finalize(at::Tensor ws, at::Tensor not_prob, bool accumulate, at::Tensor tp, at::Tensor fp,
                        at::Tensor tn, at::Tensor fn);
void bin_confmat_finalize(at::Tensor ws, at::Tensor not_prob, at::Tensor confmat);
at::Tensor moments_update(const at::Tensor& preds, const at::Tensor& target, int64_t num_outputs, int64_t mask,
                          double eps, double power, const c10::optional<at::Tensor>& shift_p,
                          const c10::optional<at::Tensor>& shift_t, at::TensorList dests, at::IntArrayRef sum_ids,
                          bool want_sums, int64_t fold);
void stat_reduce(const at::Tensor& tp, const at::Tensor& fp, const at::Tensor& tn, const at::Tensor& fn,
                 at::Tensor out, int64_t kind, int64_t average, bool multilabel, double beta);
void launch_probe(at::Tensor flag);
void confmat_reduce(const at::Tensor& confmat, int64_t kind, int64_t average, int64_t ignore, int64_t kw,
                    at::Tensor out);
void calibration_bins(const at::Tensor& conf, const at::Tensor& acc, const at::Tensor& bounds, at::Tensor sums,
                      at::Tensor bad);
void curve_score(const at::Tensor& state, int64_t kind, int64_t average, at::Tensor out, at::Tensor nan_flag);
void calibration_reduce(const at::Tensor& sums, int64_t norm, at::Tensor out);
void calibration_reduce_clear(at::Tensor sums, int64_t norm, at::Tensor out);
void regression_compute(int64_t kind, at::TensorList states, const c10::optional<at::Tensor>& n, double n_value,
                        int64_t multioutput, double bound, at::Tensor out);
void mc_calibration_update(const at::Tensor& preds, const at::Tensor& target, at::Tensor cand, at::Tensor conf,
                           at::Tensor acc, at::Tensor notprob, int64_t slot, at::Tensor flag);
void agg_update(const at::Tensor& x, const at::Tensor& w, double wconst, int64_t kind, int64_t nan_mode,
                double impute, at::Tensor part, at::Tensor ctl, at::Tensor s0, at::Tensor s1, at::Tensor flag);
void exact_match_update(const at::Tensor& preds, const at::Tensor& target, int64_t kind, int64_t C, int64_t P,
                        bool has_c, double threshold, int64_t ignore_index, bool has_ignore, bool samplewise,
                        at::Tensor ws, at::Tensor notprob, at::Tensor correct, at::Tensor total, at::Tensor out);
void group_stats_update(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& groups, int64_t G,
                        double threshold, int64_t ignore_index, bool has_ignore, at::Tensor ws, at::Tensor notprob,
                        at::Tensor tp, at::Tensor fp, at::Tensor tn, at::Tensor fn);
}  // namespace tm_amd

namespace {

void arg_probe(const at::Tensor&, const at::Tensor&, at::Tensor, at::Tensor, int64_t, int64_t, bool, int64_t, bool) {}

// inputs may arrive non-contiguous: make them contiguous here (free when they already are) instead of in Python
void mc_update_fc(const at::Tensor& preds, const at::Tensor& target, at::Tensor out, at::Tensor flag,
                  int64_t num_classes, int64_t ignore_index, bool has_ignore, int64_t mode, bool samplewise) {
  tm_amd::mc_update(preds.contiguous(), target.contiguous(), out, flag, num_classes, ignore_index, has_ignore, mode,
                    samplewise);
}

void bin_update_fc(const at::Tensor& preds, const at::Tensor& target, at::Tensor ws, at::Tensor flag,
                   at::Tensor not_prob, int64_t num_labels, double threshold, int64_t ignore_index, bool has_ignore,
                   bool samplewise, bool prob_check_all) {
  tm_amd::bin_update(preds.contiguous(), target.contiguous(), ws, flag, not_prob, num_labels, threshold, ignore_index,
                     has_ignore, samplewise, prob_check_all);
}

at::Tensor moments_update_fc(const at::Tensor& preds, const at::Tensor& target, int64_t num_outputs, int64_t mask,
                             double eps, double power, const c10::optional<at::Tensor>& shift_p,
                             const c10::optional<at::Tensor>& shift_t, at::TensorList dests, at::IntArrayRef sum_ids,
                             bool want_sums, int64_t fold) {
  return tm_amd::moments_update(preds.contiguous(), target.contiguous(), num_outputs, mask, eps, power, shift_p,
                                shift_t, dests, sum_ids, want_sums, fold);
}

void stat_reduce_fc(const at::Tensor& tp, const at::Tensor& fp, const at::Tensor& tn, const at::Tensor& fn,
                    at::Tensor out, int64_t kind, int64_t average, bool multilabel, double beta) {
  tm_amd::stat_reduce(tp.contiguous(), fp.contiguous(), tn.contiguous(), fn.contiguous(), out, kind, average,
                      multilabel, beta);
}

struct ArgError {
  int index;
  const char* what;
};

// ---------------------------------------------------------------------------------------------- argument decoding
template <typename T>
struct Arg;

template <>
struct Arg<at::Tensor> {
  using holder = at::Tensor;
  static holder get(PyObject* o, int i) {
    if (!THPVariable_Check(o)) throw ArgError{i, "expected a Tensor"};
    return THPVariable_Unpack(o);
  }
  static const at::Tensor& pass(const holder& h) { return h; }
};

template <>
struct Arg<c10::optional<at::Tensor>> {
  using holder = c10::optional<at::Tensor>;
  static holder get(PyObject* o, int i) {
    if (o == Py_None) return c10::nullopt;
    return Arg<at::Tensor>::get(o, i);
  }
  static const holder& pass(const holder& h) { return h; }
};

template <>
struct Arg<int64_t> {
  using holder = int64_t;
  static holder get(PyObject* o, int i) {
    const long long v = PyLong_AsLongLong(o);
    if (v == -1 && PyErr_Occurred()) throw ArgError{i, "expected an int"};
    return v;
  }
  static holder pass(holder h) { return h; }
};

template <>
struct Arg<double> {
  using holder = double;
  static holder get(PyObject* o, int i) {
    const double v = PyFloat_AsDouble(o);
    if (v == -1.0 && PyErr_Occurred()) throw ArgError{i, "expected a float"};
    return v;
  }
  static holder pass(holder h) { return h; }
};

template <>
struct Arg<bool> {
  using holder = bool;
  static holder get(PyObject* o, int i) {
    const int v = PyObject_IsTrue(o);
    if (v < 0) throw ArgError{i, "expected a bool"};
    return v != 0;
  }
  static holder pass(holder h) { return h; }
};

template <>
struct Arg<at::TensorList> {
  using holder = std::vector<at::Tensor>;
  static holder get(PyObject* o, int i) {
    if (!PyList_Check(o) && !PyTuple_Check(o)) throw ArgError{i, "expected a list of Tensors"};
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(o);
    PyObject** items = PySequence_Fast_ITEMS(o);
    holder v;
    v.reserve(n);
    for (Py_ssize_t k = 0; k < n; ++k) v.push_back(Arg<at::Tensor>::get(items[k], i));
    return v;
  }
  static at::TensorList pass(const holder& h) { return at::TensorList(h); }
};

template <>
struct Arg<at::IntArrayRef> {
  using holder = std::vector<int64_t>;
  static holder get(PyObject* o, int i) {
    if (!PyList_Check(o) && !PyTuple_Check(o)) throw ArgError{i, "expected a list of ints"};
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(o);
    PyObject** items = PySequence_Fast_ITEMS(o);
    holder v(n);
    for (Py_ssize_t k = 0; k < n; ++k) v[k] = Arg<int64_t>::get(items[k], i);
    return v;
  }
  static at::IntArrayRef pass(const holder& h) { return at::IntArrayRef(h); }
};

template <typename T>
using arg_t = Arg<std::remove_cv_t<std::remove_reference_t<T>>>;

template <typename R>
PyObject* wrap_result(R&& r) {
  return THPVariable_Wrap(std::forward<R>(r));
}

template <typename R, typename... A, size_t... I>
PyObject* invoke(R (*fn)(A...), PyObject* const* args, std::index_sequence<I...>) {
  std::tuple<typename arg_t<A>::holder...> held{arg_t<A>::get(args[I], static_cast<int>(I))...};
  if constexpr (std::is_void_v<R>) {
    fn(arg_t<A>::pass(std::get<I>(held))...);
    Py_RETURN_NONE;
  } else {
    return wrap_result(fn(arg_t<A>::pass(std::get<I>(held))...));
  }
}

template <auto Fn>
struct FastCall;

template <typename R, typename... A, R (*Fn)(A...)>
struct FastCall<Fn> {
  static PyObject* call(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != static_cast<Py_ssize_t>(sizeof...(A))) {
      PyErr_Format(PyExc_TypeError, "expected %d arguments, got %zd", static_cast<int>(sizeof...(A)), nargs);
      return nullptr;
    }
    try {
      return invoke(Fn, args, std::index_sequence_for<A...>{});
    } catch (const ArgError& e) {
      if (!PyErr_Occurred()) PyErr_Format(PyExc_TypeError, "argument %d: %s", e.index, e.what);
      return nullptr;
    } catch (const c10::Error& e) {
      PyErr_SetString(PyExc_RuntimeError, e.what_without_backtrace());
      return nullptr;
    } catch (const std::exception& e) {
      PyErr_SetString(PyExc_RuntimeError, e.what());
      return nullptr;
    }
  }
};

#define TM_FAST(name, fn) \
  { name, reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&FastCall<&fn>::call)), METH_FASTCALL, nullptr }

PyMethodDef kMethods[] = {
    TM_FAST("mc_update", mc_update_fc),
    TM_FAST("mc_stats_finalize", tm_amd::mc_stats_finalize),
    TM_FAST("bin_update", bin_update_fc),
    TM_FAST("bin_stats_finalize", tm_amd::bin_stats_finalize),
    TM_FAST("bin_confmat_finalize", tm_amd::bin_confmat_finalize),
    TM_FAST("moments_update", moments_update_fc),
    TM_FAST("stat_reduce", stat_reduce_fc),
    TM_FAST("launch_probe", tm_amd::launch_probe),
    TM_FAST("confmat_reduce", tm_amd::confmat_reduce),
    TM_FAST("calibration_bins", tm_amd::calibration_bins),
    TM_FAST("calibration_reduce", tm_amd::calibration_reduce),
    TM_FAST("calibration_reduce_clear", tm_amd::calibration_reduce_clear),
    TM_FAST("curve_score", tm_amd::curve_score),
    TM_FAST("regression_compute", tm_amd::regression_compute),
    TM_FAST("mc_calibration_update", tm_amd::mc_calibration_update),
    TM_FAST("agg_update", tm_amd::agg_update),
    TM_FAST("exact_match_update", tm_amd::exact_match_update),
    TM_FAST("group_stats_update", tm_amd::group_stats_update),
    TM_FAST("arg_probe", arg_probe),
    {nullptr, nullptr, 0, nullptr},
};

// ------------------------------------------------------------------------------------------ native metric update
// ``MulticlassConfusionMatrix.update`` as ONE native callable (installed as the instance's ``update``): the shape /
// dtype / device checks of the reference's tensor validation (F/classification/stat_scores.py:281-319), the metric's
// bookkeeping through its ``__dict__`` (``_update_count``, ``_computed``: what Metric._wrap_update does,
// S/metric.py:459-481) and the kernel launch, with no Python frame in between.  Anything off the fast path -- CPU or
// non-contiguous inputs, other ranks of input, a state not on the input's device, kwargs, ``compute_on_cpu`` -- goes to
// the regular Python ``update`` (``fallback``), which raises the reference's exceptions.
PyObject* g_k_confmat = nullptr;
PyObject* g_k_err = nullptr;
PyObject* g_k_count = nullptr;
PyObject* g_k_computed = nullptr;
PyObject* g_k_cpu = nullptr;
PyObject* g_k_classes = nullptr;
PyObject* g_k_ignore = nullptr;
PyObject* g_k_validate = nullptr;

struct NativeUpdate {
  PyObject_HEAD
  vectorcallfunc vectorcall;
  PyObject* state;     // the metric's __dict__
  PyObject* fallback;  // the Python update (Metric._wrap_update wrapper)
  at::Tensor* sink;    // flag word for validate_args=False (kernels always have somewhere to report)
  int64_t calls;       // fast-path calls (tests / benchmarks read it)
};

inline const at::Tensor* tensor_item(PyObject* dict, PyObject* key) {
  PyObject* o = PyDict_GetItem(dict, key);  // borrowed
  if (o == nullptr || !THPVariable_Check(o)) return nullptr;
  return &THPVariable_Unpack(o);
}

// 1 = done, 0 = not handled (take the Python path), -1 = Python error set
int confmat_fast(NativeUpdate* self, PyObject* a, PyObject* b) {
  if (!THPVariable_Check(a) || !THPVariable_Check(b)) return 0;
  const at::Tensor& p = THPVariable_Unpack(a);
  const at::Tensor& t = THPVariable_Unpack(b);
  if (!p.is_cuda() || !t.is_cuda()) return 0;
  const auto pd = p.scalar_type();
  const auto td = t.scalar_type();
  if (pd != at::kBFloat16 && pd != at::kHalf && pd != at::kFloat) return 0;
  if (td != at::kLong && td != at::kInt) return 0;
  PyObject* st = self->state;
  PyObject* co = PyDict_GetItem(st, g_k_classes);
  if (co == nullptr || !PyLong_CheckExact(co)) return 0;
  const long long C = PyLong_AsLongLong(co);
  if (p.dim() != 2 || t.dim() != 1 || p.size(1) != C || p.size(0) != t.size(0) || p.size(0) == 0) return 0;
  if (!p.is_contiguous() || !t.is_contiguous()) return 0;
  const int dev = p.get_device();
  if (t.get_device() != dev) return 0;
  if (PyDict_GetItem(st, g_k_cpu) != Py_False) return 0;
  const at::Tensor* cm = tensor_item(st, g_k_confmat);
  if (cm == nullptr || !cm->is_cuda() || cm->get_device() != dev || cm->scalar_type() != at::kLong ||
      !cm->is_contiguous() || cm->numel() != C * C)
    return 0;
  PyObject* vo = PyDict_GetItem(st, g_k_validate);
  if (vo == nullptr) return 0;
  const bool validate = vo == Py_True;
  const at::Tensor* flag;
  if (validate) {
    flag = tensor_item(st, g_k_err);  // created by the first (Python) update on this device
    if (flag == nullptr || !flag->is_cuda() || flag->get_device() != dev || flag->scalar_type() != at::kInt) return 0;
  } else {
    if (self->sink == nullptr || self->sink->get_device() != dev) {
      delete self->sink;
      self->sink = new at::Tensor(at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev)));
    }
    flag = self->sink;
  }
  PyObject* io = PyDict_GetItem(st, g_k_ignore);
  if (io == nullptr) return 0;
  long long ignore = 0;
  const bool has_ignore = io != Py_None;
  if (has_ignore) {
    if (!PyLong_CheckExact(io)) return 0;
    ignore = PyLong_AsLongLong(io);
  }
  PyObject* cnt = PyDict_GetItem(st, g_k_count);
  if (cnt == nullptr || !PyLong_CheckExact(cnt)) return 0;
  const long long n = PyLong_AsLongLong(cnt);
  try {
    tm_amd::mc_update(p, t, *cm, *flag, C, ignore, has_ignore, 0, false);
  } catch (const c10::Error& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what_without_backtrace());
    return -1;
  }
  PyObject* n1 = PyLong_FromLongLong(n + 1);
  if (n1 == nullptr) return -1;
  const int rc = PyDict_SetItem(st, g_k_count, n1);
  Py_DECREF(n1);
  if (rc != 0 || PyDict_SetItem(st, g_k_computed, Py_None) != 0) return -1;
  ++self->calls;
  return 1;
}

PyObject* native_update_vectorcall(PyObject* o, PyObject* const* args, size_t nargsf, PyObject* kwnames) {
  auto* self = reinterpret_cast<NativeUpdate*>(o);
  const Py_ssize_t nargs = PyVectorcall_NARGS(nargsf);
  if (nargs == 2 && (kwnames == nullptr || PyTuple_GET_SIZE(kwnames) == 0)) {
    const int r = confmat_fast(self, args[0], args[1]);
    if (r == 1) Py_RETURN_NONE;
    if (r < 0) return nullptr;
  }
  return PyObject_Vectorcall(self->fallback, args, nargsf, kwnames);
}

int native_update_traverse(PyObject* o, visitproc visit, void* arg) {
  auto* self = reinterpret_cast<NativeUpdate*>(o);
  Py_VISIT(self->state);
  Py_VISIT(self->fallback);
  return 0;
}

int native_update_clear(PyObject* o) {
  auto* self = reinterpret_cast<NativeUpdate*>(o);
  Py_CLEAR(self->state);
  Py_CLEAR(self->fallback);
  return 0;
}

void native_update_dealloc(PyObject* o) {
  auto* self = reinterpret_cast<NativeUpdate*>(o);
  PyObject_GC_UnTrack(o);
  native_update_clear(o);
  delete self->sink;
  self->sink = nullptr;
  Py_TYPE(o)->tp_free(o);
}

PyObject* native_update_wrapped(PyObject* o, void*) {
  // what the Python wrapper wraps (the bound ``update``): ``is_overridden`` and ``inspect.signature`` unwrap to it
  return PyObject_GetAttrString(reinterpret_cast<NativeUpdate*>(o)->fallback, "__wrapped__");
}

PyObject* native_update_fallback(PyObject* o, void*) {
  PyObject* f = reinterpret_cast<NativeUpdate*>(o)->fallback;
  Py_INCREF(f);
  return f;
}

PyObject* native_update_calls(PyObject* o, void*) {
  return PyLong_FromLongLong(reinterpret_cast<NativeUpdate*>(o)->calls);
}

PyGetSetDef kNativeUpdateGetSet[] = {
    {"__wrapped__", native_update_wrapped, nullptr, nullptr, nullptr},
    {"fallback", native_update_fallback, nullptr, nullptr, nullptr},
    {"native_calls", native_update_calls, nullptr, nullptr, nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr},
};

PyTypeObject NativeUpdateType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// confmat_updater(state_dict, fallback) -> callable
PyObject* make_confmat_updater(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyDict_Check(args[0]) || !PyCallable_Check(args[1])) {
    PyErr_SetString(PyExc_TypeError, "confmat_updater(state: dict, fallback: callable)");
    return nullptr;
  }
  auto* self = PyObject_GC_New(NativeUpdate, &NativeUpdateType);
  if (self == nullptr) return nullptr;
  self->vectorcall = native_update_vectorcall;
  Py_INCREF(args[0]);
  self->state = args[0];
  Py_INCREF(args[1]);
  self->fallback = args[1];
  self->sink = nullptr;
  self->calls = 0;
  PyObject_GC_Track(reinterpret_cast<PyObject*>(self));
  return reinterpret_cast<PyObject*>(self);
}

PyMethodDef kFactoryMethods[] = {
    {"confmat_updater", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&make_confmat_updater)),
     METH_FASTCALL, "native MulticlassConfusionMatrix.update bound to a metric's __dict__"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fastcall", "dispatcher-free entry points of libtm_amd", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__fastcall() {
  NativeUpdateType.tp_name = "torchmetrics_amd._C._fastcall.NativeUpdate";
  NativeUpdateType.tp_basicsize = sizeof(NativeUpdate);
  NativeUpdateType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC | Py_TPFLAGS_HAVE_VECTORCALL;
  NativeUpdateType.tp_vectorcall_offset = offsetof(NativeUpdate, vectorcall);
  NativeUpdateType.tp_call = PyVectorcall_Call;
  NativeUpdateType.tp_traverse = native_update_traverse;
  NativeUpdateType.tp_clear = native_update_clear;
  NativeUpdateType.tp_dealloc = native_update_dealloc;
  NativeUpdateType.tp_getset = kNativeUpdateGetSet;
  NativeUpdateType.tp_doc = "native metric update (see csrc/bindings/fastcall.cpp)";
  if (PyType_Ready(&NativeUpdateType) < 0) return nullptr;
  g_k_confmat = PyUnicode_InternFromString("confmat");
  g_k_err = PyUnicode_InternFromString("_device_errors");
  g_k_count = PyUnicode_InternFromString("_update_count");
  g_k_computed = PyUnicode_InternFromString("_computed");
  g_k_cpu = PyUnicode_InternFromString("compute_on_cpu");
  g_k_classes = PyUnicode_InternFromString("num_classes");
  g_k_ignore = PyUnicode_InternFromString("ignore_index");
  g_k_validate = PyUnicode_InternFromString("validate_args");
  PyObject* m = PyModule_Create(&kModule);
  if (m == nullptr) return nullptr;
  if (PyModule_AddFunctions(m, kFactoryMethods) < 0) return nullptr;
  return m;
}
