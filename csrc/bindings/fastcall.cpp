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

#include "../common/pack.h"
#include <c10/util/Optional.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <string>
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
int64_t read_word_sync(const at::Tensor& word);
std::vector<int64_t> read_words(const at::Tensor& words, const at::Tensor& anchor, int64_t spin_us);
bool mc_stats_direct(const at::Tensor& preds, const at::Tensor& target, at::Tensor tp, at::Tensor fp, at::Tensor tn,
                     at::Tensor fn, at::Tensor flag, int64_t num_classes);
void mc_family_update(const at::Tensor& preds, const at::Tensor& target, at::TensorList cm, at::TensorList st,
                      at::IntArrayRef st_micro, const at::Tensor& curve, const at::Tensor& thr_sorted,
                      const at::Tensor& perm, const at::Tensor& conf, const at::Tensor& acc, const at::Tensor& bounds,
                      const at::Tensor& bins, at::TensorList err, at::Tensor work, int64_t slot, at::Tensor cand);
void zero_async(at::Tensor t);
bool mc_confmat_dual(const at::Tensor& preds, const at::Tensor& target, at::Tensor batch, at::Tensor global,
                     at::Tensor flag, int64_t num_classes, int64_t ignore_index, bool has_ignore);
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
void mc_stats_forward(at::Tensor ws, int64_t num_classes, bool micro, at::Tensor tp, at::Tensor fp, at::Tensor tn,
                      at::Tensor fn, int64_t kind, int64_t average, double beta, at::Tensor out);
void bin_stats_forward(at::Tensor ws, at::Tensor not_prob, at::Tensor tp, at::Tensor fp, at::Tensor tn, at::Tensor fn,
                       int64_t kind, int64_t average, double beta, at::Tensor out);
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
    TM_FAST("mc_stats_forward", tm_amd::mc_stats_forward),
    TM_FAST("bin_stats_forward", tm_amd::bin_stats_forward),
    TM_FAST("arg_probe", arg_probe),
    TM_FAST("mc_family_update", tm_amd::mc_family_update),
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

struct NativeUpdate;
// 1 = handled (*result: a new reference), 0 = not handled (take the Python path), -1 = Python error set
using FastFn = int (*)(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** result);

struct NativeUpdate {
  PyObject_HEAD
  vectorcallfunc vectorcall;
  PyObject* state;     // the metric's __dict__
  PyObject* fallback;  // the Python update (Metric._wrap_update wrapper) / forward (bound Metric.forward)
  at::Tensor* sink;    // flag word for validate_args=False (kernels always have somewhere to report)
  int64_t calls;       // fast-path calls (tests / benchmarks read it)
  FastFn fast;         // the native body
  int stat_kind;       // NativeForward of the stat-score family: the score (cbody::StatKind)
  int decline;         // source line of the last fast-path decline (0: none yet) -- ``decline_line`` for diagnostics
  char range_name[120];  // roctx range of the native call ("tm.update/<Metric>"); "" = no range
};

// ---------------------------------------------------------------------------------------------- roctx ranges
// Profiler ranges on the PRODUCTION path: with ranges on (``profiling.enable()`` /
// TORCHMETRICS_AMD_ROCTX=1 -> set_ranges(True)), every native update / forward opens "tm.update/<Metric>" /
// "tm.forward/<Metric>" around its checks and kernel launch, so rocprofv3 --marker-trace shows the launch inside the
// range while the fast path stays the one that runs.  The roctx library is opened on first use (rocprofiler-sdk's,
// which rocprofv3 intercepts, else the legacy libroctx64); no library -> no ranges.  Off: one branch on a global.
using RoctxPush = int (*)(const char*);
using RoctxPop = int (*)();
RoctxPush g_roctx_push = nullptr;
RoctxPop g_roctx_pop = nullptr;
bool g_ranges_on = false;

bool bind_roctx() {
  if (g_roctx_push != nullptr) return true;
  for (const char* lib : {"librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                          "/opt/rocm/lib/libroctx64.so"}) {
    void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) continue;
    auto push = reinterpret_cast<RoctxPush>(dlsym(h, "roctxRangePushA"));
    auto pop = reinterpret_cast<RoctxPop>(dlsym(h, "roctxRangePop"));
    if (push != nullptr && pop != nullptr) {
      g_roctx_push = push;
      g_roctx_pop = pop;
      return true;
    }
  }
  return false;
}

struct RangeScope {  // one roctx range for the lifetime of the scope (nothing when ranges are off / unnamed)
  bool on;
  explicit RangeScope(const NativeUpdate* self) : on(g_ranges_on && self->range_name[0] != '\0') {
    if (on) g_roctx_push(self->range_name);
  }
  ~RangeScope() {
    if (on) g_roctx_pop();
  }
};

// set_ranges(on: bool) -> bool: turn the native ranges on / off; returns whether they are on (False: no roctx library)
PyObject* set_ranges(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 1) {
    PyErr_SetString(PyExc_TypeError, "set_ranges(on: bool)");
    return nullptr;
  }
  const int on = PyObject_IsTrue(args[0]);
  if (on < 0) return nullptr;
  g_ranges_on = on && bind_roctx();
  return PyBool_FromLong(g_ranges_on);
}

// leave the fast path, remembering where (NativeUpdate.decline_line names the check that sent a call to Python)
#define TM_DECLINE        \
  do {                    \
    self->decline = __LINE__; \
    return 0;             \
  } while (0)

inline const at::Tensor* tensor_item(PyObject* dict, PyObject* key) {
  PyObject* o = PyDict_GetItem(dict, key);  // borrowed
  if (o == nullptr || !THPVariable_Check(o)) return nullptr;
  return &THPVariable_Unpack(o);
}

// 1 = done, 0 = not handled (take the Python path), -1 = Python error set
int confmat_fast(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** result) {
  if (!THPVariable_Check(a) || !THPVariable_Check(b)) TM_DECLINE;
  const at::Tensor& p = THPVariable_Unpack(a);
  const at::Tensor& t = THPVariable_Unpack(b);
  if (!p.is_cuda() || !t.is_cuda()) TM_DECLINE;
  const auto pd = p.scalar_type();
  const auto td = t.scalar_type();
  if (pd != at::kBFloat16 && pd != at::kHalf && pd != at::kFloat) TM_DECLINE;
  if (td != at::kLong && td != at::kInt) TM_DECLINE;
  PyObject* st = self->state;
  PyObject* co = PyDict_GetItem(st, g_k_classes);
  if (co == nullptr || !PyLong_CheckExact(co)) TM_DECLINE;
  const long long C = PyLong_AsLongLong(co);
  if (p.dim() != 2 || t.dim() != 1 || p.size(1) != C || p.size(0) != t.size(0) || p.size(0) == 0) TM_DECLINE;
  if (!p.is_contiguous() || !t.is_contiguous()) TM_DECLINE;
  const int dev = p.get_device();
  if (t.get_device() != dev) TM_DECLINE;
  if (PyDict_GetItem(st, g_k_cpu) != Py_False) TM_DECLINE;
  const at::Tensor* cm = tensor_item(st, g_k_confmat);
  if (cm == nullptr || !cm->is_cuda() || cm->get_device() != dev || cm->scalar_type() != at::kLong ||
      !cm->is_contiguous() || cm->numel() != C * C)
    TM_DECLINE;
  PyObject* vo = PyDict_GetItem(st, g_k_validate);
  if (vo == nullptr) TM_DECLINE;
  const bool validate = vo == Py_True;
  const at::Tensor* flag;
  if (validate) {
    flag = tensor_item(st, g_k_err);  // created by the first (Python) update on this device
    if (flag == nullptr || !flag->is_cuda() || flag->get_device() != dev || flag->scalar_type() != at::kInt) TM_DECLINE;
  } else {
    if (self->sink == nullptr || self->sink->get_device() != dev) {
      delete self->sink;
      self->sink = new at::Tensor(at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev)));
    }
    flag = self->sink;
  }
  PyObject* io = PyDict_GetItem(st, g_k_ignore);
  if (io == nullptr) TM_DECLINE;
  long long ignore = 0;
  const bool has_ignore = io != Py_None;
  if (has_ignore) {
    if (!PyLong_CheckExact(io)) TM_DECLINE;
    ignore = PyLong_AsLongLong(io);
  }
  PyObject* cnt = PyDict_GetItem(st, g_k_count);
  if (cnt == nullptr || !PyLong_CheckExact(cnt)) TM_DECLINE;
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
  Py_INCREF(Py_None);
  *result = Py_None;
  return 1;
}

PyObject* native_update_vectorcall(PyObject* o, PyObject* const* args, size_t nargsf, PyObject* kwnames) {
  auto* self = reinterpret_cast<NativeUpdate*>(o);
  const Py_ssize_t nargs = PyVectorcall_NARGS(nargsf);
  if (nargs == 2 && (kwnames == nullptr || PyTuple_GET_SIZE(kwnames) == 0)) {
    PyObject* result = nullptr;
    int r;
    {
      RangeScope range(self);  // (a declined call's Python path opens its own range)
      r = self->fast(self, args[0], args[1], &result);
    }
    if (r == 1) return result;
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

PyObject* native_update_decline(PyObject* o, void*) {
  return PyLong_FromLong(reinterpret_cast<NativeUpdate*>(o)->decline);
}

PyObject* native_update_range_get(PyObject* o, void*) {
  return PyUnicode_FromString(reinterpret_cast<NativeUpdate*>(o)->range_name);
}

int native_update_range_set(PyObject* o, PyObject* v, void*) {
  if (v == nullptr || !PyUnicode_Check(v)) {
    PyErr_SetString(PyExc_TypeError, "range_name must be a str");
    return -1;
  }
  Py_ssize_t n = 0;
  const char* c = PyUnicode_AsUTF8AndSize(v, &n);
  if (c == nullptr) return -1;
  auto* self = reinterpret_cast<NativeUpdate*>(o);
  const size_t k = std::min<size_t>(static_cast<size_t>(n), sizeof(self->range_name) - 1);
  std::memcpy(self->range_name, c, k);
  self->range_name[k] = '\0';
  return 0;
}

PyObject* native_update_calls(PyObject* o, void*) {
  return PyLong_FromLongLong(reinterpret_cast<NativeUpdate*>(o)->calls);
}

PyGetSetDef kNativeUpdateGetSet[] = {
    {"__wrapped__", native_update_wrapped, nullptr, nullptr, nullptr},
    {"fallback", native_update_fallback, nullptr, nullptr, nullptr},
    {"native_calls", native_update_calls, nullptr, nullptr, nullptr},
    {"decline_line", native_update_decline, nullptr, nullptr, nullptr},
    {"range_name", native_update_range_get, native_update_range_set, nullptr, nullptr},
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
  self->decline = 0;
  self->range_name[0] = '\0';
  self->fast = confmat_fast;
  self->stat_kind = 0;
  PyObject_GC_Track(reinterpret_cast<PyObject*>(self));
  return reinterpret_cast<PyObject*>(self);
}

// ----------------------------------------------------------------------------------------- native metric forward
// ``metric(preds, target)`` for the confusion-matrix and stat-score families as ONE native callable (installed as the
// instance's ``forward``; nn.Module.__call__ dispatches to it).  The reference forward (S/metric.py:275-306,353-391)
// saves the global state, resets, updates, computes the batch value and merges state by state; here it is
//   confmat:     zeros(C, C) -> one kernel adding every row into it and into the global matrix (16-bit logits; else
//                mc_update into it -> global += batch); the batch matrix is the value,
//   stat scores: the update kernel into the per-metric workspace -> ONE fused launch (classification/forward.hip)
//                that folds the batch counts into the global states and scores the batch with compute()'s own body,
// plus the bookkeeping of Metric.forward (``_update_count``, ``_computed``, ``_forward_cache``).  Taken only when the
// result is the reference's: no dist_sync_on_step, not synced, no compute_on_cpu, and global states that nothing
// outside the metric can observe (the reference merges out of place, so a held state / view must not change: the
// same Python-refcount + storage-use-count test as Metric._merge_sums_in_place).  Everything else -> Metric.forward.
// Deviation (as for update on ROCm): value-range errors of the batch surface at the next compute(), not in forward.
PyObject* g_k_tp = nullptr;
PyObject* g_k_fp = nullptr;
PyObject* g_k_tn = nullptr;
PyObject* g_k_fn = nullptr;
PyObject* g_k_wsobj = nullptr;
PyObject* g_k_ws = nullptr;
PyObject* g_k_notprob = nullptr;
PyObject* g_k_topk = nullptr;
PyObject* g_k_mdavg = nullptr;
PyObject* g_k_average = nullptr;
PyObject* g_k_micro = nullptr;
PyObject* g_k_labels = nullptr;
PyObject* g_k_threshold = nullptr;
PyObject* g_k_beta = nullptr;
PyObject* g_k_synced = nullptr;
PyObject* g_k_dsos = nullptr;
PyObject* g_k_fcache = nullptr;
PyObject* g_k_defaults = nullptr;
PyObject* g_k_normalize = nullptr;

enum FwdKind : int { kFwdConfmat = 0, kFwdMulticlass = 1, kFwdBinary = 2, kFwdMultilabel = 3 };

// the batch-mode preconditions of Metric.forward's reduce-state path
bool forward_allowed(PyObject* st) {
  return PyDict_GetItem(st, g_k_synced) == Py_False && PyDict_GetItem(st, g_k_dsos) == Py_False &&
         PyDict_GetItem(st, g_k_cpu) == Py_False;
}

// No reference to the state tensors outside the metric: each state object is held by the metric's __dict__ only, and
// its storage by nothing but the metric's own states on it and their view base (a packed arena's buffer).
// why (optional): 1 no _defaults, 2 a state missing / not a tensor, 3 a Python reference besides the dict (detail: the
// refcount), 4 no storage, 5 more than 16 tensors on the storage, 6 other tensors on the storage (detail: use count
// * 100 + allowed), 7 the view base held from Python (detail: its refcount), 8 a free-threaded CPython build
template <typename Keys>
bool states_unobserved_why(PyObject* st, const Keys& keys, int* why, long long* detail) {
  auto fail = [&](int w, long long d) {
    if (why != nullptr) *why = w;
    if (detail != nullptr) *detail = d;
    return false;
  };
#ifdef Py_GIL_DISABLED
  // free-threaded CPython: biased reference counts make Py_REFCNT an approximation of the owners, not an exact count
  // (8): never merge in place there -- the reference's out-of-place forward runs instead
  return fail(8, 0);
#endif
  PyObject* defaults = PyDict_GetItem(st, g_k_defaults);
  if (defaults == nullptr || !PyDict_Check(defaults)) return fail(1, 0);
  for (PyObject* key : keys) {
    PyObject* o = PyDict_GetItem(st, key);
    if (o == nullptr || !THPVariable_Check(o)) return fail(2, 0);
    if (Py_REFCNT(o) != 1) return fail(3, Py_REFCNT(o));
    const at::Tensor& t = THPVariable_Unpack(o);
    if (!t.has_storage()) return fail(4, 0);
    const c10::StorageImpl* si = t.storage().unsafeGetStorageImpl();
    const c10::TensorImpl* impls[16];
    size_t n = 0;
    auto add = [&](const c10::TensorImpl* p) {
      for (size_t i = 0; i < n; ++i)
        if (impls[i] == p) return true;
      if (n == 16) return false;
      impls[n++] = p;
      return true;
    };
    PyObject *k, *v;
    Py_ssize_t pos = 0;
    while (PyDict_Next(defaults, &pos, &k, &v)) {
      PyObject* so = PyDict_GetItem(st, k);
      if (so == nullptr || !THPVariable_Check(so)) continue;
      const at::Tensor& s = THPVariable_Unpack(so);
      if (!s.has_storage() || s.storage().unsafeGetStorageImpl() != si) continue;
      if (!add(s.unsafeGetTensorImpl())) return fail(5, 0);
      if (s.is_view()) {
        const c10::TensorImpl* bi = s._base().unsafeGetTensorImpl();
        if (!add(bi)) return fail(5, 0);
        // the view base (a packed arena's buffer) as a Python object: alive only through its views (one reference
        // held for them), unless someone outside holds it
        PyObject* bp = bi->pyobj_slot()->load_pyobj();
        if (bp != nullptr && Py_REFCNT(bp) > 1) return fail(7, Py_REFCNT(bp));
      }
    }
    // a Python UntypedStorage object of this storage, once created (untyped_storage(): the arena, the sync engine),
    // is preserved by the StorageImpl for its lifetime and holds one reference of its own
    if (si->pyobj_slot()->load_pyobj() != nullptr) ++n;
    if (static_cast<size_t>(t.storage().use_count()) > n) return fail(6, t.storage().use_count() * 100 + n);
  }
  return true;
}

bool states_unobserved(PyObject* st, std::initializer_list<PyObject*> keys) {
  return states_unobserved_why(st, keys, nullptr, nullptr);
}

// _sole_ref(d: dict, key) -> bool: d[key] is a Tensor whose Python object nothing but `d` references.  Read from C with
// the object fetched from the dict (borrowed), the count is exactly the strong references to the object -- no
// argument / local-variable / interpreter-version convention enters it (sys.getrefcount counts its own argument and
// the caller's locals, and CPython changes what the eval stack holds across versions).  The metric's reset() and
// forward() ask this BEFORE binding the tensor to a local.
PyObject* sole_ref(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyDict_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "_sole_ref(d: dict, key)");
    return nullptr;
  }
  PyObject* o = PyDict_GetItemWithError(args[0], args[1]);  // borrowed
  if (o == nullptr) {
    if (PyErr_Occurred()) return nullptr;
    Py_RETURN_FALSE;
  }
#ifdef Py_GIL_DISABLED
  Py_RETURN_FALSE;  // (see states_unobserved_why: no exact count on a free-threaded build)
#else
  return PyBool_FromLong(THPVariable_Check(o) && Py_REFCNT(o) == 1);
#endif
}

// _states_unobserved(state_dict, keys) -> (ok, why, detail): the forward's aliasing test on its own (tests, diagnostics)
PyObject* states_unobserved_probe(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyDict_Check(args[0]) || !PyTuple_Check(args[1])) {
    PyErr_SetString(PyExc_TypeError, "_states_unobserved(state: dict, keys: tuple)");
    return nullptr;
  }
  std::vector<PyObject*> keys;
  for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(args[1]); ++i) keys.push_back(PyTuple_GET_ITEM(args[1], i));
  int why = 0;
  long long detail = 0;
  const bool ok = states_unobserved_why(args[0], keys, &why, &detail);
  return Py_BuildValue("(OiL)", ok ? Py_True : Py_False, why, detail);
}

// the int32 flag word the kernels report into: the metric's validation word (validate_args) or a private sink
const at::Tensor* forward_flag(NativeUpdate* self, PyObject* st, int dev) {
  PyObject* vo = PyDict_GetItem(st, g_k_validate);
  if (vo == nullptr) return nullptr;
  if (vo == Py_True) {
    const at::Tensor* flag = tensor_item(st, g_k_err);  // created by the first (Python) update on this device
    if (flag == nullptr || !flag->is_cuda() || flag->get_device() != dev || flag->scalar_type() != at::kInt)
      return nullptr;
    return flag;
  }
  if (self->sink == nullptr || self->sink->get_device() != dev) {
    delete self->sink;
    self->sink = new at::Tensor(at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev)));
  }
  return self->sink;
}

bool read_ignore(PyObject* st, long long& ignore, bool& has_ignore) {
  PyObject* io = PyDict_GetItem(st, g_k_ignore);
  if (io == nullptr) return false;
  has_ignore = io != Py_None;
  ignore = 0;
  if (has_ignore) {
    if (!PyLong_CheckExact(io)) return false;
    ignore = PyLong_AsLongLong(io);
  }
  return true;
}

// average string -> cbody::StatAvg (micro 0, macro 1, weighted 2, none 3); -1 = not a fused average
int read_average(PyObject* st) {
  PyObject* a = PyDict_GetItem(st, g_k_average);
  if (a == nullptr) return -1;
  if (a == Py_None) return 3;
  if (!PyUnicode_Check(a)) return -1;
  if (PyUnicode_CompareWithASCIIString(a, "micro") == 0) return 0;
  if (PyUnicode_CompareWithASCIIString(a, "macro") == 0) return 1;
  if (PyUnicode_CompareWithASCIIString(a, "weighted") == 0) return 2;
  if (PyUnicode_CompareWithASCIIString(a, "none") == 0) return 3;
  return -1;
}

const at::Tensor* state_tensor(PyObject* st, PyObject* key, int dev, long long numel) {
  const at::Tensor* t = tensor_item(st, key);
  if (t == nullptr || !t->is_cuda() || t->get_device() != dev || t->scalar_type() != at::kLong ||
      !t->is_contiguous() || t->numel() != numel)
    return nullptr;
  return t;
}

// the metric's _StatWorkspace buffers (created by its first Python update)
bool workspace(PyObject* st, int dev, long long numel, at::Tensor& ws, at::Tensor* not_prob) {
  PyObject* wo = PyDict_GetItem(st, g_k_wsobj);
  if (wo == nullptr) return false;
  PyObject* w = PyObject_GetAttr(wo, g_k_ws);
  if (w == nullptr) {
    PyErr_Clear();
    return false;
  }
  bool ok = THPVariable_Check(w);
  if (ok) {
    ws = THPVariable_Unpack(w);
    ok = ws.is_cuda() && ws.get_device() == dev && ws.scalar_type() == at::kLong && ws.is_contiguous() &&
         ws.numel() == numel;
  }
  Py_DECREF(w);
  if (ok && not_prob != nullptr) {
    PyObject* np = PyObject_GetAttr(wo, g_k_notprob);
    if (np == nullptr) {
      PyErr_Clear();
      return false;
    }
    ok = THPVariable_Check(np);
    if (ok) {
      *not_prob = THPVariable_Unpack(np);
      ok = not_prob->is_cuda() && not_prob->get_device() == dev && not_prob->scalar_type() == at::kInt;
    }
    Py_DECREF(np);
  }
  return ok;
}

int forward_bookkeeping(NativeUpdate* self, PyObject* st, const at::Tensor& value, PyObject** result) {
  PyObject* cnt = PyDict_GetItem(st, g_k_count);
  if (cnt == nullptr || !PyLong_CheckExact(cnt)) return -1;
  const long long n = PyLong_AsLongLong(cnt);
  PyObject* out = THPVariable_Wrap(value);
  if (out == nullptr) return -1;
  PyObject* n1 = PyLong_FromLongLong(n + 1);
  if (n1 == nullptr || PyDict_SetItem(st, g_k_count, n1) != 0 || PyDict_SetItem(st, g_k_fcache, out) != 0) {
    Py_XDECREF(n1);
    Py_DECREF(out);
    return -1;
  }
  Py_DECREF(n1);
  ++self->calls;
  *result = out;
  return 1;
}

bool float_preds(const at::Tensor& p) {
  const auto d = p.scalar_type();
  return d == at::kBFloat16 || d == at::kHalf || d == at::kFloat;
}

bool int_target(const at::Tensor& t) {
  const auto d = t.scalar_type();
  return d == at::kLong || d == at::kInt;
}

int confmat_forward(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** result) {
  if (!THPVariable_Check(a) || !THPVariable_Check(b)) TM_DECLINE;
  const at::Tensor& p = THPVariable_Unpack(a);
  const at::Tensor& t = THPVariable_Unpack(b);
  if (!p.is_cuda() || !t.is_cuda() || !float_preds(p) || !int_target(t)) TM_DECLINE;
  PyObject* st = self->state;
  if (!forward_allowed(st) || PyDict_GetItem(st, g_k_normalize) != Py_None) TM_DECLINE;
  PyObject* co = PyDict_GetItem(st, g_k_classes);
  if (co == nullptr || !PyLong_CheckExact(co)) TM_DECLINE;
  const long long C = PyLong_AsLongLong(co);
  if (p.dim() != 2 || t.dim() != 1 || p.size(1) != C || p.size(0) != t.size(0) || p.size(0) == 0) TM_DECLINE;
  if (!p.is_contiguous() || !t.is_contiguous()) TM_DECLINE;
  const int dev = p.get_device();
  if (t.get_device() != dev) TM_DECLINE;
  // forward() clears the cached compute() value first (a held compute() result of a confusion matrix IS the state)
  if (PyDict_SetItem(st, g_k_computed, Py_None) != 0) return -1;
  const at::Tensor* cm = state_tensor(st, g_k_confmat, dev, C * C);
  if (cm == nullptr || !states_unobserved(st, {g_k_confmat})) TM_DECLINE;
  const at::Tensor* flag = forward_flag(self, st, dev);
  long long ignore;
  bool has_ignore;
  if (flag == nullptr || !read_ignore(st, ignore, has_ignore)) TM_DECLINE;
  at::Tensor batch;
  try {
    batch = at::empty({C, C}, cm->options());
    tm_amd::zero_async(batch);
    // 16-bit logits: one kernel adds each row into the batch matrix and the global state; else update + add
    if (!tm_amd::mc_confmat_dual(p, t, batch, *cm, *flag, C, ignore, has_ignore)) {
      tm_amd::mc_update(p, t, batch, *flag, C, ignore, has_ignore, 0, false);
      cm->add_(batch);
    }
  } catch (const c10::Error& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what_without_backtrace());
    return -1;
  }
  return forward_bookkeeping(self, st, batch, result);
}

// update_only: the family's ``update`` (accumulate the batch into the global states, the reference's in-place
// ``_update_state``) -- the same checks and kernels as the forward below without the batch score.
int stats_forward(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** result, int fkind, bool update_only = false) {
  if (!THPVariable_Check(a) || !THPVariable_Check(b)) TM_DECLINE;
  const at::Tensor& p = THPVariable_Unpack(a);
  const at::Tensor& t = THPVariable_Unpack(b);
  if (!p.is_cuda() || !t.is_cuda() || !float_preds(p) || !int_target(t)) TM_DECLINE;
  if (!p.is_contiguous() || !t.is_contiguous() || p.numel() == 0) TM_DECLINE;
  const int dev = p.get_device();
  if (t.get_device() != dev) TM_DECLINE;
  PyObject* st = self->state;
  if (update_only ? PyDict_GetItem(st, g_k_cpu) != Py_False : !forward_allowed(st)) TM_DECLINE;
  PyObject* md = PyDict_GetItem(st, g_k_mdavg);
  if (md == nullptr || !PyUnicode_Check(md) || PyUnicode_CompareWithASCIIString(md, "global") != 0) TM_DECLINE;
  double beta = 1.0;
  if (self->stat_kind == 5 && !update_only) {
    PyObject* bo = PyDict_GetItem(st, g_k_beta);
    if (bo == nullptr || !PyFloat_Check(bo) && !PyLong_Check(bo)) TM_DECLINE;
    beta = PyFloat_AsDouble(bo);
  }
  long long ignore;
  bool has_ignore;
  if (!read_ignore(st, ignore, has_ignore)) TM_DECLINE;
  long long size;  // classes / labels
  int avg;
  bool micro = false;
  if (fkind == kFwdMulticlass) {
    PyObject* co = PyDict_GetItem(st, g_k_classes);
    PyObject* ko = PyDict_GetItem(st, g_k_topk);
    if (co == nullptr || !PyLong_CheckExact(co) || ko == nullptr || !PyLong_CheckExact(ko)) TM_DECLINE;
    if (PyLong_AsLongLong(ko) != 1) TM_DECLINE;
    size = PyLong_AsLongLong(co);
    if (p.dim() != 2 || t.dim() != 1 || p.size(1) != size || p.size(0) != t.size(0)) TM_DECLINE;
    micro = PyDict_GetItem(st, g_k_micro) == Py_True;
    avg = micro ? 0 : (update_only ? 1 : read_average(st));
  } else if (fkind == kFwdBinary) {
    size = 1;
    if (p.dim() != 1 || t.dim() != 1 || p.size(0) != t.size(0)) TM_DECLINE;
    avg = 0;  // the binary score = the micro body with the binary (multilabel) formula over one label
  } else {
    PyObject* lo = PyDict_GetItem(st, g_k_labels);
    if (lo == nullptr || !PyLong_CheckExact(lo)) TM_DECLINE;
    size = PyLong_AsLongLong(lo);
    if (p.dim() != 2 || t.dim() != 2 || p.size(1) != size || p.sizes() != t.sizes()) TM_DECLINE;
    avg = update_only ? 1 : read_average(st);
  }
  if (avg < 0) TM_DECLINE;
  double threshold = 0.5;
  if (fkind != kFwdMulticlass) {
    PyObject* th = PyDict_GetItem(st, g_k_threshold);
    if (th == nullptr || !(PyFloat_Check(th) || PyLong_Check(th))) TM_DECLINE;
    threshold = PyFloat_AsDouble(th);
  }
  if (PyDict_SetItem(st, g_k_computed, Py_None) != 0) return -1;
  const long long ssize = micro ? 1 : size;
  const at::Tensor* tp = state_tensor(st, g_k_tp, dev, ssize);
  const at::Tensor* fp = state_tensor(st, g_k_fp, dev, ssize);
  const at::Tensor* tn = state_tensor(st, g_k_tn, dev, ssize);
  const at::Tensor* fn = state_tensor(st, g_k_fn, dev, ssize);
  if (tp == nullptr || fp == nullptr || tn == nullptr || fn == nullptr) TM_DECLINE;
  if (!update_only && !states_unobserved(st, {g_k_tp, g_k_fp, g_k_tn, g_k_fn})) TM_DECLINE;
  const at::Tensor* flag = forward_flag(self, st, dev);
  if (flag == nullptr) TM_DECLINE;
  at::Tensor ws, not_prob;
  const bool mc = fkind == kFwdMulticlass;
  if (!workspace(st, dev, mc ? 3 * size + 1 : 7 * size, ws, mc ? nullptr : &not_prob)) TM_DECLINE;
  if (update_only) {
    try {
      if (mc && !micro && !has_ignore && tm_amd::mc_stats_direct(p, t, *tp, *fp, *tn, *fn, *flag, size)) {
        // one launch straight into the states (wide 16-bit rows)
      } else if (mc) {
        tm_amd::mc_update(p, t, ws, *flag, size, ignore, has_ignore, 1, false);
        tm_amd::mc_stats_finalize(ws, size, micro, true, *tp, *fp, *tn, *fn);
      } else {
        tm_amd::bin_update(p, t, ws, *flag, not_prob, size, threshold, ignore, has_ignore, false, true);
        tm_amd::bin_stats_finalize(ws, not_prob, true, *tp, *fp, *tn, *fn);
      }
    } catch (const c10::Error& e) {
      PyErr_SetString(PyExc_RuntimeError, e.what_without_backtrace());
      return -1;
    }
    PyObject* cnt = PyDict_GetItem(st, g_k_count);
    if (cnt == nullptr || !PyLong_CheckExact(cnt)) return -1;
    PyObject* n1 = PyLong_FromLongLong(PyLong_AsLongLong(cnt) + 1);
    if (n1 == nullptr) return -1;
    const int rc = PyDict_SetItem(st, g_k_count, n1);
    Py_DECREF(n1);
    if (rc != 0) return -1;
    ++self->calls;
    Py_INCREF(Py_None);
    *result = Py_None;
    return 1;
  }
  const bool per_class = avg == 3 && !micro;
  at::Tensor out;
  try {
    out = at::empty({per_class ? size : 1}, p.options().dtype(at::kFloat));
    if (mc) {
      tm_amd::mc_update(p, t, ws, *flag, size, ignore, has_ignore, 1, false);
      tm_amd::mc_stats_forward(ws, size, micro, *tp, *fp, *tn, *fn, self->stat_kind, avg, beta, out);
    } else {
      tm_amd::bin_update(p, t, ws, *flag, not_prob, size, threshold, ignore, has_ignore, false, true);
      tm_amd::bin_stats_forward(ws, not_prob, *tp, *fp, *tn, *fn, self->stat_kind, avg, beta, out);
    }
  } catch (const c10::Error& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what_without_backtrace());
    return -1;
  }
  // compute() squeezes one-element values
  return forward_bookkeeping(self, st, out.numel() == 1 ? out.view(at::IntArrayRef{}) : out, result);
}

int mc_stats_forward_fast(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** r) {
  return stats_forward(self, a, b, r, kFwdMulticlass);
}
int bin_stats_forward_fast(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** r) {
  return stats_forward(self, a, b, r, kFwdBinary);
}
int ml_stats_forward_fast(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** r) {
  return stats_forward(self, a, b, r, kFwdMultilabel);
}
int mc_stats_update_fast(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** r) {
  return stats_forward(self, a, b, r, kFwdMulticlass, true);
}
int bin_stats_update_fast(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** r) {
  return stats_forward(self, a, b, r, kFwdBinary, true);
}
int ml_stats_update_fast(NativeUpdate* self, PyObject* a, PyObject* b, PyObject** r) {
  return stats_forward(self, a, b, r, kFwdMultilabel, true);
}

// stats_updater(kind, state_dict, fallback) -> callable: the stat-score family's native update (kind 1 multiclass,
// 2 binary, 3 multilabel; see stats_forward)
PyObject* make_stats_updater(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3 || !PyLong_Check(args[0]) || !PyDict_Check(args[1]) || !PyCallable_Check(args[2])) {
    PyErr_SetString(PyExc_TypeError, "stats_updater(kind: int, state: dict, fallback: callable)");
    return nullptr;
  }
  const long kind = PyLong_AsLong(args[0]);
  if (kind < 1 || kind > 3) {
    PyErr_SetString(PyExc_ValueError, "stats_updater: bad kind");
    return nullptr;
  }
  auto* self = PyObject_GC_New(NativeUpdate, &NativeUpdateType);
  if (self == nullptr) return nullptr;
  self->vectorcall = native_update_vectorcall;
  Py_INCREF(args[1]);
  self->state = args[1];
  Py_INCREF(args[2]);
  self->fallback = args[2];
  self->sink = nullptr;
  self->calls = 0;
  self->decline = 0;
  self->range_name[0] = '\0';
  static const FastFn kFns[] = {nullptr, mc_stats_update_fast, bin_stats_update_fast, ml_stats_update_fast};
  self->fast = kFns[kind];
  self->stat_kind = 0;
  PyObject_GC_Track(reinterpret_cast<PyObject*>(self));
  return reinterpret_cast<PyObject*>(self);
}

PyTypeObject NativeForwardType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// forward_native(kind, state_dict, fallback, stat_kind) -> callable;
// kind: 0 confusion matrix, 1 multiclass / 2 binary / 3 multilabel stat scores; stat_kind: cbody::StatKind
PyObject* make_forward(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 4 || !PyLong_Check(args[0]) || !PyDict_Check(args[1]) || !PyCallable_Check(args[2]) ||
      !PyLong_Check(args[3])) {
    PyErr_SetString(PyExc_TypeError, "forward_native(kind: int, state: dict, fallback: callable, stat_kind: int)");
    return nullptr;
  }
  const long kind = PyLong_AsLong(args[0]);
  const long sk = PyLong_AsLong(args[3]);
  if (kind < 0 || kind > 3 || sk < 0 || sk > 5) {
    PyErr_SetString(PyExc_ValueError, "forward_native: bad kind / stat_kind");
    return nullptr;
  }
  auto* self = PyObject_GC_New(NativeUpdate, &NativeForwardType);
  if (self == nullptr) return nullptr;
  self->vectorcall = native_update_vectorcall;
  Py_INCREF(args[1]);
  self->state = args[1];
  Py_INCREF(args[2]);
  self->fallback = args[2];
  self->sink = nullptr;
  self->calls = 0;
  self->decline = 0;
  self->range_name[0] = '\0';
  static const FastFn kFns[] = {confmat_forward, mc_stats_forward_fast, bin_stats_forward_fast,
                                ml_stats_forward_fast};
  self->fast = kFns[kind];
  self->stat_kind = static_cast<int>(sk);
  PyObject_GC_Track(reinterpret_cast<PyObject*>(self));
  return reinterpret_cast<PyObject*>(self);
}

// ------------------------------------------------------------------------------------- mAP update front end
// map_pack(preds, target, box_mode) -> (det_box, det_scores, det_labels, gt_box, gt_labels, gt_crowds, gt_area,
// det_sizes, gt_sizes) or None.  MeanAveragePrecision.update's whole per-image walk in C++: the same acceptance test
// as detection/helpers.py _inputs_ok (dict keys, tensor types, per-image lengths) plus the conditions for one flat
// buffer per state (one CUDA device, one dtype per state, contiguous [n] / [n, 4] tensors), then ONE pack kernel
// launch per 128 (image, state) segments (csrc/detection/pack_images.hip).  box_mode 1 converts xyxy boxes to xywh in
// the copy; 0 copies them.  None: anything else -- the Python path validates (raising the reference's errors) and
// packs.
namespace {

struct ImgTensors {
  const at::Tensor* t[7];  // det box, scores, labels, gt box, labels, crowds (or null), area (or null)
  int64_t dn, gn;
};

const at::Tensor* dict_tensor(PyObject* d, const char* key) {
  PyObject* o = PyDict_GetItemString(d, key);  // borrowed
  if (o == nullptr || !THPVariable_Check(o)) return nullptr;
  return &THPVariable_Unpack(o);
}

}  // namespace

PyObject* map_pack(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3 || !PyLong_Check(args[2])) {
    PyErr_SetString(PyExc_TypeError, "map_pack(preds, target, box_mode)");
    return nullptr;
  }
  const int box_mode = static_cast<int>(PyLong_AsLong(args[2]));
  if (!(PyList_Check(args[0]) || PyTuple_Check(args[0])) || !(PyList_Check(args[1]) || PyTuple_Check(args[1])))
    Py_RETURN_NONE;
  PyObject* pf = PySequence_Fast(args[0], "preds");
  PyObject* tf = PySequence_Fast(args[1], "target");
  if (pf == nullptr || tf == nullptr) {
    Py_XDECREF(pf);
    Py_XDECREF(tf);
    return nullptr;
  }
  auto done_none = [&]() {
    Py_DECREF(pf);
    Py_DECREF(tf);
    Py_RETURN_NONE;
  };
  const Py_ssize_t N = PySequence_Fast_GET_SIZE(pf);
  if (N == 0 || N != PySequence_Fast_GET_SIZE(tf)) return done_none();
  std::vector<ImgTensors> imgs(static_cast<size_t>(N));
  at::ScalarType dt[7];
  bool have[7] = {false, false, false, false, false, false, false};
  int dev = -1;
  int64_t D = 0, G = 0;
  for (Py_ssize_t i = 0; i < N; ++i) {
    PyObject* p = PySequence_Fast_GET_ITEM(pf, i);
    PyObject* t = PySequence_Fast_GET_ITEM(tf, i);
    if (!PyDict_Check(p) || !PyDict_Check(t)) return done_none();
    ImgTensors& im = imgs[static_cast<size_t>(i)];
    im.t[0] = dict_tensor(p, "boxes");
    im.t[1] = dict_tensor(p, "scores");
    im.t[2] = dict_tensor(p, "labels");
    im.t[3] = dict_tensor(t, "boxes");
    im.t[4] = dict_tensor(t, "labels");
    im.t[5] = PyDict_GetItemString(t, "iscrowd") ? dict_tensor(t, "iscrowd") : nullptr;
    im.t[6] = PyDict_GetItemString(t, "area") ? dict_tensor(t, "area") : nullptr;
    if (!im.t[0] || !im.t[1] || !im.t[2] || !im.t[3] || !im.t[4]) return done_none();
    if ((PyDict_GetItemString(t, "iscrowd") && !im.t[5]) || (PyDict_GetItemString(t, "area") && !im.t[6]))
      return done_none();
    if (im.t[2]->dim() != 1 || im.t[4]->dim() != 1) return done_none();
    im.dn = im.t[2]->size(0);
    im.gn = im.t[4]->size(0);
    for (int k = 0; k < 7; ++k) {
      const at::Tensor* x = im.t[k];
      if (x == nullptr) continue;
      const int64_t n = k < 3 ? im.dn : im.gn;
      if (!x->is_cuda() || !x->is_contiguous()) return done_none();
      if (dev < 0) dev = x->get_device();
      if (x->get_device() != dev) return done_none();
      if (k == 0 || k == 3) {  // boxes [n, 4] (an empty image may hold any empty shape)
        if (x->numel() == 0 ? n != 0 : (x->dim() != 2 || x->size(0) != n || x->size(1) != 4)) return done_none();
      } else if (x->dim() != 1 || x->size(0) != n) {
        return done_none();
      }
      if (!have[k]) {
        dt[k] = x->scalar_type();
        have[k] = true;
      } else if (dt[k] != x->scalar_type()) {
        return done_none();
      }
    }
    D += im.dn;
    G += im.gn;
  }
  // missing iscrowd / area are zeros of the labels' dtype (zeros_like(labels)): one dtype per state in any case
  for (int k = 5; k < 7; ++k) {
    bool missing = false;
    for (const auto& im : imgs) missing |= im.t[k] == nullptr;
    if (!have[k]) dt[k] = dt[4];
    else if (missing && dt[k] != dt[4]) return done_none();
  }
  if (dt[0] != at::kFloat && dt[0] != at::kDouble) return done_none();
  if (dt[3] != at::kFloat && dt[3] != at::kDouble) return done_none();
  PyObject* result = nullptr;
  try {
    const auto opt = at::TensorOptions().device(at::kCUDA, dev);
    at::Tensor out[7] = {
        at::empty({D, 4}, opt.dtype(dt[0])), at::empty({D}, opt.dtype(dt[1])), at::empty({D}, opt.dtype(dt[2])),
        at::empty({G, 4}, opt.dtype(dt[3])), at::empty({G}, opt.dtype(dt[4])), at::empty({G}, opt.dtype(dt[5])),
        at::empty({G}, opt.dtype(dt[6]))};
    std::vector<tm_amd::PackSeg> segs;
    segs.reserve(static_cast<size_t>(N) * 7);
    int64_t doff = 0, goff = 0;
    for (const auto& im : imgs) {
      for (int k = 0; k < 7; ++k) {
        const int64_t n = k < 3 ? im.dn : im.gn;
        if (n == 0) continue;
        const int64_t off = k < 3 ? doff : goff;
        const bool box = k == 0 || k == 3;
        const int64_t es = static_cast<int64_t>(out[k].element_size());
        tm_amd::PackSeg sg;
        sg.dst = static_cast<char*>(out[k].data_ptr()) + off * es * (box ? 4 : 1);
        sg.src = im.t[k] != nullptr ? im.t[k]->data_ptr() : nullptr;
        sg.esize = static_cast<int16_t>(es);
        if (box && box_mode == 1) {
          sg.mode = tm_amd::kPackXyxyToXywh;
          sg.n = static_cast<int32_t>(n);
        } else {
          sg.mode = sg.src == nullptr ? tm_amd::kPackZero : tm_amd::kPackCopy;
          sg.n = static_cast<int32_t>(n * (box ? 4 : 1));
        }
        segs.push_back(sg);
      }
      doff += im.dn;
      goff += im.gn;
    }
    tm_amd::pack_segments(segs.data(), static_cast<int>(segs.size()), dev);
    PyObject* ds = PyList_New(N);
    PyObject* gs = PyList_New(N);
    if (ds == nullptr || gs == nullptr) {
      Py_XDECREF(ds);
      Py_XDECREF(gs);
      Py_DECREF(pf);
      Py_DECREF(tf);
      return nullptr;
    }
    for (Py_ssize_t i = 0; i < N; ++i) {
      PyList_SET_ITEM(ds, i, PyLong_FromLongLong(imgs[static_cast<size_t>(i)].dn));
      PyList_SET_ITEM(gs, i, PyLong_FromLongLong(imgs[static_cast<size_t>(i)].gn));
    }
    result = PyTuple_New(9);
    for (int k = 0; k < 7; ++k) PyTuple_SET_ITEM(result, k, THPVariable_Wrap(out[k]));
    PyTuple_SET_ITEM(result, 7, ds);
    PyTuple_SET_ITEM(result, 8, gs);
  } catch (const c10::Error& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what_without_backtrace());
  }
  Py_DECREF(pf);
  Py_DECREF(tf);
  return result;
}

// read_word(word: Tensor) -> int: an int32 device word through mapped host memory + a stream sync
// (compute_tasks.hip read_word_sync), the GIL released while the stream drains
PyObject* read_word(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 1 || !THPVariable_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "read_word(word: Tensor)");
    return nullptr;
  }
  const at::Tensor w = THPVariable_Unpack(args[0]);
  int64_t v = 0;
  std::string err;
  Py_BEGIN_ALLOW_THREADS
  try {
    v = tm_amd::read_word_sync(w);
  } catch (const c10::Error& e) {
    err = e.what_without_backtrace();
  } catch (const std::exception& e) {
    err = e.what();
  }
  Py_END_ALLOW_THREADS
  if (!err.empty()) {
    PyErr_SetString(PyExc_RuntimeError, err.c_str());
    return nullptr;
  }
  return PyLong_FromLongLong(v);
}

// read_words(table: CPU int64 [n, 2], anchor: Tensor, spin_us: int) -> list[int]: every status word of a collection
// compute() through one gather kernel + a sequence-number spin on mapped host memory (compute_tasks.hip), the GIL
// released while it waits
PyObject* read_words_fc(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3 || !THPVariable_Check(args[0]) || !THPVariable_Check(args[1]) || !PyLong_Check(args[2])) {
    PyErr_SetString(PyExc_TypeError, "read_words(table: Tensor, anchor: Tensor, spin_us: int)");
    return nullptr;
  }
  const at::Tensor table = THPVariable_Unpack(args[0]);
  const at::Tensor anchor = THPVariable_Unpack(args[1]);
  const int64_t spin = PyLong_AsLongLong(args[2]);
  std::vector<int64_t> v;
  std::string err;
  Py_BEGIN_ALLOW_THREADS
  try {
    v = tm_amd::read_words(table, anchor, spin);
  } catch (const c10::Error& e) {
    err = e.what_without_backtrace();
  } catch (const std::exception& e) {
    err = e.what();
  }
  Py_END_ALLOW_THREADS
  if (!err.empty()) {
    PyErr_SetString(PyExc_RuntimeError, err.c_str());
    return nullptr;
  }
  PyObject* out = PyList_New(static_cast<Py_ssize_t>(v.size()));
  if (out == nullptr) return nullptr;
  for (size_t i = 0; i < v.size(); ++i) PyList_SET_ITEM(out, static_cast<Py_ssize_t>(i), PyLong_FromLongLong(v[i]));
  return out;
}

PyMethodDef kFactoryMethods[] = {
    {"read_words", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&read_words_fc)), METH_FASTCALL,
     "every status word of a collection compute() in one gather kernel + a sequence spin on mapped host memory"},
    {"read_word", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&read_word)), METH_FASTCALL,
     "an int32 device word read through mapped host memory after a stream sync"},
    {"stats_updater", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&make_stats_updater)),
     METH_FASTCALL, "native update of the stat-score family bound to a metric's __dict__"},
    {"forward_native", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&make_forward)), METH_FASTCALL,
     "native Metric.forward of the confusion-matrix / stat-score families bound to a metric's __dict__"},
    {"confmat_updater", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&make_confmat_updater)),
     METH_FASTCALL, "native MulticlassConfusionMatrix.update bound to a metric's __dict__"},
    {"map_pack", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&map_pack)), METH_FASTCALL,
     "MeanAveragePrecision.update's per-image validation and packing in one native call"},
    {"set_ranges", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&set_ranges)), METH_FASTCALL,
     "turn the roctx ranges of the native update / forward entry points on or off"},
    {"_sole_ref", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&sole_ref)), METH_FASTCALL,
     "whether a dict entry is a tensor referenced by nothing but that dict"},
    {"_states_unobserved", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(&states_unobserved_probe)),
     METH_FASTCALL, "the native forward's test that nothing outside the metric holds the given states"},
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
  NativeForwardType.tp_name = "torchmetrics_amd._C._fastcall.NativeForward";
  NativeForwardType.tp_basicsize = sizeof(NativeUpdate);
  NativeForwardType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC | Py_TPFLAGS_HAVE_VECTORCALL;
  NativeForwardType.tp_vectorcall_offset = offsetof(NativeUpdate, vectorcall);
  NativeForwardType.tp_call = PyVectorcall_Call;
  NativeForwardType.tp_traverse = native_update_traverse;
  NativeForwardType.tp_clear = native_update_clear;
  NativeForwardType.tp_dealloc = native_update_dealloc;
  NativeForwardType.tp_getset = kNativeUpdateGetSet;
  NativeForwardType.tp_doc = "native metric forward (see csrc/bindings/fastcall.cpp)";
  if (PyType_Ready(&NativeForwardType) < 0) return nullptr;
  g_k_confmat = PyUnicode_InternFromString("confmat");
  g_k_err = PyUnicode_InternFromString("_device_errors");
  g_k_count = PyUnicode_InternFromString("_update_count");
  g_k_computed = PyUnicode_InternFromString("_computed");
  g_k_cpu = PyUnicode_InternFromString("compute_on_cpu");
  g_k_classes = PyUnicode_InternFromString("num_classes");
  g_k_ignore = PyUnicode_InternFromString("ignore_index");
  g_k_validate = PyUnicode_InternFromString("validate_args");
  g_k_tp = PyUnicode_InternFromString("tp");
  g_k_fp = PyUnicode_InternFromString("fp");
  g_k_tn = PyUnicode_InternFromString("tn");
  g_k_fn = PyUnicode_InternFromString("fn");
  g_k_wsobj = PyUnicode_InternFromString("_ws");
  g_k_ws = PyUnicode_InternFromString("ws");
  g_k_notprob = PyUnicode_InternFromString("not_prob");
  g_k_topk = PyUnicode_InternFromString("top_k");
  g_k_mdavg = PyUnicode_InternFromString("multidim_average");
  g_k_average = PyUnicode_InternFromString("average");
  g_k_micro = PyUnicode_InternFromString("_micro");
  g_k_labels = PyUnicode_InternFromString("num_labels");
  g_k_threshold = PyUnicode_InternFromString("threshold");
  g_k_beta = PyUnicode_InternFromString("beta");
  g_k_synced = PyUnicode_InternFromString("_is_synced");
  g_k_dsos = PyUnicode_InternFromString("dist_sync_on_step");
  g_k_fcache = PyUnicode_InternFromString("_forward_cache");
  g_k_defaults = PyUnicode_InternFromString("_defaults");
  g_k_normalize = PyUnicode_InternFromString("normalize");
  PyObject* m = PyModule_Create(&kModule);
  if (m == nullptr) return nullptr;
  if (PyModule_AddFunctions(m, kFactoryMethods) < 0) return nullptr;
  return m;
}
