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

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fastcall", "dispatcher-free entry points of libtm_amd", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__fastcall() { return PyModule_Create(&kModule); }
