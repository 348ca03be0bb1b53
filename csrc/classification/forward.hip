// Fused ``forward()`` epilogues of the stat-score family (Accuracy, Precision, Recall, F-beta, Specificity, Hamming,
// StatScores' tp/fp/tn/fn): ONE block that reads the batch counts straight out of the update workspace and
//   1. folds them into the metric's global states (tp += batch, ...: the reference's `_reduce_states` merge),
//   2. evaluates the metric on the batch counts alone (the reference's `compute()` on a freshly reset state),
//   3. re-zeros the workspace for the next call.
//
// The reference forward (S/metric.py:275-306,353-391: `_forward_reduce_state_update`) is: save the global states,
// reset(), update(), compute(), then merge global + batch state by state -- on the stat-score classes that is ~10 clones
// / adds / score launches plus the Python bookkeeping around them.  Here a forward is the update kernel + this launch
// (driven from C++, csrc/bindings/fastcall.cpp `NativeForward`); the score is the very body `compute()` uses
// (common/compute_bodies.h `stat_reduce_body`), so forward's batch value is bit-identical to `compute()` on the batch.
#include "common/compute_bodies.h"

namespace tm_amd {
NpView notprob_view(const at::Tensor& np, hipStream_t s);  // stat_scores.hip
void bin_flush_pending(const at::Tensor& ws);  // stat_scores.hip
namespace {

constexpr int kThreads = cbody::kThreads;
constexpr int kBinSlots = 7;  // binary / multilabel workspace slots per label (stat_scores.hip)

// Multiclass workspace [3C + 1]: [tp(C) | fp(C) | fn(C) | -]; tn of class c = rows - tp - fp - fn.
// micro: the states are [1] (sums over classes).
__global__ void __launch_bounds__(kThreads) mc_stats_forward_kernel(int64_t* __restrict__ ws, int C, bool micro,
                                                                    int64_t* __restrict__ tp, int64_t* __restrict__ fp,
                                                                    int64_t* __restrict__ tn, int64_t* __restrict__ fn,
                                                                    int kind, int avg, float beta2,
                                                                    float* __restrict__ out) {
  __shared__ double red[kThreads / kWave];
  __shared__ long long rows_sh[kThreads / kWave];
  // rows of the batch = sum over classes of tp + fn (each valid row is a hit or a miss of its target class)
  long long rows = 0;
  for (int c = threadIdx.x; c < C; c += kThreads) rows += ws[c] + ws[2 * C + c];
  rows = wave_sum_ll(rows);
  if ((threadIdx.x & (kWave - 1)) == 0) rows_sh[threadIdx.x / kWave] = rows;
  __syncthreads();
  long long cnt = 0;
  for (int i = 0; i < kThreads / kWave; ++i) cnt += rows_sh[i];
  auto get = [&](int k, long long& a, long long& b, long long& c, long long& d) {
    a = ws[k];
    b = ws[C + k];
    d = ws[2 * C + k];
    c = cnt - a - b - d;
  };
  if (micro) {
    double s[3] = {0, 0, 0};
    for (int k = threadIdx.x; k < C; k += kThreads) {
      s[0] += static_cast<double>(ws[k]);
      s[1] += static_cast<double>(ws[C + k]);
      s[2] += static_cast<double>(ws[2 * C + k]);
    }
    for (int i = 0; i < 3; ++i) s[i] = cbody::block_sum(s[i], red);
    if (threadIdx.x == 0) {
      const long long a = static_cast<long long>(s[0]), b = static_cast<long long>(s[1]),
                      d = static_cast<long long>(s[2]);
      const long long e = static_cast<long long>(C) * cnt - a - b - d;
      tp[0] += a;
      fp[0] += b;
      fn[0] += d;
      tn[0] += e;
      // compute() of a micro state is the class formula on the [1] sums (avg micro over one "class")
      out[0] = cbody::class_score(kind, static_cast<float>(a), static_cast<float>(b), static_cast<float>(e),
                                  static_cast<float>(d), false, beta2);
    }
  } else {
    for (int k = threadIdx.x; k < C; k += kThreads) {
      long long a, b, c, d;
      get(k, a, b, c, d);
      tp[k] += a;
      fp[k] += b;
      tn[k] += c;
      fn[k] += d;
    }
    cbody::stat_reduce_body(get, C, kind, avg, false, beta2, out, red);
  }
  __syncthreads();  // every read of the workspace is done
  for (int k = threadIdx.x; k < 3 * C + 1; k += kThreads) ws[k] = 0;
}

// Binary / multilabel workspace [L, 7] = (tpA, fpA, fnA, tpB, fpB, fnB, count); not_prob picks B (preds were logits).
__global__ void __launch_bounds__(kThreads) bin_stats_forward_kernel(int64_t* __restrict__ ws, int L,
                                                                     int* __restrict__ not_prob,
                                                                     int64_t* __restrict__ tp, int64_t* __restrict__ fp,
                                                                     int64_t* __restrict__ tn, int64_t* __restrict__ fn,
                                                                     int kind, int avg, float beta2,
                                                                     float* __restrict__ out, int slot,
                                                                     bool two_slots) {
  __shared__ double red[kThreads / kWave];
  const bool use_b = not_prob[slot] != 0;
  auto get = [&](int k, long long& a, long long& b, long long& c, long long& d) {
    const int64_t* w = ws + static_cast<long long>(k) * kBinSlots;
    a = use_b ? w[3] : w[0];
    b = use_b ? w[4] : w[1];
    d = use_b ? w[5] : w[2];
    c = w[6] - a - b - d;
  };
  for (int k = threadIdx.x; k < L; k += kThreads) {
    long long a, b, c, d;
    get(k, a, b, c, d);
    tp[k] += a;
    fp[k] += b;
    tn[k] += c;
    fn[k] += d;
  }
  // binary tasks come in as avg = micro over L = 1 with the multilabel (binary) formula
  cbody::stat_reduce_body(get, L, kind, avg, true, beta2, out, red);
  __syncthreads();
  for (long long k = threadIdx.x; k < static_cast<long long>(L) * kBinSlots; k += kThreads) ws[k] = 0;
  if (threadIdx.x == 0) not_prob[two_slots ? (slot ^ 1) : 0] = 0;  // (two words: the next update's)
}

void check_states(const at::Tensor& ws, std::initializer_list<const at::Tensor*> states, long long n, const char* what) {
  for (const at::Tensor* t : states) {
    TM_SAME_DEVICE(ws, (*t));
    TORCH_CHECK(t->scalar_type() == at::kLong && t->is_contiguous() && t->numel() == n, what,
                ": states must be contiguous int64 of the right size");
  }
}

}  // namespace

// ws: [3C + 1] int64 multiclass workspace filled by mc_update(mode = stats); tp..fn: [C] (or [1] if micro) global
// states, accumulated in place; out: fp32 [C] (avg none) or [1].
void mc_stats_forward(at::Tensor ws, int64_t num_classes, bool micro, at::Tensor tp, at::Tensor fp, at::Tensor tn,
                      at::Tensor fn, int64_t kind, int64_t average, double beta, at::Tensor out) {
  TM_CHECK_CUDA(ws);
  const int C = static_cast<int>(num_classes);
  TORCH_CHECK(ws.scalar_type() == at::kLong && ws.is_contiguous() && ws.numel() == 3LL * C + 1,
              "mc_stats_forward: workspace must be int64 [3C + 1]");
  check_states(ws, {&tp, &fp, &tn, &fn}, micro ? 1 : C, "mc_stats_forward");
  TORCH_CHECK(kind >= 0 && kind <= 5 && average >= 0 && average <= 3, "mc_stats_forward: bad kind / average");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.device() == ws.device() &&
                  out.numel() == (average == 3 && !micro ? C : 1),
              "mc_stats_forward: bad output");
  hipLaunchKernelGGL(mc_stats_forward_kernel, dim3(1), dim3(kThreads), 0, stream(), ws.data_ptr<int64_t>(), C, micro,
                     tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(),
                     static_cast<int>(kind), static_cast<int>(average), static_cast<float>(beta * beta),
                     out.data_ptr<float>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// ws: [L, 7] int64 workspace filled by bin_update (global); not_prob: int32[1]; tp..fn: [L] global states.
void bin_stats_forward(at::Tensor ws, at::Tensor not_prob, at::Tensor tp, at::Tensor fp, at::Tensor tn, at::Tensor fn,
                       int64_t kind, int64_t average, double beta, at::Tensor out) {
  TM_CHECK_CUDA(ws);
  TM_SAME_DEVICE(ws, not_prob);
  TORCH_CHECK(ws.scalar_type() == at::kLong && ws.is_contiguous() && ws.numel() % kBinSlots == 0,
              "bin_stats_forward: workspace must be int64 [L, 7]");
  const long long L = ws.numel() / kBinSlots;
  TORCH_CHECK(L >= 1 && L < (1LL << 31), "bin_stats_forward: bad label count");
  bin_flush_pending(ws);  // bin_update may have deferred its fold to the finalize
  check_states(ws, {&tp, &fp, &tn, &fn}, L, "bin_stats_forward");
  TORCH_CHECK(kind >= 0 && kind <= 5 && average >= 0 && average <= 3, "bin_stats_forward: bad kind / average");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.device() == ws.device() &&
                  out.numel() == (average == 3 ? L : 1),
              "bin_stats_forward: bad output");
  const NpView nv = notprob_view(not_prob, stream());
  hipLaunchKernelGGL(bin_stats_forward_kernel, dim3(1), dim3(kThreads), 0, stream(), ws.data_ptr<int64_t>(),
                     static_cast<int>(L), not_prob.data_ptr<int>(), tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(),
                     tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(), static_cast<int>(kind), static_cast<int>(average),
                     static_cast<float>(beta * beta), out.data_ptr<float>(), nv.slot, nv.two);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// A contiguous CUDA tensor zeroed with one hipMemsetAsync on the current stream (the native forward's batch matrix:
// no TensorIterator fill setup on the host).
void zero_async(at::Tensor t) {
  TM_CHECK_CUDA(t);
  TM_CHECK_CONTIG(t);
  C10_HIP_CHECK(hipMemsetAsync(t.data_ptr(), 0, t.numel() * t.element_size(), stream()));
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "mc_stats_forward(Tensor(a!) ws, int num_classes, bool micro, Tensor(b!) tp, Tensor(c!) fp, Tensor(d!) tn, "
      "Tensor(e!) fn, int kind, int average, float beta, Tensor(f!) out) -> ()");
  m.def(
      "bin_stats_forward(Tensor(a!) ws, Tensor(b!) not_prob, Tensor(c!) tp, Tensor(d!) fp, Tensor(e!) tn, "
      "Tensor(f!) fn, int kind, int average, float beta, Tensor(g!) out) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("mc_stats_forward", &mc_stats_forward);
  m.impl("bin_stats_forward", &bin_stats_forward);
}

}  // namespace tm_amd
