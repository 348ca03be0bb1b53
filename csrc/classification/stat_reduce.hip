// Fused compute() of the stat-score family (Accuracy, Precision, Recall, F-beta, Specificity, Hamming).
//
// The composite reduction (F/classification/{accuracy,precision_recall,f_beta,specificity,hamming}.py `_*_reduce`,
// utilities/compute.py `_adjust_weights_safe_divide`) is ~15-20 tiny ATen launches per metric compute (casts, adds,
// safe divides, where, weighted sum): host-launch bound at ~0.17 ms per metric.  One block per row (global: 1 row,
// samplewise: N rows) loads the C-class tp/fp/tn/fn, evaluates the per-class score, and reduces micro / macro /
// weighted in one pass -- a single launch.  Scores are computed in fp32 from the int64 counts, as ATen does.
#include "common/compute_bodies.h"

namespace tm_amd {
namespace {

constexpr int kThreads = cbody::kThreads;

__global__ void __launch_bounds__(kThreads) stat_reduce_kernel(const int64_t* __restrict__ tp,
                                                               const int64_t* __restrict__ fp,
                                                               const int64_t* __restrict__ tn,
                                                               const int64_t* __restrict__ fn, int C, int kind,
                                                               int avg, bool multilabel, float beta2,
                                                               float* __restrict__ out) {
  __shared__ double red[kThreads / kWave];
  cbody::stat_reduce_row(tp, fp, tn, fn, C, kind, avg, multilabel, beta2, out, blockIdx.x, red);
}

}  // namespace

// tp/fp/tn/fn: [R, C] int64 contiguous; out: [R] (micro/macro/weighted) or [R, C] (none) fp32.
void stat_reduce(const at::Tensor& tp, const at::Tensor& fp, const at::Tensor& tn, const at::Tensor& fn,
                 at::Tensor out, int64_t kind, int64_t average, bool multilabel, double beta) {
  TM_CHECK_CUDA(tp);
  for (const at::Tensor* t : {&tp, &fp, &tn, &fn}) {
    TORCH_CHECK(t->scalar_type() == at::kLong && t->is_contiguous(), "stat_reduce: int64 contiguous states");
    TORCH_CHECK(t->sizes() == tp.sizes(), "stat_reduce: state shapes differ");
  }
  TORCH_CHECK(tp.dim() == 2, "stat_reduce: states must be [rows, classes]");
  TORCH_CHECK(kind >= 0 && kind <= 5 && average >= 0 && average <= 3, "stat_reduce: bad kind / average");
  const long long R = tp.size(0);
  const int C = static_cast<int>(tp.size(1));
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() &&
                  out.numel() == (average == 3 ? R * C : R),
              "stat_reduce: bad output");
  if (R == 0) return;
  hipLaunchKernelGGL(stat_reduce_kernel, dim3(static_cast<unsigned>(R)), dim3(kThreads), 0, stream(),
                     tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(), C,
                     static_cast<int>(kind), static_cast<int>(average), multilabel, static_cast<float>(beta * beta),
                     out.data_ptr<float>());
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "stat_reduce(Tensor tp, Tensor fp, Tensor tn, Tensor fn, Tensor(a!) out, int kind, int average, bool multilabel, "
      "float beta) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("stat_reduce", &stat_reduce); }

}  // namespace tm_amd
