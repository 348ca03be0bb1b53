// Fused compute() of the stat-score family (Accuracy, Precision, Recall, F-beta, Specificity, Hamming).
//
// The composite reduction (F/classification/{accuracy,precision_recall,f_beta,specificity,hamming}.py `_*_reduce`,
// utilities/compute.py `_adjust_weights_safe_divide`) is ~15-20 tiny ATen launches per metric compute (casts, adds,
// safe divides, where, weighted sum): host-launch bound at ~0.17 ms per metric.  One block per row (global: 1 row,
// samplewise: N rows) loads the C-class tp/fp/tn/fn, evaluates the per-class score, and reduces micro / macro /
// weighted in one pass -- a single launch.  Scores are computed in fp32 from the int64 counts, as ATen does.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;
enum Kind : int { kAccuracy = 0, kHamming = 1, kPrecision = 2, kRecall = 3, kSpecificity = 4, kFBeta = 5 };
enum Avg : int { kMicro = 0, kMacro = 1, kWeighted = 2, kNone = 3 };

__device__ __forceinline__ float sdiv(float n, float d) { return n / (d == 0.f ? 1.f : d); }

// per-class score (`_score` in functional/classification/_reductions.py)
__device__ __forceinline__ float class_score(int kind, float tp, float fp, float tn, float fn, bool multilabel,
                                             float beta2) {
  switch (kind) {
    case kAccuracy: return multilabel ? sdiv(tp + tn, tp + tn + fp + fn) : sdiv(tp, tp + fn);
    case kHamming: return 1.f - (multilabel ? sdiv(tp + tn, tp + tn + fp + fn) : sdiv(tp, tp + fn));
    case kPrecision: return sdiv(tp, tp + fp);
    case kRecall: return sdiv(tp, tp + fn);
    case kSpecificity: return sdiv(tn, tn + fp);
    default: return sdiv((1.f + beta2) * tp, (1.f + beta2) * tp + beta2 * fn + fp);
  }
}

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kThreads / kWave; ++w) s += red[w];
  return s;
}

__global__ void __launch_bounds__(kThreads) stat_reduce_kernel(const int64_t* __restrict__ tp,
                                                               const int64_t* __restrict__ fp,
                                                               const int64_t* __restrict__ tn,
                                                               const int64_t* __restrict__ fn, int C, int kind,
                                                               int avg, bool multilabel, float beta2,
                                                               float* __restrict__ out) {
  __shared__ double red[kThreads / kWave];
  const long long row = blockIdx.x;
  const int64_t* a = tp + row * C;
  const int64_t* b = fp + row * C;
  const int64_t* c = tn + row * C;
  const int64_t* d = fn + row * C;
  if (avg == kNone) {
    for (int k = threadIdx.x; k < C; k += kThreads)
      out[row * C + k] = class_score(kind, static_cast<float>(a[k]), static_cast<float>(b[k]), static_cast<float>(c[k]),
                                     static_cast<float>(d[k]), multilabel, beta2);
    return;
  }
  if (avg == kMicro) {
    double s[4] = {0, 0, 0, 0};
    for (int k = threadIdx.x; k < C; k += kThreads) {
      s[0] += static_cast<double>(a[k]);
      s[1] += static_cast<double>(b[k]);
      s[2] += static_cast<double>(c[k]);
      s[3] += static_cast<double>(d[k]);
    }
    for (int i = 0; i < 4; ++i) s[i] = block_sum(s[i], red);
    if (threadIdx.x == 0) {
      // micro accuracy / hamming of a multilabel problem use the binary formula, everything else the class formula
      const bool binary_form = multilabel && (kind == kAccuracy || kind == kHamming);
      out[row] = class_score(kind, static_cast<float>(s[0]), static_cast<float>(s[1]), static_cast<float>(s[2]),
                             static_cast<float>(s[3]), binary_form, beta2);
    }
    return;
  }
  double num = 0.0, den = 0.0;
  for (int k = threadIdx.x; k < C; k += kThreads) {
    const float ftp = static_cast<float>(a[k]), ffp = static_cast<float>(b[k]), ftn = static_cast<float>(c[k]),
                ffn = static_cast<float>(d[k]);
    const float sc = class_score(kind, ftp, ffp, ftn, ffn, multilabel, beta2);
    float w;
    if (avg == kWeighted)
      w = ftp + ffn;
    else
      w = (!multilabel && a[k] + b[k] + d[k] == 0) ? 0.f : 1.f;
    num += static_cast<double>(w * sc);
    den += static_cast<double>(w);
  }
  num = block_sum(num, red);
  den = block_sum(den, red);
  if (threadIdx.x == 0) out[row] = static_cast<float>(num / (den == 0.0 ? 1.0 : den));
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
