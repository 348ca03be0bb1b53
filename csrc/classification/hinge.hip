// Hinge loss update in two launches (K9 in SURVEY.md §2.5).
//
// Reference (F/classification/hinge.py:50-190): a host sync to decide whether the scores are probabilities
// (`torch.all((preds >= 0) & (preds <= 1))`, else sigmoid / softmax), the transformed copy of the scores, a one-hot
// matrix, a masked fill + row max (Crammer-Singer) or a where (one-vs-all), clamp, pow, sum: ~10 launches and one
// sync per update, plus `torch.unique(target)` for validation.
// Here one pass accumulates the losses of BOTH readings of the scores -- as given (A) and transformed (B: sigmoid for
// binary, softmax for multiclass, from the row's logsumexp without a probability copy) -- together with a "not a
// probability" word; the fold kernel keeps A or B for the batch, adds it to the metric state and re-zeroes the
// workspace.  Target values outside {0, 1, ignore} (binary) or [0, C) (multiclass) raise validation bits instead of a
// host check.  Accumulation in fp64.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;
enum Mode : int { kBinary = 0, kCrammerSinger = 1, kOneVsAll = 2 };

__device__ __forceinline__ double hinge(double margin, bool squared) {
  const double m = 1.0 - margin > 0.0 ? 1.0 - margin : 0.0;
  return squared ? m * m : m;
}

// ws layout: [K] sum A, [K] sum B, [1] count; notprob: int [1]
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) hinge_binary_kernel(const scalar_t* __restrict__ preds,
                                                              const target_t* __restrict__ target, long long N,
                                                              bool squared, long long ignore, bool has_ignore,
                                                              double* __restrict__ ws, int* __restrict__ notprob,
                                                              int* __restrict__ flag) {
  __shared__ double red[3][kBlock / kWave];
  double sa = 0.0, sb = 0.0, cnt = 0.0;
  int np = 0, bad = 0;
  for (long long i = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; i < N;
       i += static_cast<long long>(gridDim.x) * kBlock) {
    const long long t = static_cast<long long>(target[i]);
    if (has_ignore && t == ignore) continue;
    if (t != 0 && t != 1) {
      bad = 1;
      continue;
    }
    const float x = to_f32(preds[i]);
    np |= !(x >= 0.f && x <= 1.f);
    const float s = round_to<scalar_t>(1.f / (1.f + expf(-x)));  // sigmoid in the scores' dtype, as ATen
    sa += hinge(t == 1 ? x : -x, squared);
    sb += hinge(t == 1 ? s : -s, squared);
    cnt += 1.0;
  }
  if (__any(bad) && (threadIdx.x & (kWave - 1)) == 0) raise_flag(flag, kErrTargetNotBinary);
  if (__any(np) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(notprob, 1);
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  cnt = wave_sum(cnt);
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    red[0][w] = sa;
    red[1][w] = sb;
    red[2][w] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0, c = 0;
    for (int k = 0; k < kBlock / kWave; ++k) {
      a += red[0][k];
      b += red[1][k];
      c += red[2][k];
    }
    atomicAdd(ws, a);
    atomicAdd(ws + 1, b);
    atomicAdd(ws + 2, c);
  }
}

// one wave per row of [N, C] scores
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) hinge_multiclass_kernel(const scalar_t* __restrict__ preds,
                                                                  const target_t* __restrict__ target, long long N,
                                                                  int C, int mode, bool squared, long long ignore,
                                                                  bool has_ignore, double* __restrict__ ws,
                                                                  int* __restrict__ notprob, int* __restrict__ flag) {
  const int lane = threadIdx.x & (kWave - 1);
  const long long nw = static_cast<long long>(gridDim.x) * (kBlock / kWave);
  const int K = mode == kOneVsAll ? C : 1;
  double sa = 0.0, sb = 0.0, cnt = 0.0;
  int np = 0;
  for (long long row = (static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x) / kWave; row < N; row += nw) {
    const long long t = static_cast<long long>(target[row]);
    if (has_ignore && t == ignore) continue;
    if (t < 0 || t >= C) {
      if (lane == 0) raise_flag(flag, kErrTargetOutOfRange);
      continue;
    }
    const scalar_t* r = preds + row * C;
    float mx = -INFINITY, other = -INFINITY;
    for (int j = lane; j < C; j += kWave) {
      const float x = to_f32(r[j]);
      np |= !(x >= 0.f && x <= 1.f);
      mx = fmaxf(mx, x);
      if (j != t) other = fmaxf(other, x);
    }
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
      mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
      other = fmaxf(other, __shfl_xor(other, off, kWave));
    }
    float se = 0.f;
    for (int j = lane; j < C; j += kWave) se += expf(to_f32(r[j]) - mx);
    se = wave_sum(se);
    const float lse = mx + logf(se);
    if (mode == kCrammerSinger) {
      const float own = to_f32(r[t]);
      const float own_p = round_to<scalar_t>(expf(own - lse)), other_p = round_to<scalar_t>(expf(other - lse));
      if (lane == 0) {
        sa += hinge(static_cast<double>(own) - other, squared);
        sb += hinge(static_cast<double>(own_p) - other_p, squared);
        cnt += 1.0;
      }
    } else {
      for (int j = lane; j < C; j += kWave) {
        const float x = to_f32(r[j]);
        const float p = round_to<scalar_t>(expf(x - lse));
        atomicAdd(ws + j, hinge(j == t ? x : -x, squared));
        atomicAdd(ws + K + j, hinge(j == t ? p : -p, squared));
      }
      if (lane == 0) cnt += 1.0;
    }
  }
  if (__any(np) && lane == 0) atomicOr(notprob, 1);
  if (lane == 0) {
    if (mode == kCrammerSinger) {
      atomicAdd(ws, sa);
      atomicAdd(ws + 1, sb);
    }
    if (cnt != 0.0) atomicAdd(ws + 2 * K, cnt);
  }
}

// measures += (notprob ? B : A); total += count; zero the workspace
template <typename out_t>
__global__ void hinge_fold_kernel(double* __restrict__ ws, int K, int* __restrict__ notprob,
                                  out_t* __restrict__ measures, int64_t* __restrict__ total) {
  const bool use_b = *notprob != 0;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const double v = use_b ? ws[K + k] : ws[k];
    measures[k] = static_cast<out_t>(static_cast<double>(measures[k]) + v);
    ws[k] = 0.0;
    ws[K + k] = 0.0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    *total += static_cast<int64_t>(ws[2 * K]);
    ws[2 * K] = 0.0;
    *notprob = 0;
  }
}

}  // namespace

// mode 0 binary (preds/target [N]), 1 Crammer-Singer / 2 one-vs-all (preds [N, C], target [N]).
// ws: f64 [2K + 1] zero (K = C for one-vs-all, else 1); notprob: i32 [1] zero; measures: f32/f64 [K] state;
// total: i64 [1] state.
void hinge_update(const at::Tensor& preds, const at::Tensor& target, int64_t mode, bool squared, int64_t ignore_index,
                  bool has_ignore, at::Tensor ws, at::Tensor notprob, at::Tensor measures, at::Tensor total,
                  at::Tensor flag) {
  TM_CHECK_CUDA(preds);
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&target, &ws, &notprob, &measures, &total, &flag})
    TM_SAME_DEVICE(preds, (*t));
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(mode >= 0 && mode <= 2, "hinge_update: bad mode");
  const long long N = target.numel();
  const int C = mode == kBinary ? 1 : static_cast<int>(preds.numel() / (N > 0 ? N : 1));
  TORCH_CHECK(mode == kBinary ? preds.numel() == N : preds.numel() == N * C, "hinge_update: preds shape");
  const int K = mode == kOneVsAll ? C : 1;
  TORCH_CHECK(ws.scalar_type() == at::kDouble && ws.numel() == 2 * K + 1 && ws.is_contiguous(), "hinge_update: ws");
  TORCH_CHECK(notprob.scalar_type() == at::kInt && notprob.numel() == 1, "hinge_update: notprob");
  TORCH_CHECK((measures.scalar_type() == at::kFloat || measures.scalar_type() == at::kDouble) &&
                  measures.numel() == K && measures.is_contiguous(), "hinge_update: measures state");
  TORCH_CHECK(total.scalar_type() == at::kLong && total.numel() == 1, "hinge_update: total state");
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "hinge_update: flag");
  auto s = stream();
  if (N > 0) {
    TM_DISPATCH_TARGET(target.scalar_type(), "hinge_update", [&] {
      TM_DISPATCH_FLOAT(preds.scalar_type(), "hinge_update", [&] {
        const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
        const target_t* t = reinterpret_cast<const target_t*>(target.data_ptr());
        if (mode == kBinary) {
          hipLaunchKernelGGL((hinge_binary_kernel<scalar_t, target_t>), dim3(grid_cap((N + kBlock - 1) / kBlock, 1024)),
                             dim3(kBlock), 0, s, p, t, N, squared, static_cast<long long>(ignore_index), has_ignore,
                             ws.data_ptr<double>(), notprob.data_ptr<int>(), flag.data_ptr<int>());
        } else {
          hipLaunchKernelGGL((hinge_multiclass_kernel<scalar_t, target_t>),
                             dim3(grid_cap((N + (kBlock / kWave) - 1) / (kBlock / kWave), 2048)), dim3(kBlock), 0, s,
                             p, t, N, C, static_cast<int>(mode), squared, static_cast<long long>(ignore_index),
                             has_ignore, ws.data_ptr<double>(), notprob.data_ptr<int>(), flag.data_ptr<int>());
        }
      });
    });
  }
  if (measures.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(hinge_fold_kernel<float>, dim3(1), dim3(256), 0, s, ws.data_ptr<double>(), K,
                       notprob.data_ptr<int>(), measures.data_ptr<float>(), total.data_ptr<int64_t>());
  else
    hipLaunchKernelGGL(hinge_fold_kernel<double>, dim3(1), dim3(256), 0, s, ws.data_ptr<double>(), K,
                       notprob.data_ptr<int>(), measures.data_ptr<double>(), total.data_ptr<int64_t>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "hinge_update(Tensor preds, Tensor target, int mode, bool squared, int ignore_index, bool has_ignore, "
      "Tensor(a!) ws, Tensor(b!) notprob, Tensor(c!) measures, Tensor(d!) total, Tensor(e!) flag) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("hinge_update", &hinge_update); }

}  // namespace tm_amd
