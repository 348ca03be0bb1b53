// Batched bootstrap update of the multiclass stat-score family (BootStrapper, SURVEY.md §7.3 P10 / VERDICT r1 item 7).
//
// The reference keeps `num_bootstraps` metric copies and, per update, draws one resampling on the host, copies it to
// the device, gathers every input tensor and runs a full metric update -- B x (H2D copy + gathers + update launches)
// (S/wrappers/bootstrapping.py:125-146).  A resampling is a vector of integer multiplicities w[i] >= 0 per sample
// (Poisson(1) draws, or multinomial counts), and the stat-score states are sums over samples, so bootstrap b's update
// is the weighted histogram  tp[b, t] += w[b, i] (p == t),  fp[b, p] / fn[b, t] += w[b, i] (p != t).
// One wave per row computes the row's argmax once (torch.argmax semantics), then the wave's lanes walk the B
// bootstraps (weights stored [n, B]: contiguous per row) and add the non-zero multiplicities to the [B, 3C + 1]
// workspace that mc_finalize_kernel folds into the stacked [B, C] states: 2 launches per update for all bootstraps.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;

template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) mc_bootstrap_kernel(const scalar_t* __restrict__ preds,
                                                              const target_t* __restrict__ target,
                                                              const int* __restrict__ weights, long long N, int C,
                                                              int B, bool label_preds, long long ignore,
                                                              bool has_ignore, int64_t* __restrict__ ws,
                                                              int* __restrict__ flag) {
  const int lane = threadIdx.x & (kWave - 1);
  const long long nwaves = static_cast<long long>(gridDim.x) * (kBlock / kWave);
  for (long long row = (static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x) / kWave; row < N;
       row += nwaves) {  // wave-uniform
    const long long t = static_cast<long long>(target[row]);
    if (has_ignore && t == ignore) continue;
    if (t < 0 || t >= C) {
      if (lane == 0) raise_flag(flag, kErrTargetOutOfRange);
      continue;
    }
    int p;
    if (label_preds) {
      const long long v = static_cast<long long>(preds[row]);
      if (v < 0 || v >= C) {
        if (lane == 0) raise_flag(flag, kErrPredsOutOfRange);
        continue;
      }
      p = static_cast<int>(v);
    } else {
      float best = -INFINITY;
      int bi = 0x7fffffff;
      const scalar_t* r = preds + row * C;
      for (int c = lane; c < C; c += kWave) {
        const float v = to_f32(r[c]);
        if (argmax_better(v, c, best, bi)) {
          best = v;
          bi = c;
        }
      }
      wave_argmax(best, bi);
      p = bi;
    }
    const int* w = weights + row * B;
    const long long stride = 3LL * C + 1;
    for (int b = lane; b < B; b += kWave) {
      const int m = w[b];
      if (m == 0) continue;
      int64_t* g = ws + b * stride;
      if (p == t) {
        atomic_add_i64(g + t, m);
      } else {
        atomic_add_i64(g + C + p, m);
        atomic_add_i64(g + 2 * C + t, m);
      }
    }
  }
}

}  // namespace

// preds: [N, C] float scores or [N] integer labels; target: [N] integer; weights: int32 [N, B] multiplicities;
// ws: int64 [B, 3C + 1] zero workspace (mc_stats_finalize folds it into the [B, C] states and re-zeroes it).
void mc_bootstrap_update(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& weights, at::Tensor ws,
                         at::Tensor flag, int64_t num_classes, int64_t ignore_index, bool has_ignore) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, weights);
  TM_SAME_DEVICE(preds, ws);
  TM_SAME_DEVICE(preds, flag);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TM_CHECK_CONTIG(weights);
  TM_CHECK_CONTIG(ws);
  const long long N = target.numel();
  const int C = static_cast<int>(num_classes);
  TORCH_CHECK(C >= 1, "mc_bootstrap_update: num_classes >= 1");
  const bool label_preds = !at::isFloatingType(preds.scalar_type());
  TORCH_CHECK(label_preds ? preds.numel() == N : preds.numel() == N * C,
              "mc_bootstrap_update: preds must be [N, C] scores or [N] labels");
  TORCH_CHECK(weights.scalar_type() == at::kInt && weights.dim() == 2 && weights.size(0) == N,
              "mc_bootstrap_update: weights must be int32 [N, B]");
  const int B = static_cast<int>(weights.size(1));
  TORCH_CHECK(ws.scalar_type() == at::kLong && ws.numel() == static_cast<long long>(B) * (3LL * C + 1),
              "mc_bootstrap_update: ws must be int64 [B, 3C + 1]");
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "mc_bootstrap_update: flag");
  if (N == 0 || B == 0) return;
  const int grid = grid_cap((N + (kBlock / kWave) - 1) / (kBlock / kWave), 256 * 8);
  TM_DISPATCH_TARGET(target.scalar_type(), "mc_bootstrap_update", [&] {
    TM_DISPATCH_PREDS(preds.scalar_type(), "mc_bootstrap_update", [&] {
      hipLaunchKernelGGL((mc_bootstrap_kernel<scalar_t, target_t>), dim3(grid), dim3(kBlock), 0, stream(),
                         reinterpret_cast<const scalar_t*>(preds.data_ptr()),
                         reinterpret_cast<const target_t*>(target.data_ptr()), weights.data_ptr<int>(), N, C, B,
                         label_preds, static_cast<long long>(ignore_index), has_ignore, ws.data_ptr<int64_t>(),
                         flag.data_ptr<int>());
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "mc_bootstrap_update(Tensor preds, Tensor target, Tensor weights, Tensor(a!) ws, Tensor(b!) flag, int num_classes, "
      "int ignore_index, bool has_ignore) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("mc_bootstrap_update", &mc_bootstrap_update); }

}  // namespace tm_amd
