// Group-fairness stat scores (BinaryGroupStatRates / BinaryFairness updates) in two launches (K10 in SURVEY.md §2.5).
//
// Reference (F/classification/group_fairness.py:57-79 + _binary_stat_scores_format/update): a host sync for the
// probability check, sigmoid and threshold copies, `torch.argsort(groups)`, a `.cpu()` of the group sizes and a
// `torch.split` into one tensor per group, then one stat-score pass per group (four masked sums each).  Here one pass
// classifies every element (tp / fp / tn / fn under BOTH readings of float scores -- as given and sigmoid in the
// scores' dtype -- with a "not a probability" word) into a per-group LDS histogram of 2 x 4G bins; blocks flush with
// int64 atomics (deterministic), and the fold adds the reading the batch calls for into the tp / fp / tn / fn states
// in place.  Group ids are clamped into range as the torch path does (the module validates them when asked to).
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxLdsBins = 8192;  // 2 readings x 4 cells x 1024 groups (64 KiB of int64 counters)

__device__ __forceinline__ int cell_of(bool pred_pos, long long t) {
  return pred_pos ? (t == 1 ? 0 : 1) : (t == 0 ? 2 : 3);
}

template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) group_stats_kernel(const scalar_t* __restrict__ preds,
                                                             const target_t* __restrict__ target,
                                                             const int64_t* __restrict__ groups, long long N, int G,
                                                             float thr, long long ignore, bool has_ignore,
                                                             int64_t* __restrict__ ws, int* __restrict__ notprob) {
  extern __shared__ unsigned long long lds[];
  const int bins = 8 * G;
  const bool use_lds = bins <= kMaxLdsBins;
  if (use_lds) {
    for (int b = threadIdx.x; b < bins; b += kBlock) lds[b] = 0ull;
    __syncthreads();
  }
  int np = 0;
  for (long long i = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; i < N;
       i += static_cast<long long>(gridDim.x) * kBlock) {
    const long long t = static_cast<long long>(target[i]);
    bool pa, pb;
    if constexpr (IsFloating<scalar_t>::value) {
      const float x = to_f32(preds[i]);
      np |= !(x >= 0.f && x <= 1.f);
      pa = x > thr;
      pb = round_to<scalar_t>(1.f / (1.f + expf(-x))) > thr;
    } else {
      pa = pb = static_cast<long long>(preds[i]) == 1;
    }
    if (has_ignore && t == ignore) continue;
    const long long g = groups[i];
    long long ka = g * 4 + cell_of(pa, t), kb = g * 4 + cell_of(pb, t);
    ka = ka < 0 ? 0 : (ka >= 4LL * G ? 4LL * G - 1 : ka);  // the torch path's clamp
    kb = kb < 0 ? 0 : (kb >= 4LL * G ? 4LL * G - 1 : kb);
    if (use_lds) {
      atomicAdd(&lds[ka], 1ull);
      atomicAdd(&lds[4 * G + kb], 1ull);
    } else {
      atomic_add_i64(ws + ka, 1);
      atomic_add_i64(ws + 4LL * G + kb, 1);
    }
  }
  if (__any(np) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(notprob, 1);
  if (use_lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < bins; b += kBlock)
      if (lds[b]) atomic_add_i64(ws + b, static_cast<long long>(lds[b]));
  }
}

// states[k] += ws[(notprob ? 4G : 0) + 4g + k] for the tp / fp / tn / fn states; zero ws and notprob
__global__ void group_stats_fold_kernel(int64_t* __restrict__ ws, int G, int* __restrict__ notprob,
                                        int64_t* __restrict__ tp, int64_t* __restrict__ fp, int64_t* __restrict__ tn,
                                        int64_t* __restrict__ fn) {
  const bool use_b = *notprob != 0;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    const int64_t* src = ws + (use_b ? 4 * G : 0) + 4 * g;
    tp[g] += src[0];
    fp[g] += src[1];
    tn[g] += src[2];
    fn[g] += src[3];
    for (int k = 0; k < 4; ++k) {
      ws[4 * g + k] = 0;
      ws[4 * G + 4 * g + k] = 0;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) *notprob = 0;
}

}  // namespace

// preds / target / groups: [N] contiguous ROCm tensors (groups int64); ws: i64 [8G] zero; notprob: i32 [1] zero;
// tp / fp / tn / fn: i64 [G] states, updated in place.
void group_stats_update(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& groups, int64_t G,
                        double threshold, int64_t ignore_index, bool has_ignore, at::Tensor ws, at::Tensor notprob,
                        at::Tensor tp, at::Tensor fp, at::Tensor tn, at::Tensor fn) {
  TM_CHECK_CUDA(preds);
  for (const at::Tensor* t :
       std::initializer_list<const at::Tensor*>{&target, &groups, &ws, &notprob, &tp, &fp, &tn, &fn})
    TM_SAME_DEVICE(preds, (*t));
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TM_CHECK_CONTIG(groups);
  const long long N = preds.numel();
  TORCH_CHECK(target.numel() == N && groups.numel() == N, "group_stats_update: preds / target / groups sizes");
  TORCH_CHECK(groups.scalar_type() == at::kLong, "group_stats_update: groups must be int64");
  TORCH_CHECK(G >= 1 && G < (1 << 26), "group_stats_update: bad number of groups");
  TORCH_CHECK(ws.scalar_type() == at::kLong && ws.numel() == 8 * G && ws.is_contiguous(), "group_stats_update: ws");
  TORCH_CHECK(notprob.scalar_type() == at::kInt && notprob.numel() == 1, "group_stats_update: notprob");
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&tp, &fp, &tn, &fn})
    TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() == G && t->is_contiguous(),
                "group_stats_update: tp / fp / tn / fn states must be int64 [num_groups]");
  auto s = stream();
  if (N > 0) {
    const size_t lds = 8 * G <= kMaxLdsBins ? static_cast<size_t>(8 * G) * sizeof(unsigned long long) : 0;
    TM_DISPATCH_TARGET(target.scalar_type(), "group_stats_update", [&] {
      TM_DISPATCH_PREDS(preds.scalar_type(), "group_stats_update", [&] {
        float thr = static_cast<float>(threshold);
        if constexpr (std::is_same<scalar_t, c10::BFloat16>::value) thr = static_cast<float>(c10::BFloat16(thr));
        if constexpr (std::is_same<scalar_t, c10::Half>::value) thr = static_cast<float>(c10::Half(thr));
        hipLaunchKernelGGL((group_stats_kernel<scalar_t, target_t>), dim3(grid_cap((N + kBlock - 1) / kBlock, 1024)),
                           dim3(kBlock), lds, s, reinterpret_cast<const scalar_t*>(preds.data_ptr()),
                           reinterpret_cast<const target_t*>(target.data_ptr()), groups.data_ptr<int64_t>(), N,
                           static_cast<int>(G), thr, static_cast<long long>(ignore_index), has_ignore,
                           ws.data_ptr<int64_t>(), notprob.data_ptr<int>());
      });
    });
  }
  hipLaunchKernelGGL(group_stats_fold_kernel, dim3(1), dim3(256), 0, s, ws.data_ptr<int64_t>(), static_cast<int>(G),
                     notprob.data_ptr<int>(), tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(),
                     fn.data_ptr<int64_t>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "group_stats_update(Tensor preds, Tensor target, Tensor groups, int G, float threshold, int ignore_index, "
      "bool has_ignore, Tensor(a!) ws, Tensor(b!) notprob, Tensor(c!) tp, Tensor(d!) fp, Tensor(e!) tn, "
      "Tensor(f!) fn) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("group_stats_update", &group_stats_update); }

}  // namespace tm_amd
