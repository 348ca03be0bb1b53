// Multiclass calibration-error update: per-row top-label confidence and correctness in two launches.
//
// Reference (F/classification/calibration_error.py, `_multiclass_calibration_error_update` + format/validation):
//   if not torch.all((preds >= 0) * (preds <= 1)): preds = preds.softmax(1)   # host sync on the whole batch
//   confidences, predictions = preds.max(dim=1); accuracies = predictions.eq(target)
// plus a target range check -- ~15 ATen launches and a device->host round trip per update.
//
// Here:  launch A, one pass per row, computes BOTH candidates -- the raw top-1 (value, first index) and the top-1 of
// the softmax rounded to the input dtype (torch's softmax output dtype; rounding can create ties that move the first
// max index, so the softmax argmax is taken on the rounded values, not copied from the raw argmax) -- and ORs a
// per-batch "not a probability" bit and the target range bit into device words.  Launch B selects the candidate the
// batch-wide bit asks for and writes the two list-state tensors.  The "not a probability" word is double-buffered:
// B of update k re-zeros the slot update k+1 will use.
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;

template <typename scalar_t>
__device__ __forceinline__ float ld(const scalar_t* p, long long i) {
  return to_f32(p[i]);
}

// raw and softmax candidates of one row, serial over its C scores (rows of <= 64 classes: one thread per row)
template <typename scalar_t>
__device__ __forceinline__ void row_candidates(const scalar_t* __restrict__ r, int C, float& raw_v, int& raw_i,
                                               float& soft_v, int& soft_i, bool& outside) {
  float mx = -INFINITY;
  int mi = 0x7fffffff;
  bool out = false;
  for (int c = 0; c < C; ++c) {
    const float v = to_f32(r[c]);
    out |= !(v >= 0.f && v <= 1.f);
    if (argmax_better(v, c, mx, mi)) {
      mx = v;
      mi = c;
    }
  }
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += expf(to_f32(r[c]) - mx);
  float sv = -INFINITY;
  int si = 0x7fffffff;
  for (int c = 0; c < C; ++c) {
    const float p = round_to<scalar_t>(expf(to_f32(r[c]) - mx) / s);
    if (argmax_better(p, c, sv, si)) {
      sv = p;
      si = c;
    }
  }
  raw_v = mx;
  raw_i = mi;
  soft_v = sv;
  soft_i = si;
  outside = out;
}

template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) calib_rows_kernel(const scalar_t* __restrict__ preds,
                                                            const target_t* __restrict__ target, long long M, int C,
                                                            float4* __restrict__ cand, int* __restrict__ notprob,
                                                            int* __restrict__ flag) {
  const long long row = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  bool outside = false;
  if (row < M) {
    float rv, sv;
    int ri, si;
    row_candidates(preds + row * C, C, rv, ri, sv, si, outside);
    const long long t = static_cast<long long>(target[row]);
    if (flag != nullptr && (t < 0 || t >= C)) raise_flag(flag, kErrTargetOutOfRange);
    cand[row] = make_float4(rv, ri == t ? 1.f : 0.f, sv, si == t ? 1.f : 0.f);
  }
  // one atomic per wave that saw a score outside [0, 1] (NaN counts as outside, as in the reference's test)
  if (__any(outside) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(notprob, 1);
}

// wave per row for wide rows (C > 64): lanes stride the row, wave reductions for max / sum / softmax argmax
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) calib_wide_kernel(const scalar_t* __restrict__ preds,
                                                            const target_t* __restrict__ target, long long M, int C,
                                                            float4* __restrict__ cand, int* __restrict__ notprob,
                                                            int* __restrict__ flag) {
  const int lane = threadIdx.x & (kWave - 1);
  const long long nwaves = static_cast<long long>(gridDim.x) * (blockDim.x / kWave);
  bool outside = false;
  for (long long row = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) / kWave; row < M;
       row += nwaves) {
    const scalar_t* r = preds + row * C;
    float mx = -INFINITY;
    int mi = 0x7fffffff;
    for (int c = lane; c < C; c += kWave) {
      const float v = to_f32(r[c]);
      outside |= !(v >= 0.f && v <= 1.f);
      if (argmax_better(v, c, mx, mi)) {
        mx = v;
        mi = c;
      }
    }
    wave_argmax(mx, mi);
    float s = 0.f;
    for (int c = lane; c < C; c += kWave) s += expf(to_f32(r[c]) - mx);
    s = wave_sum(s);
    float sv = -INFINITY;
    int si = 0x7fffffff;
    for (int c = lane; c < C; c += kWave) {
      const float p = round_to<scalar_t>(expf(to_f32(r[c]) - mx) / s);
      if (argmax_better(p, c, sv, si)) {
        sv = p;
        si = c;
      }
    }
    wave_argmax(sv, si);
    if (lane == 0) {
      const long long t = static_cast<long long>(target[row]);
      if (flag != nullptr && (t < 0 || t >= C)) raise_flag(flag, kErrTargetOutOfRange);
      cand[row] = make_float4(mx, mi == t ? 1.f : 0.f, sv, si == t ? 1.f : 0.f);
    }
  }
  if (__any(outside) && lane == 0) atomicOr(notprob, 1);
}

// raw scores are returned in the input precision (torch.max keeps the dtype), softmax ones are already rounded
template <typename scalar_t>
__global__ void __launch_bounds__(kBlock) calib_select_kernel(const float4* __restrict__ cand, long long M,
                                                              const int* __restrict__ notprob_cur,
                                                              int* __restrict__ notprob_next, float* __restrict__ conf,
                                                              float* __restrict__ acc) {
  const bool soft = *notprob_cur != 0;
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < M;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const float4 c = cand[i];
    conf[i] = soft ? c.z : round_to<scalar_t>(c.x);
    acc[i] = soft ? c.w : c.y;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *notprob_next = 0;
}

}  // namespace

// preds: [M, C] float, target: [M] int (ignored rows already removed); cand: f32 [>= 4M] scratch;
// notprob: i32 [2] double-buffered word (slot = update parity); flag: i32 [1] metric error word or empty.
void mc_calibration_update(const at::Tensor& preds, const at::Tensor& target, at::Tensor cand, at::Tensor conf,
                           at::Tensor acc, at::Tensor notprob, int64_t slot, at::Tensor flag) {
  TM_CHECK_CUDA(preds);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.dim() == 2 && target.dim() == 1 && target.size(0) == preds.size(0),
              "mc_calibration_update: preds [M, C] and target [M]");
  const long long M = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  TORCH_CHECK(cand.scalar_type() == at::kFloat && cand.numel() >= 4 * M && cand.is_contiguous(),
              "mc_calibration_update: candidate scratch too small");
  TORCH_CHECK(conf.scalar_type() == at::kFloat && acc.scalar_type() == at::kFloat && conf.numel() == M &&
                  acc.numel() == M && conf.is_contiguous() && acc.is_contiguous(),
              "mc_calibration_update: outputs must be f32 [M]");
  TORCH_CHECK(notprob.scalar_type() == at::kInt && notprob.numel() == 2 && (slot == 0 || slot == 1),
              "mc_calibration_update: notprob must be i32 [2]");
  int* flagp = nullptr;
  if (flag.numel() > 0) {
    TORCH_CHECK(flag.scalar_type() == at::kInt, "mc_calibration_update: flag must be i32");
    flagp = flag.data_ptr<int>();
  }
  if (M == 0) return;
  auto s = stream();
  int* np = notprob.data_ptr<int>();
  // inside a hipGraph capture the host parity would be frozen: word 0 is zeroed before and re-armed after the select
  // on every replay, so the graph leaves both words zero for eager updates around it (the caller keeps its parity)
  const bool captured = stream_capturing(s);
  if (captured) {
    slot = 0;
    launch_zero_words(np, 2, s);
  }
  float4* cp = reinterpret_cast<float4*>(cand.data_ptr<float>());
  TM_DISPATCH_TARGET(target.scalar_type(), "mc_calibration_update", [&] {
    const target_t* tp = reinterpret_cast<const target_t*>(target.data_ptr());
    TM_DISPATCH_FLOAT(preds.scalar_type(), "mc_calibration_update", [&] {
      const scalar_t* pp = reinterpret_cast<const scalar_t*>(preds.data_ptr());
      if (C <= 64) {
        const int grid = static_cast<int>((M + kBlock - 1) / kBlock);
        hipLaunchKernelGGL((calib_rows_kernel<scalar_t, target_t>), dim3(grid), dim3(kBlock), 0, s, pp, tp, M, C, cp,
                           np + slot, flagp);
      } else {
        const int grid = grid_cap((M + kBlock / kWave - 1) / (kBlock / kWave), 256 * 8);
        hipLaunchKernelGGL((calib_wide_kernel<scalar_t, target_t>), dim3(grid), dim3(kBlock), 0, s, pp, tp, M, C, cp,
                           np + slot, flagp);
      }
      const int grid2 = grid_cap((M + kBlock - 1) / kBlock, 256 * 4);
      hipLaunchKernelGGL((calib_select_kernel<scalar_t>), dim3(grid2), dim3(kBlock), 0, s, cp, M, np + slot,
                         np + (1 - slot), conf.data_ptr<float>(), acc.data_ptr<float>());
    });
  });
  if (captured) launch_zero_words(np, 2, s);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "mc_calibration_update(Tensor preds, Tensor target, Tensor(a!) cand, Tensor(b!) conf, Tensor(c!) acc, "
      "Tensor(d!) notprob, int slot, Tensor(e!) flag) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("mc_calibration_update", &tm_amd::mc_calibration_update); }
