// Multilabel ranking metrics per sample row: coverage error, label ranking average precision, ranking loss (K8,
// SURVEY.md §2.5).
//
// Reference (F/classification/ranking.py): coverage = a masked min + compare-count; LRAP = two sorts + two
// searchsorted per row (`_rank_data` max-ranks); ranking loss = `argsort().argsort()` inverse ranks -- each a chain of
// ~6-10 ATen launches with [N, L] temporaries.  Here one wave owns one row: the row's scores and relevance flags are
// staged in LDS and every lane counts, for its labels j, the labels ranked at or above j (all-pairs counting: exact
// for ties, no sort, O(L^2 / 64) LDS broadcast reads per row -- cheaper than sorting for the label counts these
// metrics see, L <= kMaxLabels).  Outputs one fp64 value per row (plus a validity flag for the ranking loss); the
// caller's sum keeps the fixed reduction order.
//
// mode 0 coverage:      #{k : p_k >= min(p_j + off_j)}, off_j = |global min| + 10 for irrelevant j (reference offset)
// mode 1 LRAP:          mean over relevant j of #{k relevant : p_k >= p_j} / #{k : p_k >= p_j}; 1 if no / all relevant
// mode 2 ranking loss:  (sum over relevant j of (L - inv_j) - n(n+1)/2) / (n (L - n)), inv_j = ascending position
//                       (ties by index, a stable argsort); valid iff 0 < n < L, else 0
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kRows = 4;  // waves (rows) per block
constexpr int kMaxLabels = 2048;

template <typename T>
__device__ __forceinline__ double to_f64(T v) {
  return static_cast<double>(to_f32(v));
}
template <>
__device__ __forceinline__ double to_f64<double>(double v) {
  return v;
}

// p + offset rounded like the reference's elementwise op in the input dtype (f32 / f16 / bf16 arithmetic)
template <typename T>
__device__ __forceinline__ double shifted(double p, double off) {
  return static_cast<double>(round_to<T>(static_cast<float>(p) + static_cast<float>(off)));
}
template <>
__device__ __forceinline__ double shifted<double>(double p, double off) {
  return p + off;
}

template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kRows * kWave) label_ranking_kernel(const scalar_t* __restrict__ preds,
                                                                      const target_t* __restrict__ target, long long M,
                                                                      int L, int mode,
                                                                      const scalar_t* __restrict__ gmin,
                                                                      double* __restrict__ out,
                                                                      uint8_t* __restrict__ valid) {
  extern __shared__ unsigned char smem[];
  const int wid = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  double* p = reinterpret_cast<double*>(smem) + static_cast<long long>(wid) * L;
  uint8_t* rel = reinterpret_cast<uint8_t*>(reinterpret_cast<double*>(smem) + kRows * L) + wid * L;
  const long long row = static_cast<long long>(blockIdx.x) * kRows + wid;
  const bool active = row < M;  // inactive waves still reach the barrier
  int nrel = 0;
  if (active) {
    const scalar_t* pr = preds + row * L;
    const target_t* tr = target + row * L;
    for (int j = lane; j < L; j += kWave) {
      p[j] = to_f64(pr[j]);
      // code 0: target 0, 1: relevant (target 1), 2: anything else (the ignore sentinel)
      const long long tv = static_cast<long long>(tr[j]);
      const int r = tv == 1 ? 1 : 0;
      rel[j] = static_cast<uint8_t>(tv == 0 ? 0 : (r ? 1 : 2));
      nrel += r;
    }
  }
  nrel = wave_sum(nrel);
  __syncthreads();
  if (!active) return;
  double acc = 0.0;
  if (mode == 0) {
    const double off = static_cast<double>(round_to<scalar_t>(fabsf(static_cast<float>(to_f64(gmin[0]))) + 10.f));
    double mn = INFINITY;
    // the reference shifts only target == 0 entries (ignored ones keep their sentinel score)
    for (int j = lane; j < L; j += kWave) mn = fmin(mn, rel[j] != 0 ? p[j] : shifted<scalar_t>(p[j], off));
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) mn = fmin(mn, __shfl_xor(mn, o, kWave));
    int cnt = 0;
    for (int j = lane; j < L; j += kWave) cnt += p[j] >= mn ? 1 : 0;
    acc = static_cast<double>(wave_sum(cnt));
  } else if (mode == 1) {
    double s = 0.0;
    for (int j = lane; j < L; j += kWave) {
      if (rel[j] != 1) continue;
      const double pj = p[j];
      int all = 0, rr = 0;
      for (int k = 0; k < L; ++k) {
        const int ge = p[k] >= pj ? 1 : 0;
        all += ge;
        rr += ge & (rel[k] == 1 ? 1 : 0);
      }
      s += static_cast<double>(rr) / static_cast<double>(all);
    }
    s = wave_sum(s);
    acc = (nrel == 0 || nrel == L) ? 1.0 : s / static_cast<double>(nrel);
  } else {
    long long s = 0;
    for (int j = lane; j < L; j += kWave) {
      if (rel[j] != 1) continue;
      const double pj = p[j];
      int inv = 0;  // ascending position: smaller scores, then equal scores at a smaller index
      for (int k = 0; k < L; ++k) inv += (p[k] < pj || (p[k] == pj && k < j)) ? 1 : 0;
      s += L - inv;
    }
    s = wave_sum_ll(s);
    const bool ok = nrel > 0 && nrel < L;
    acc = ok ? (static_cast<double>(s) - 0.5 * nrel * (nrel + 1)) / (static_cast<double>(nrel) * (L - nrel)) : 0.0;
    if (lane == 0) valid[row] = ok ? 1 : 0;
  }
  if (lane == 0) out[row] = acc;
}

}  // namespace

// preds [M, L] float (f32/f16/bf16), target [M, L] integer; gmin: 1-element tensor with the global min of preds
// (coverage only); out f64 [M]; valid u8 [M] (ranking loss).
void label_ranking(const at::Tensor& preds, const at::Tensor& target, int64_t mode, const at::Tensor& gmin,
                   at::Tensor out, at::Tensor valid) {
  TM_CHECK_CUDA(preds);
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&target, &gmin, &out, &valid})
    TM_SAME_DEVICE(preds, *t);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.dim() == 2 && target.sizes() == preds.sizes(), "label_ranking: preds / target [M, L]");
  const long long M = preds.size(0);
  const int L = static_cast<int>(preds.size(1));
  TORCH_CHECK(L >= 1 && L <= kMaxLabels, "label_ranking: 1 <= num_labels <= ", kMaxLabels);
  TORCH_CHECK(mode >= 0 && mode <= 2, "label_ranking: mode 0 coverage / 1 LRAP / 2 ranking loss");
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.numel() == M && out.is_contiguous(), "label_ranking: out f64 [M]");
  TORCH_CHECK(valid.scalar_type() == at::kByte && valid.numel() == M && valid.is_contiguous(),
              "label_ranking: valid u8 [M]");
  TORCH_CHECK(gmin.scalar_type() == preds.scalar_type() && gmin.numel() >= 1, "label_ranking: gmin");
  if (M == 0) return;
  const long long blocks = (M + kRows - 1) / kRows;
  TORCH_CHECK(blocks < (1LL << 31), "label_ranking: too many rows");
  const size_t lds = static_cast<size_t>(kRows) * L * (sizeof(double) + 1);
  TM_DISPATCH_FLOAT(preds.scalar_type(), "label_ranking", [&] {
    TM_DISPATCH_TARGET(target.scalar_type(), "label_ranking", [&] {
      hipLaunchKernelGGL((label_ranking_kernel<scalar_t, target_t>), dim3(static_cast<unsigned>(blocks)),
                         dim3(kRows * kWave), lds, stream(), preds.data_ptr<scalar_t>(), target.data_ptr<target_t>(),
                         M, L, static_cast<int>(mode), gmin.data_ptr<scalar_t>(), out.data_ptr<double>(),
                         valid.data_ptr<uint8_t>());
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("label_ranking(Tensor preds, Tensor target, int mode, Tensor gmin, Tensor(a!) out, Tensor(b!) valid) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("label_ranking", &label_ranking); }

}  // namespace tm_amd
