// Statistics of a batch of contingency tables for the nominal association metrics.
//
// Reference: F/nominal/utils.py:34-59 (`_compute_expected_freqs` einsum, chi^2 with the scipy Yates correction,
// `_drop_empty_rows_and_cols` boolean indexing) and F/nominal/theils_u.py:28-62 (conditional entropy with masked logs),
// evaluated per table, per pair of columns in the `*_matrix` variants.  Here ONE block per table computes, in fp64:
//   [0] n   [1] r (non-empty rows)   [2] c (non-empty columns)
//   [3] chi^2 over the non-empty rows / columns            [4] the same with the Yates correction (+-0.5 toward the
//       expected count, scipy semantics; the caller uses it when (r-1)(c-1) == 1)
//   [5] sum p_xy log(p_y / p_xy)  (Theil's U: -H(X|Y))     [6] H(X) = -sum p_x log p_x   [7] 0
// Row sums: one wave per row (coalesced lanes); column sums: one thread per column; margins live in LDS (K <= 1024),
// so the table is read three times from L2 and nothing of size K x K is written.  Empty rows / columns are masked,
// not dropped: the statistics equal those of the compacted table.
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256, kMaxK = 1024;

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kThreads / 64; ++w) s += red[w];
  return s;
}

__global__ void __launch_bounds__(kThreads) table_stats_kernel(const int64_t* __restrict__ cm, int K,
                                                               double* __restrict__ out) {
  __shared__ double rs[kMaxK], cs[kMaxK];
  __shared__ double red[kThreads / 64];
  const int64_t* T = cm + static_cast<long long>(blockIdx.x) * K * K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = wave; i < K; i += kThreads / 64) {
    double s = 0.0;
    for (int j = lane; j < K; j += 64) s += static_cast<double>(T[static_cast<long long>(i) * K + j]);
    s = wave_sum(s);
    if (lane == 0) rs[i] = s;
  }
  for (int j = tid; j < K; j += kThreads) {
    double s = 0.0;
    for (int i = 0; i < K; ++i) s += static_cast<double>(T[static_cast<long long>(i) * K + j]);
    cs[j] = s;
  }
  __syncthreads();
  double n_part = 0.0, r_part = 0.0, c_part = 0.0;
  for (int i = tid; i < K; i += kThreads) {
    n_part += rs[i];
    r_part += rs[i] > 0.0 ? 1.0 : 0.0;
    c_part += cs[i] > 0.0 ? 1.0 : 0.0;
  }
  const double n = block_sum(n_part, red);
  const double r = block_sum(r_part, red);
  const double c = block_sum(c_part, red);
  const double inv_n = n > 0.0 ? 1.0 / n : 0.0;
  double chi = 0.0, chi_y = 0.0, sxy = 0.0;
  const long long kk = static_cast<long long>(K) * K;
  for (long long e = tid; e < kk; e += kThreads) {
    const int i = static_cast<int>(e / K), j = static_cast<int>(e - static_cast<long long>(i) * K);
    const double ri = rs[i], cj = cs[j];
    if (ri <= 0.0 || cj <= 0.0) continue;
    const double o = static_cast<double>(T[e]);
    const double ex = ri * cj * inv_n;
    const double d = o - ex;
    chi += d * d / ex;
    const double oy = o + (ex > o ? 0.5 : (ex < o ? -0.5 : 0.0));
    chi_y += (oy - ex) * (oy - ex) / ex;
    if (o > 0.0) {
      const double pxy = o * inv_n;
      sxy += pxy * log(ri / o);  // log(p_y / p_xy) = log(r_i / o)
    }
  }
  double hx = 0.0;
  for (int j = tid; j < K; j += kThreads) {
    if (cs[j] > 0.0) {
      const double p = cs[j] * inv_n;
      hx -= p * log(p);
    }
  }
  chi = block_sum(chi, red);
  chi_y = block_sum(chi_y, red);
  sxy = block_sum(sxy, red);
  hx = block_sum(hx, red);
  if (tid == 0) {
    double* o = out + static_cast<long long>(blockIdx.x) * 8;
    o[0] = n;
    o[1] = r;
    o[2] = c;
    o[3] = chi;
    o[4] = chi_y;
    o[5] = sxy;
    o[6] = hx;
    o[7] = 0.0;
  }
}

}  // namespace

// cm: int64 [B, K, K] contiguous (K <= 1024) -> out: fp64 [B, 8] (see the header)
void nominal_table_stats(const at::Tensor& cm, at::Tensor out) {
  TM_CHECK_CUDA(cm);
  TM_SAME_DEVICE(cm, out);
  TM_CHECK_CONTIG(cm);
  TORCH_CHECK(cm.scalar_type() == at::kLong && cm.dim() == 3 && cm.size(1) == cm.size(2),
              "nominal_table_stats: cm must be int64 [B, K, K]");
  const long long B = cm.size(0), K = cm.size(1);
  TORCH_CHECK(K >= 1 && K <= kMaxK, "nominal_table_stats: 1 <= K <= ", kMaxK);
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.is_contiguous() && out.numel() == B * 8,
              "nominal_table_stats: out must be fp64 [B, 8]");
  TORCH_CHECK(B < (1LL << 31), "nominal_table_stats: too many tables");
  if (B == 0) return;
  hipLaunchKernelGGL(table_stats_kernel, dim3(static_cast<unsigned>(B)), dim3(kThreads), 0, stream(),
                     cm.data_ptr<int64_t>(), static_cast<int>(K), out.data_ptr<double>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("nominal_table_stats(Tensor cm, Tensor(a!) out) -> ()"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("nominal_table_stats", &nominal_table_stats); }

}  // namespace tm_amd
