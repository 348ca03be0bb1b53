// Expected mutual information under the hypergeometric model (adjusted_mutual_info_score's EMI term).
//
//   EMI = sum_{i,j} sum_{n = max(1, a_i + b_j - N)}^{min(a_i, b_j)} n/N * log(N n / (a_i b_j)) * exp(g(n))
//   g(n) = lnG(a_i+1) + lnG(b_j+1) + lnG(N-a_i+1) + lnG(N-b_j+1) - lnG(N+1)
//          - lnG(n+1) - lnG(a_i-n+1) - lnG(b_j-n+1) - lnG(N-a_i-b_j+n+1)
//
// The reference (F/clustering/utils.py calculate_expected_mutual_information via torch.lgamma on every term;
// scikit-learn's Cython loop) evaluates nine log-gamma calls per term; a torch formulation also materialises every
// (i, j, n) term -- ~N x #clusters terms, 39 ms at N = 1e7 on MI355X.  Here a thread owns kRun consecutive n of one
// (i, j) pair: g at its first n from lgamma, every next weight by the exact recurrence
//   exp(g(n+1)) = exp(g(n)) (a-n)(b-n) / ((n+1)(N-a-b+n+1))
// (one log per term, fp64; the additive form with four logs and an exp per term took 3.2 ms at N = 1e7), nothing
// materialised.  Small tables: grid y = pair, x = run-blocks over the longest
// pair's range.  Any larger table: blocks of 256 consecutive pairs deal their runs out to their threads.  Each block
// writes one partial (deterministic: summed by the caller).
#include "../common/tm_common.h"
#include "sort/sortscan.h"

namespace tm_amd {
namespace {

constexpr int kEmiThreads = 256;
constexpr int kRun = 32;  // consecutive terms per thread (the recurrence resets from lgamma every kRun terms)

// kRun terms n = first, first + 1, ... (<= hi) of one (A, B) pair.  The hypergeometric weight p(n) = exp(g(n)) is
// carried multiplicatively, p(n + 1) = p(n) (A - n)(B - n) / ((n + 1)(N - A - B + n + 1)): one log (of n) per term
// instead of four logs and an exp (the additive form of the recurrence); it restarts from lgamma every kRun terms.
__device__ __forceinline__ double emi_run(double A, double B, double N, double lgN1, double first, double hi) {
  const double cst = lgamma(A + 1.0) + lgamma(B + 1.0) + lgamma(N - A + 1.0) + lgamma(N - B + 1.0) - lgN1;
  const double lab = log(A) + log(B), lN = log(N), rest = N - A - B;
  double n = first, acc = 0.0;
  double p = exp(cst - lgamma(n + 1.0) - lgamma(A - n + 1.0) - lgamma(B - n + 1.0) - lgamma(rest + n + 1.0));
  for (int k = 0; k < kRun && n <= hi; ++k) {
    acc += (n / N) * (lN + log(n) - lab) * p;
    p *= ((A - n) * (B - n)) / ((n + 1.0) * (rest + n + 1.0));
    n += 1.0;
  }
  return acc;
}

__device__ __forceinline__ void emi_block_store(double acc, double* __restrict__ dst) {
  __shared__ double red[kEmiThreads / kWave];
  acc = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < kEmiThreads / kWave; ++w) s += red[w];
    *dst = s;
  }
}

// small tables (< 65536 pairs): grid y = pair, x = run-blocks over the longest pair's range
__global__ void __launch_bounds__(kEmiThreads) emi_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                         int C, double N, double lgN1, double* __restrict__ partial,
                                                         int nblk) {
  const int pair = blockIdx.y;
  const double A = a[pair / C], B = b[pair % C];
  const double lo = fmax(1.0, A + B - N), hi = fmin(A, B);  // inclusive range of n
  const double first = lo + (static_cast<double>(blockIdx.x) * kEmiThreads + threadIdx.x) * kRun;
  double acc = 0.0;
  if (A > 0.0 && B > 0.0 && first <= hi) acc = emi_run(A, B, N, lgN1, first, hi);
  emi_block_store(acc, partial + static_cast<long long>(pair) * nblk + blockIdx.x);
}

// any table size: a block owns kEmiThreads consecutive pairs, scans their run counts in LDS and deals the block's
// runs out to its threads (a binary search over the 256-entry prefix finds a run's pair); one partial per block
__global__ void __launch_bounds__(kEmiThreads) emi_tile_kernel(const double* __restrict__ a,
                                                              const double* __restrict__ b, long long pairs, int C,
                                                              double N, double lgN1, double* __restrict__ partial) {
  __shared__ long long pre[kEmiThreads];
  __shared__ long long scan_lds[kEmiThreads / kWave];
  const long long pair0 = static_cast<long long>(blockIdx.x) * kEmiThreads;
  const long long pair = pair0 + threadIdx.x;
  long long runs = 0;
  if (pair < pairs) {
    const double A = a[pair / C], B = b[pair % C];
    const double lo = fmax(1.0, A + B - N), hi = fmin(A, B);
    if (A > 0.0 && B > 0.0 && hi >= lo) runs = static_cast<long long>((hi - lo) / kRun) + 1;
  }
  long long excl, total;
  pre[threadIdx.x] = sortscan::block_inclusive_scan<kEmiThreads / kWave>(
      runs, [](long long x, long long y) { return x + y; }, 0LL, scan_lds, excl, total);
  __syncthreads();
  double acc = 0.0;
  for (long long t = threadIdx.x; t < total; t += kEmiThreads) {
    int l = 0, h = kEmiThreads - 1;  // the first slot whose inclusive prefix exceeds t
    while (l < h) {
      const int mid = (l + h) >> 1;
      if (pre[mid] > t) h = mid;
      else l = mid + 1;
    }
    const long long p = pair0 + l;
    const long long k = t - (l ? pre[l - 1] : 0);
    const double A = a[p / C], B = b[p % C];
    const double lo = fmax(1.0, A + B - N), hi = fmin(A, B);
    acc += emi_run(A, B, N, lgN1, lo + static_cast<double>(k) * kRun, hi);
  }
  emi_block_store(acc, partial + blockIdx.x);
}

}  // namespace

// a [R], b [C]: fp64 cluster sizes (row / column sums of the contingency table); n: samples.  Returns the fp64 EMI
// (a 0-d tensor on the device).
at::Tensor expected_mutual_info(const at::Tensor& a, const at::Tensor& b, double n) {
  TM_CHECK_CUDA(a);
  TM_SAME_DEVICE(a, b);
  TORCH_CHECK(a.scalar_type() == at::kDouble && b.scalar_type() == at::kDouble && a.dim() == 1 && b.dim() == 1 &&
                  a.is_contiguous() && b.is_contiguous(),
              "expected_mutual_info: fp64 1-D contiguous cluster sizes");
  TORCH_CHECK(n >= 1.0 && n < 9.0e15, "expected_mutual_info: bad sample count");
  const long long R = a.numel(), C = b.numel();
  TORCH_CHECK(R >= 1 && C >= 1 && C < (1LL << 31), "expected_mutual_info: empty or oversized cluster sizes");
  const long long pairs = R * C;
  if (pairs >= 65536) {
    const long long nb = (pairs + kEmiThreads - 1) / kEmiThreads;
    TORCH_CHECK(nb < (1LL << 31), "expected_mutual_info: too many cluster pairs");
    at::Tensor partial = at::empty({nb}, a.options());
    hipLaunchKernelGGL(emi_tile_kernel, dim3(static_cast<unsigned>(nb)), dim3(kEmiThreads), 0, stream(),
                       a.data_ptr<double>(), b.data_ptr<double>(), pairs, static_cast<int>(C), n,
                       std::lgamma(n + 1.0), partial.data_ptr<double>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return partial.sum();
  }
  // the longest range any pair can have: min(max a, max b) <= n terms
  const double longest = std::min(a.max().item<double>(), b.max().item<double>());
  const long long per_blk = static_cast<long long>(kEmiThreads) * kRun;
  const int nblk = static_cast<int>(std::max<long long>(1, (static_cast<long long>(longest) + per_blk - 1) / per_blk));
  TORCH_CHECK(nblk < (1 << 30), "expected_mutual_info: range too long");
  at::Tensor partial = at::empty({R * C, nblk}, a.options());
  hipLaunchKernelGGL(emi_kernel, dim3(nblk, static_cast<unsigned>(R * C)), dim3(kEmiThreads), 0, stream(),
                     a.data_ptr<double>(), b.data_ptr<double>(), static_cast<int>(C), n, std::lgamma(n + 1.0),
                     partial.data_ptr<double>(), nblk);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return partial.sum();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("expected_mutual_info(Tensor a, Tensor b, float n) -> Tensor"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("expected_mutual_info", &expected_mutual_info); }

}  // namespace tm_amd
