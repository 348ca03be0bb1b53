// Pairwise distance matrices  D[i, j] = dist(x_i, y_j)  for x [N, d], y [M, d]  (K19 in SURVEY.md).
//
// The reference materialises the full [N, M, d] difference tensor for the L1 / Lp cases (F/pairwise/manhattan.py:39,
// F/pairwise/minkowski.py:43) and uses the fp64 norm-expansion GEMM for L2 (F/pairwise/euclidean.py:37-41).  Here one
// LDS-tiled VALU kernel evaluates the difference form directly for every metric:
//   * 64 x 64 output tile per 256-thread block (4 x 4 register tile per thread, 16 lanes share an x row so the stores
//     of a row are one 256 B transaction), k-chunks of 32 staged transposed in LDS, next chunk prefetched into
//     registers while the current one is consumed;
//   * the difference form has no catastrophic cancellation, so fp32 accumulation matches the reference's fp64 norm
//     trick to ~1e-6 relative while running at the fp32 VALU rate;  fp64 inputs accumulate in fp64;
//   * epilogue fuses the root (sqrt / ^(1/p)), zero_diagonal and -- for reduction='sum'/'mean' -- the row reduction:
//     each column tile writes one deterministic partial per row, so a reduced call never materialises [N, M];
//   * tile ids are remapped so each of the 8 XCDs works on a contiguous band of row tiles (its own L2 keeps them).
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBM = 64, kBN = 64, kBK = 32, kThreads = 256;
constexpr int kPad = 4;

enum Metric : int { kL1 = 0, kL2 = 1, kLp = 2, kLpInt = 3 };

template <typename T, typename A>
__device__ __forceinline__ A load_as(const T* p) {
  if constexpr (std::is_same<A, double>::value)
    return static_cast<double>(*p);
  else
    return to_f32<T>(*p);
}

template <typename A>
__device__ __forceinline__ A pw_pow(A v, A p) {
  if constexpr (std::is_same<A, double>::value)
    return v == 0.0 ? 0.0 : pow(v, p);
  else
    return v == 0.0f ? 0.0f : exp2f(p * log2f(v));
}

template <typename A, int MET>
__device__ __forceinline__ A accum(A acc, A d, A p) {
  if constexpr (MET == kL1) return acc + (d < A(0) ? -d : d);
  else if constexpr (MET == kL2) return fma(d, d, acc);
  else if constexpr (MET == kLp) return acc + pw_pow<A>(d < A(0) ? -d : d, p);
  else {
    // integer exponent 1..15 by binary powering; `ip` is wave-uniform so the branches are scalar
    const int ip = static_cast<int>(p);
    A b = d < A(0) ? -d : d;
    A r = (ip & 1) ? b : A(1);
    b = b * b;
    if (ip & 2) r *= b;
    b = b * b;
    if (ip & 4) r *= b;
    b = b * b;
    if (ip & 8) r *= b;
    return acc + r;
  }
}

template <typename A, int MET>
__device__ __forceinline__ A finish(A v, A inv_p) {
  if constexpr (MET == kL1) return v;
  else if constexpr (MET == kL2) return sqrt(v);
  else return pw_pow<A>(v, inv_p);  // kLp, kLpInt
}

template <typename T, typename A, int MET>
__global__ void __launch_bounds__(kThreads) pairwise_kernel(const T* __restrict__ x, const T* __restrict__ y, int n,
                                                            int m, int d, A p, int zero_diag, int reduce,
                                                            int tiles_n, int tiles_m, A* __restrict__ out) {
  __shared__ A xs[kBK][kBM + kPad];
  __shared__ A ys[kBK][kBN + kPad];

  // XCD-aware tile mapping: hardware dispatches linear block ids round-robin over 8 XCDs; give XCD k the k-th
  // contiguous band of (row-major) tiles so neighbouring tiles that share x / y rows hit the same L2.
  const int total = tiles_n * tiles_m;
  int bid = blockIdx.x;
  if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);
  const int tile_r = bid / tiles_m, tile_c = bid % tiles_m;
  const int r0 = tile_r * kBM, c0 = tile_c * kBN;

  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;

  A acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = A(0);

  // each thread stages 8 x-elements and 8 y-elements per chunk: idx = tid + 256 * e -> (row = idx / 32, k = idx % 32)
  A px[8], py[8];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = tid + kThreads * e, r = idx >> 5, k = k0 + (idx & 31);
      const int gx = r0 + r, gy = c0 + r;
      px[e] = (gx < n && k < d) ? load_as<T, A>(x + static_cast<long long>(gx) * d + k) : A(0);
      py[e] = (gy < m && k < d) ? load_as<T, A>(y + static_cast<long long>(gy) * d + k) : A(0);
    }
  };
  fetch(0);
  for (int k0 = 0; k0 < d; k0 += kBK) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = tid + kThreads * e, r = idx >> 5, k = idx & 31;
      xs[k][r] = px[e];
      ys[k][r] = py[e];
    }
    __syncthreads();
    if (k0 + kBK < d) fetch(k0 + kBK);
    const int kn = min(kBK, d - k0);
#pragma unroll 8
    for (int k = 0; k < kn; ++k) {
      A a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = xs[k][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = ys[k][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = accum<A, MET>(acc[i][j], a[i] - b[j], p);
    }
  }

  const A inv_p = A(1) / p;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = r0 + ty * 4 + i;
    A rsum = A(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = c0 + tx * 4 + j;
      A v = finish<A, MET>(acc[i][j], inv_p);
      if (zero_diag && row == col) v = A(0);
      if (row < n && col < m) {
        if (reduce)
          rsum += v;
        else
          out[static_cast<long long>(row) * m + col] = v;
      }
    }
    if (reduce) {
      // the 16 lanes with equal ty hold the 64 columns of this row: reduce inside the 16-lane group
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) rsum += __shfl_xor(rsum, off, 16);
      if (tx == 0 && row < n) out[static_cast<long long>(row) * tiles_m + tile_c] = rsum;
    }
  }
}

template <typename T, typename A>
void launch(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, int metric, double p, bool zero_diag,
            bool reduce) {
  const int n = x.size(0), m = y.size(0), d = x.size(1);
  const int tn = (n + kBM - 1) / kBM, tm = (m + kBN - 1) / kBN;
  const long long blocks = static_cast<long long>(tn) * tm;
  TORCH_CHECK(blocks < (1LL << 31), "pairwise_distance: problem too large");
  auto* o = out.data_ptr<A>();
  const A pp = static_cast<A>(p);
#define TM_PW_LAUNCH(MET)                                                                                     \
  hipLaunchKernelGGL((pairwise_kernel<T, A, MET>), dim3(static_cast<unsigned>(blocks)), dim3(kThreads), 0,  \
                     stream(), x.data_ptr<T>(), y.data_ptr<T>(), n, m, d, pp, zero_diag ? 1 : 0, reduce ? 1 : 0, \
                     tn, tm, o)
  if (metric == kL1)
    TM_PW_LAUNCH(kL1);
  else if (metric == kL2)
    TM_PW_LAUNCH(kL2);
  else if (metric == kLp)
    TM_PW_LAUNCH(kLp);
  else
    TM_PW_LAUNCH(kLpInt);
#undef TM_PW_LAUNCH
}

}  // namespace

// out: [N, M] (reduce == false) or per-column-tile row partials [N, ceil(M / 64)] (reduce == true); fp64 for fp64
// inputs, fp32 otherwise.
void pairwise_distance(const at::Tensor& x, const at::Tensor& y, at::Tensor out, int64_t metric, double p,
                       bool zero_diag, bool reduce) {
  TM_CHECK_CUDA(x);
  TM_SAME_DEVICE(x, y);
  TM_CHECK_CONTIG(x);
  TM_CHECK_CONTIG(y);
  TM_CHECK_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && y.dim() == 2 && x.size(1) == y.size(1), "pairwise_distance: bad shapes");
  TORCH_CHECK(x.scalar_type() == y.scalar_type(), "pairwise_distance: dtype mismatch");
  TORCH_CHECK(metric >= 0 && metric <= 3, "pairwise_distance: bad metric");
  TORCH_CHECK(metric != kLpInt || (p >= 1 && p <= 15 && p == static_cast<double>(static_cast<int>(p))),
              "pairwise_distance: integer exponent must be in [1, 15]");
  const int64_t cols = reduce ? (y.size(0) + kBN - 1) / kBN : y.size(0);
  TORCH_CHECK(out.size(0) == x.size(0) && out.size(1) == cols, "pairwise_distance: bad output shape");
  if (x.size(0) == 0 || y.size(0) == 0) return;
  const bool f64 = x.scalar_type() == at::kDouble;
  TORCH_CHECK(out.scalar_type() == (f64 ? at::kDouble : at::kFloat), "pairwise_distance: bad output dtype");
  TM_DISPATCH_FLOAT(x.scalar_type(), "pairwise_distance", [&] {
    if constexpr (std::is_same<scalar_t, double>::value)
      launch<double, double>(x, y, out, static_cast<int>(metric), p, zero_diag, reduce);
    else
      launch<scalar_t, float>(x, y, out, static_cast<int>(metric), p, zero_diag, reduce);
  });
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("pairwise_distance(Tensor x, Tensor y, Tensor(a!) out, int metric, float p, bool zero_diag, bool reduce) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("pairwise_distance", &pairwise_distance); }

}  // namespace tm_amd
