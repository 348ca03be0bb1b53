// Batched linear sum assignment on the device (PIT for many speakers; K31 in SURVEY.md §2.5).
//
// Reference (F/audio/pit.py:42-65): the [B, S, S] metric matrix goes to the host and scipy's
// `linear_sum_assignment` runs once per batch item.  Here one wave solves one problem with the Hungarian method in
// its O(S^3) potential / augmenting-path form (Kuhn-Munkres with row potentials u, column potentials v): each of the
// S augmentations scans the columns in parallel (lane j owns columns j, j+64, ...), the column minimum comes from a
// wave reduction (ties -> smallest column), and the potential update is one more parallel pass.  State lives in LDS
// (6 arrays of S+1 entries per wave); costs are read straight from the matrix in fp64.  Maximisation negates costs.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kMaxN = 256;

__device__ __forceinline__ void wave_argmin(double& v, int& j) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off, kWave);
    const int oj = __shfl_xor(j, off, kWave);
    if (ov < v || (ov == v && oj < j)) {
      v = ov;
      j = oj;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kWave) lsa_kernel(const T* __restrict__ cost, int n, bool maximize,
                                                    int64_t* __restrict__ assign) {
  __shared__ double u[kMaxN + 1], v[kMaxN + 1], minv[kMaxN + 1];
  __shared__ int p[kMaxN + 1], way[kMaxN + 1], used[kMaxN + 1];
  const int lane = threadIdx.x;
  const T* a = cost + static_cast<long long>(blockIdx.x) * n * n;
  const double sgn = maximize ? -1.0 : 1.0;
  for (int j = lane; j <= n; j += kWave) {
    u[j] = 0.0;
    v[j] = 0.0;
    p[j] = 0;
    way[j] = 0;
  }
  __syncthreads();
  for (int i = 1; i <= n; ++i) {
    for (int j = lane; j <= n; j += kWave) {
      minv[j] = INFINITY;
      used[j] = 0;
    }
    if (lane == 0) p[0] = i;
    __syncthreads();
    int j0 = 0;
    while (true) {
      if (lane == 0) used[j0] = 1;
      __syncthreads();
      const int i0 = p[j0];
      double best = INFINITY;
      int bj = 0x7fffffff;
      for (int j = lane + 1; j <= n; j += kWave) {
        if (used[j]) continue;
        const double cur = sgn * static_cast<double>(a[(i0 - 1) * n + (j - 1)]) - u[i0] - v[j];
        if (cur < minv[j]) {
          minv[j] = cur;
          way[j] = j0;
        }
        if (minv[j] < best || (minv[j] == best && j < bj)) {
          best = minv[j];
          bj = j;
        }
      }
      wave_argmin(best, bj);
      const double delta = best;
      const int j1 = bj;
      __syncthreads();
      for (int j = lane; j <= n; j += kWave) {
        if (used[j]) {
          u[p[j]] += delta;
          v[j] -= delta;
        } else {
          minv[j] -= delta;
        }
      }
      __syncthreads();
      j0 = j1;
      if (j0 < 0 || j0 > n || p[j0] == 0) break;  // free column reached (bounds guard: NaN costs)
    }
    if (lane == 0 && j0 >= 1 && j0 <= n) {  // augment along the alternating path
      int j = j0;
      while (j != 0) {
        const int jp = way[j];
        p[j] = p[jp];
        j = jp;
      }
    }
    __syncthreads();
  }
  for (int j = lane + 1; j <= n; j += kWave) {
    const int row = p[j];
    if (row >= 1) assign[static_cast<long long>(blockIdx.x) * n + (row - 1)] = j - 1;
  }
}

}  // namespace

// cost: [B, n, n] (f32 / f64) on the device; assign: int64 [B, n] -> column of each row in an optimal assignment.
void linear_sum_assignment(const at::Tensor& cost, bool maximize, at::Tensor assign) {
  TM_CHECK_CUDA(cost);
  TM_SAME_DEVICE(cost, assign);
  TM_CHECK_CONTIG(cost);
  TORCH_CHECK(cost.dim() == 3 && cost.size(1) == cost.size(2), "linear_sum_assignment: cost must be [B, n, n]");
  const int n = static_cast<int>(cost.size(1));
  TORCH_CHECK(n >= 1 && n <= kMaxN, "linear_sum_assignment: 1 <= n <= ", kMaxN);
  TORCH_CHECK(assign.scalar_type() == at::kLong && assign.is_contiguous() && assign.numel() == cost.size(0) * n,
              "linear_sum_assignment: assign must be int64 [B, n]");
  const long long B = cost.size(0);
  if (B == 0) return;
  TORCH_CHECK(B < (1LL << 31), "linear_sum_assignment: batch too large");
  if (cost.scalar_type() == at::kDouble)
    hipLaunchKernelGGL(lsa_kernel<double>, dim3(static_cast<unsigned>(B)), dim3(kWave), 0, stream(),
                       cost.data_ptr<double>(), n, maximize, assign.data_ptr<int64_t>());
  else if (cost.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(lsa_kernel<float>, dim3(static_cast<unsigned>(B)), dim3(kWave), 0, stream(),
                       cost.data_ptr<float>(), n, maximize, assign.data_ptr<int64_t>());
  else
    TORCH_CHECK(false, "linear_sum_assignment: f32 / f64 costs");
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("linear_sum_assignment(Tensor cost, bool maximize, Tensor(a!) assign) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("linear_sum_assignment", &linear_sum_assignment); }

}  // namespace tm_amd
