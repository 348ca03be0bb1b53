// Batched symmetric-Toeplitz solve  T(r) x = b  by Levinson recursion (SDR distortion-filter solve, SURVEY.md
// audio plan: levinson.hip).
//
// The reference materialises the [L, L] Toeplitz matrix of every sample and calls a dense LU solve
// (F/audio/sdr.py:188-189): O(L^3) flops and an [B, L, L] fp64 buffer.  Levinson uses the Toeplitz structure: L
// steps, each two length-k dot products and two length-k vector updates -> O(L^2) flops, O(L) memory.  One 64-lane
// wave owns one system; r, the forward vector (double-buffered) and the solution live in LDS, every step is two
// fused wave reductions with no block barrier.  fp64 throughout (the reference solves in fp64).
#include "common/tm_common.h"

namespace tm_amd {
namespace {

template <int WAVES>
__global__ void __launch_bounds__(kWave* WAVES)
    levinson_kernel(const double* __restrict__ r, const double* __restrict__ b, double* __restrict__ x_out, int nsys,
                    int len) {
  extern __shared__ double lds[];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  const int sys = blockIdx.x * WAVES + wave;
  if (sys >= nsys) return;  // whole wave leaves; no block barriers below
  double* rs = lds + static_cast<size_t>(wave) * 4 * len;
  double* f = rs + len;
  double* fn = f + len;
  double* x = fn + len;
  const double* rg = r + static_cast<long long>(sys) * len;
  const double* bg = b + static_cast<long long>(sys) * len;
  for (int i = lane; i < len; i += kWave) rs[i] = rg[i];
  __builtin_amdgcn_wave_barrier();
  const double r0 = rs[0];
  if (lane == 0) {
    f[0] = 1.0 / r0;
    x[0] = bg[0] / r0;
  }
  __builtin_amdgcn_wave_barrier();
  for (int k = 1; k < len; ++k) {
    double ef = 0.0, ex = 0.0;
    for (int i = lane; i < k; i += kWave) {
      const double rk = rs[k - i];
      ef = fma(rk, f[i], ef);
      ex = fma(rk, x[i], ex);
    }
    ef = wave_sum(ef);
    ex = wave_sum(ex);
    const double inv = 1.0 / (1.0 - ef * ef);
    for (int i = lane; i <= k; i += kWave) {
      const double fe = i < k ? f[i] : 0.0;
      const double be = i >= 1 ? f[k - i] : 0.0;
      fn[i] = (fe - ef * be) * inv;
    }
    __builtin_amdgcn_wave_barrier();
    const double mu = bg[k] - ex;
    for (int i = lane; i <= k; i += kWave) x[i] = (i < k ? x[i] : 0.0) + mu * fn[k - i];
    __builtin_amdgcn_wave_barrier();
    double* t = f;
    f = fn;
    fn = t;
  }
  double* xo = x_out + static_cast<long long>(sys) * len;
  for (int i = lane; i < len; i += kWave) xo[i] = x[i];
}

}  // namespace

// x[s] = T(r[s])^{-1} b[s] for every system s; r, b, x: [S, L] fp64 contiguous.
void toeplitz_solve(const at::Tensor& r, const at::Tensor& b, at::Tensor x) {
  TM_CHECK_CUDA(r);
  TM_CHECK_CONTIG(r);
  TM_CHECK_CONTIG(b);
  TM_CHECK_CONTIG(x);
  TORCH_CHECK(r.scalar_type() == at::kDouble && b.scalar_type() == at::kDouble && x.scalar_type() == at::kDouble,
              "toeplitz_solve: fp64 tensors expected");
  TORCH_CHECK(r.dim() == 2 && b.sizes() == r.sizes() && x.sizes() == r.sizes(), "toeplitz_solve: shapes [S, L]");
  const int nsys = static_cast<int>(r.size(0)), len = static_cast<int>(r.size(1));
  if (nsys == 0 || len == 0) return;
  const size_t per_wave = static_cast<size_t>(4) * len * sizeof(double);
  TORCH_CHECK(per_wave <= 160 * 1024, "toeplitz_solve: filter length ", len, " too long for the LDS kernel");
  auto go = [&](auto waves_tag) {
    constexpr int W = decltype(waves_tag)::value;
    const size_t lds = per_wave * W;
    const void* fn = reinterpret_cast<const void*>(&levinson_kernel<W>);
    if (lds > 64 * 1024)
      TORCH_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) ==
                      hipSuccess,
                  "toeplitz_solve: cannot raise LDS limit");
    hipLaunchKernelGGL((levinson_kernel<W>), dim3((nsys + W - 1) / W), dim3(kWave * W), lds, stream(),
                       r.data_ptr<double>(), b.data_ptr<double>(), x.data_ptr<double>(), nsys, len);
  };
  if (per_wave * 2 <= 64 * 1024)
    go(std::integral_constant<int, 2>{});
  else
    go(std::integral_constant<int, 1>{});
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("toeplitz_solve(Tensor r, Tensor b, Tensor(a!) x) -> ()"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("toeplitz_solve", &toeplitz_solve); }

}  // namespace tm_amd
