// SNR / SI-SDR / SI-SNR / C-SI-SNR / SA-SDR in one launch (K30 in SURVEY.md §2.5).
//
// Reference (F/audio/snr.py, F/audio/sdr.py:201-305): per call ~8-12 ATen launches over the [rows, L] signals
// (optional mean subtraction, products, three sums, the projection alpha * target, the noise, two more sums, log10).
// Here one 256-thread block owns one row and makes up to three passes over it from L2: segment means (zero_mean),
// the projection sums (scale-invariant kinds), then the signal / noise energies with the noise formed explicitly
// (no E[x^2] - E[x]^2 style cancellation at high SDR).  Accumulation is fp64 whatever the input dtype.
//
// Rows are contiguous [L] slices; `seg` splits a row into L/seg segments centred separately (SA-SDR's per-speaker
// zero_mean over a flattened (speaker, time) row); for every other kind seg = L.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kThreads / kWave; ++w) s += red[w];
  return s;
}

template <typename T>
__device__ __forceinline__ double ld(const T* p, long long i) {
  if constexpr (std::is_same<T, double>::value) return p[i];
  else return static_cast<double>(to_f32(p[i]));
}

template <typename T>
__global__ void __launch_bounds__(kThreads) snr_rows_kernel(const T* __restrict__ preds, const T* __restrict__ target,
                                                            long long L, long long seg, int scale_invariant,
                                                            int zero_mean, double eps, T* __restrict__ out) {
  extern __shared__ double mean_sm[];  // [2 * nseg]: per-segment means of preds / target (zero_mean)
  __shared__ double red[kThreads / kWave];
  const long long row = blockIdx.x;
  const T* p = preds + row * L;
  const T* t = target + row * L;
  const long long nseg = L / seg;
  if (zero_mean) {
    for (long long s = 0; s < nseg; ++s) {
      double sp = 0.0, st = 0.0;
      for (long long i = s * seg + threadIdx.x; i < (s + 1) * seg; i += kThreads) {
        sp += ld(p, i);
        st += ld(t, i);
      }
      sp = block_sum_d(sp, red);
      st = block_sum_d(st, red);
      if (threadIdx.x == 0) {
        mean_sm[2 * s] = sp / static_cast<double>(seg);
        mean_sm[2 * s + 1] = st / static_cast<double>(seg);
      }
    }
    __syncthreads();
  }
  auto centred = [&](long long i, double& pv, double& tv) {
    pv = ld(p, i);
    tv = ld(t, i);
    if (zero_mean) {
      const long long s = i / seg;
      pv -= mean_sm[2 * s];
      tv -= mean_sm[2 * s + 1];
    }
  };
  double alpha = 1.0;
  if (scale_invariant) {
    double spt = 0.0, stt = 0.0;
    for (long long i = threadIdx.x; i < L; i += kThreads) {
      double pv, tv;
      centred(i, pv, tv);
      spt += pv * tv;
      stt += tv * tv;
    }
    spt = block_sum_d(spt, red);
    stt = block_sum_d(stt, red);
    alpha = (spt + eps) / (stt + eps);
  }
  double sig = 0.0, noise = 0.0;
  for (long long i = threadIdx.x; i < L; i += kThreads) {
    double pv, tv;
    centred(i, pv, tv);
    const double s = alpha * tv;
    const double n = s - pv;
    sig += s * s;
    noise += n * n;
  }
  sig = block_sum_d(sig, red);
  noise = block_sum_d(noise, red);
  if (threadIdx.x == 0) {
    const double db = 10.0 * log10((sig + eps) / (noise + eps));
    if constexpr (std::is_same<T, double>::value) out[row] = db;
    else out[row] = static_cast<T>(static_cast<float>(db));
  }
}

}  // namespace

// preds / target: contiguous [rows, L] (same dtype, f32 / f64 / f16 / bf16); out: [rows] in that dtype.
// scale_invariant: SI-SDR / SI-SNR / C-SI-SNR / SA-SDR projection; seg: zero_mean segment length (divides L).
void snr_rows(const at::Tensor& preds, const at::Tensor& target, at::Tensor out, int64_t seg, bool scale_invariant,
              bool zero_mean, double eps) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, out);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TM_CHECK_CONTIG(out);
  TORCH_CHECK(preds.dim() == 2 && target.sizes() == preds.sizes() && target.scalar_type() == preds.scalar_type(),
              "snr_rows: preds / target must be [rows, L] of one dtype");
  const long long rows = preds.size(0), L = preds.size(1);
  TORCH_CHECK(out.numel() == rows && out.scalar_type() == preds.scalar_type(), "snr_rows: out must be [rows]");
  TORCH_CHECK(L >= 1 && seg >= 1 && L % seg == 0, "snr_rows: seg must divide L");
  const long long nseg = L / seg;
  const size_t lds = zero_mean ? static_cast<size_t>(2 * nseg) * sizeof(double) : 0;
  TORCH_CHECK(lds <= 64 * 1024, "snr_rows: too many zero-mean segments per row");
  if (rows == 0) return;
  TORCH_CHECK(rows < (1LL << 31), "snr_rows: too many rows");
  TM_DISPATCH_FLOAT(preds.scalar_type(), "snr_rows", [&] {
    hipLaunchKernelGGL((snr_rows_kernel<scalar_t>), dim3(static_cast<unsigned>(rows)), dim3(kThreads), lds, stream(),
                       reinterpret_cast<const scalar_t*>(preds.data_ptr()),
                       reinterpret_cast<const scalar_t*>(target.data_ptr()), L, static_cast<long long>(seg),
                       scale_invariant ? 1 : 0, zero_mean ? 1 : 0, eps, reinterpret_cast<scalar_t*>(out.data_ptr()));
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("snr_rows(Tensor preds, Tensor target, Tensor(a!) out, int seg, bool scale_invariant, bool zero_mean, "
        "float eps) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("snr_rows", &snr_rows); }

}  // namespace tm_amd
