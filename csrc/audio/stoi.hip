// STOI / extended STOI intermediate-intelligibility measure over all 30-frame segments of a batch, one pass.
//
// After the one-third-octave analysis both signals are [B, J = 15, F] band envelopes.  The measure correlates every
// 30-frame window (segment m = frames m .. m + 29) of the clean and processed envelopes and averages over the
// segments that lie inside each signal's kept frames (Taal et al. 2011; extended: Jensen & Taal 2016, rows then
// columns normalised).  The reference delegates this to pystoi on the host (F/audio/stoi.py:25, NumPy per sample);
// a torch formulation materialises the [B, M, J, 30] unfolded windows several times over (clip, means, norms).
// Here a block owns 64 consecutive segments of one signal: it stages the 15 x (64 + 29) envelope window of both
// signals in LDS once, each thread evaluates one segment in fp64 straight from LDS, and the block writes one partial
// sum (a [B, chunks] buffer summed on the host side of the op: deterministic, no atomics).
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kJ = 15;       // one-third-octave bands
constexpr int kN = 30;       // frames per segment
constexpr int kSeg = 64;     // segments per block (one wave)
constexpr int kWin = kSeg + kN - 1;
constexpr double kEps = 2.220446049250313e-16;  // np.finfo(np.float64).eps
constexpr double kClip = 5.623413251903491;     // 10 ** (-BETA / 20), BETA = -15 dB

template <typename scalar_t>
__global__ void __launch_bounds__(kSeg) stoi_segments_kernel(const scalar_t* __restrict__ x,
                                                            const scalar_t* __restrict__ y, int F,
                                                            const int64_t* __restrict__ nframes, bool extended,
                                                            double* __restrict__ partial, int chunks) {
  __shared__ double sx[kJ][kWin];
  __shared__ double sy[kJ][kWin];
  __shared__ double red[kSeg / kWave > 0 ? kSeg / kWave : 1];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int m0 = chunk * kSeg;
  const long long m_valid = nframes[b] - kN + 1;
  const scalar_t* xb = x + static_cast<long long>(b) * kJ * F;
  const scalar_t* yb = y + static_cast<long long>(b) * kJ * F;
  for (int i = threadIdx.x; i < kJ * kWin; i += kSeg) {
    const int j = i / kWin, f = m0 + i % kWin;
    sx[j][i % kWin] = f < F ? static_cast<double>(xb[static_cast<long long>(j) * F + f]) : 0.0;
    sy[j][i % kWin] = f < F ? static_cast<double>(yb[static_cast<long long>(j) * F + f]) : 0.0;
  }
  __syncthreads();
  const int t = threadIdx.x;  // segment m0 + t, frames t .. t + 29 of the window
  double val = 0.0;
  if (m0 + t < m_valid) {
    if (!extended) {
      for (int j = 0; j < kJ; ++j) {
        const double* xr = &sx[j][t];
        const double* yr = &sy[j][t];
        double nx = 0.0, ny = 0.0;
        for (int n = 0; n < kN; ++n) {
          nx += xr[n] * xr[n];
          ny += yr[n] * yr[n];
        }
        const double c = sqrt(nx) / (sqrt(ny) + kEps);
        double my = 0.0, mx = 0.0;
        for (int n = 0; n < kN; ++n) {
          my += fmin(yr[n] * c, xr[n] * (1.0 + kClip));
          mx += xr[n];
        }
        my /= kN;
        mx /= kN;
        double syy = 0.0, sxx = 0.0, sxy = 0.0;
        for (int n = 0; n < kN; ++n) {
          const double yp = fmin(yr[n] * c, xr[n] * (1.0 + kClip)) - my;
          const double xc = xr[n] - mx;
          syy += yp * yp;
          sxx += xc * xc;
          sxy += yp * xc;
        }
        val += sxy / ((sqrt(syy) + kEps) * (sqrt(sxx) + kEps));
      }
    } else {
      // rows (bands over the 30 frames): mean and 1 / norm (0 for a constant row)
      double rmx[kJ], rsx[kJ], rmy[kJ], rsy[kJ];
      for (int j = 0; j < kJ; ++j) {
        const double* xr = &sx[j][t];
        const double* yr = &sy[j][t];
        double ax = 0.0, ay = 0.0;
        for (int n = 0; n < kN; ++n) {
          ax += xr[n];
          ay += yr[n];
        }
        ax /= kN;
        ay /= kN;
        double qx = 0.0, qy = 0.0;
        for (int n = 0; n < kN; ++n) {
          qx += (xr[n] - ax) * (xr[n] - ax);
          qy += (yr[n] - ay) * (yr[n] - ay);
        }
        rmx[j] = ax;
        rmy[j] = ay;
        rsx[j] = qx > 0 ? 1.0 / sqrt(qx) : 0.0;
        rsy[j] = qy > 0 ? 1.0 / sqrt(qy) : 0.0;
      }
      // columns (each frame over the 15 row-normalised bands), then the correlation
      for (int n = 0; n < kN; ++n) {
        double cx = 0.0, cy = 0.0;
        for (int j = 0; j < kJ; ++j) {
          cx += (sx[j][t + n] - rmx[j]) * rsx[j];
          cy += (sy[j][t + n] - rmy[j]) * rsy[j];
        }
        cx /= kJ;
        cy /= kJ;
        double qx = 0.0, qy = 0.0, qxy = 0.0;
        for (int j = 0; j < kJ; ++j) {
          const double zx = (sx[j][t + n] - rmx[j]) * rsx[j] - cx;
          const double zy = (sy[j][t + n] - rmy[j]) * rsy[j] - cy;
          qx += zx * zx;
          qy += zy * zy;
          qxy += zx * zy;
        }
        if (qx > 0 && qy > 0) val += qxy / (sqrt(qx) * sqrt(qy));
      }
      val /= kN;
    }
  }
  val = wave_sum(val);
  if (t == 0) partial[static_cast<long long>(b) * chunks + chunk] = val;
}

}  // namespace

// x_tob, y_tob: [B, 15, F] band envelopes (float32 / float64); nframes: int64 [B] kept frames per signal.
// Returns [B] fp64: the sum over each signal's valid segments of the segment correlation (standard: summed over the
// bands; extended: the segment's d).  The caller divides by the segment (x band) count.
at::Tensor stoi_segments(const at::Tensor& x_tob, const at::Tensor& y_tob, const at::Tensor& nframes, bool extended) {
  TM_CHECK_CUDA(x_tob);
  TM_SAME_DEVICE(x_tob, y_tob);
  TM_SAME_DEVICE(x_tob, nframes);
  TM_CHECK_CONTIG(x_tob);
  TM_CHECK_CONTIG(y_tob);
  TORCH_CHECK(x_tob.dim() == 3 && x_tob.size(1) == kJ && x_tob.sizes() == y_tob.sizes(),
              "stoi_segments: envelopes must be [B, 15, F] of one shape");
  TORCH_CHECK(x_tob.scalar_type() == y_tob.scalar_type(), "stoi_segments: dtype mismatch");
  TORCH_CHECK(nframes.scalar_type() == at::kLong && nframes.numel() == x_tob.size(0) && nframes.is_contiguous(),
              "stoi_segments: nframes int64 [B]");
  const int B = static_cast<int>(x_tob.size(0));
  const int F = static_cast<int>(x_tob.size(2));
  const int M = std::max(F - kN + 1, 0);
  const int chunks = std::max((M + kSeg - 1) / kSeg, 1);
  at::Tensor partial = at::zeros({B, chunks}, x_tob.options().dtype(at::kDouble));
  if (B == 0 || M == 0) return partial.sum(1);
  TORCH_CHECK(B < 65536, "stoi_segments: at most 65535 signals per call");
  AT_DISPATCH_FLOATING_TYPES(x_tob.scalar_type(), "stoi_segments", [&] {
    hipLaunchKernelGGL(stoi_segments_kernel<scalar_t>, dim3(chunks, B), dim3(kSeg), 0, stream(),
                       x_tob.data_ptr<scalar_t>(), y_tob.data_ptr<scalar_t>(), F, nframes.data_ptr<int64_t>(),
                       extended, partial.data_ptr<double>(), chunks);
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return partial.sum(1);
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("stoi_segments(Tensor x_tob, Tensor y_tob, Tensor nframes, bool extended) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("stoi_segments", &stoi_segments); }

}  // namespace tm_amd
