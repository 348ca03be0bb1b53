// Cascaded biquad IIR filtering (SRMR's gammatone filterbank and modulation filterbank; SURVEY.md audio plan:
// biquad.hip).
//
// The reference runs torchaudio's `lfilter` once per cascade stage (4 gammatone stages + the modulation stage,
// F/audio/srmr.py:127-143,295), each a full pass over [B, channels, time] with the stage output written back to
// memory.  Here one thread owns one (signal, channel) row and pushes every sample through all S second-order
// sections in registers (direct form I, fp64, a0-normalised), optionally clamping each stage's output to [-1, 1]
// exactly like `lfilter(clamp=True)` does after the stage.  Rows are independent, so the grid is B * channels wide.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 128;
constexpr int kMaxSections = 8;

// coefs: [n_filters, S, 6] = (b0, b1, b2, a0, a1, a2) per section; row r uses filter r % n_filters and reads signal
// row r / rep (rep = n_filters when one signal feeds every filter, 1 when x is already [rows, T]).
__global__ void __launch_bounds__(kThreads) biquad_cascade_kernel(const double* __restrict__ x,
                                                                  const double* __restrict__ coefs, long long rows,
                                                                  long long len, int n_filters, int sections, int rep,
                                                                  int clamp, double* __restrict__ y) {
  const long long r = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const int f = static_cast<int>(r % n_filters);
  double b0[kMaxSections], b1[kMaxSections], b2[kMaxSections], a1[kMaxSections], a2[kMaxSections];
  double x1[kMaxSections], x2[kMaxSections], y1[kMaxSections], y2[kMaxSections];
  for (int s = 0; s < sections; ++s) {
    const double* c = coefs + (static_cast<long long>(f) * sections + s) * 6;
    const double inv = 1.0 / c[3];
    b0[s] = c[0] * inv;
    b1[s] = c[1] * inv;
    b2[s] = c[2] * inv;
    a1[s] = c[4] * inv;
    a2[s] = c[5] * inv;
    x1[s] = x2[s] = y1[s] = y2[s] = 0.0;
  }
  const double* xr = x + (r / rep) * len;
  double* yr = y + r * len;
  for (long long n = 0; n < len; ++n) {
    double v = xr[n];
    for (int s = 0; s < sections; ++s) {
      const double o = b0[s] * v + b1[s] * x1[s] + b2[s] * x2[s] - a1[s] * y1[s] - a2[s] * y2[s];
      x2[s] = x1[s];
      x1[s] = v;
      y2[s] = y1[s];
      y1[s] = o;
      v = clamp ? fmin(fmax(o, -1.0), 1.0) : o;  // lfilter(clamp=True) clamps each stage's output
    }
    yr[n] = v;
  }
}

}  // namespace

void biquad_cascade(const at::Tensor& x, const at::Tensor& coefs, at::Tensor y, int64_t rep, bool clamp) {
  TM_CHECK_CUDA(x);
  TM_CHECK_CONTIG(x);
  TM_CHECK_CONTIG(coefs);
  TM_CHECK_CONTIG(y);
  TORCH_CHECK(x.scalar_type() == at::kDouble && coefs.scalar_type() == at::kDouble && y.scalar_type() == at::kDouble,
              "biquad_cascade: fp64 tensors expected");
  TORCH_CHECK(coefs.dim() == 3 && coefs.size(2) == 6 && coefs.size(1) <= kMaxSections,
              "biquad_cascade: coefs must be [filters, sections <= 8, 6]");
  TORCH_CHECK(y.dim() == 2 && x.dim() == 2 && x.size(1) == y.size(1), "biquad_cascade: x [S, T], y [rows, T]");
  TORCH_CHECK(rep >= 1 && y.size(0) == x.size(0) * rep, "biquad_cascade: rows must equal signals * rep");
  const long long rows = y.size(0), len = y.size(1);
  if (rows == 0 || len == 0) return;
  hipLaunchKernelGGL(biquad_cascade_kernel, dim3(static_cast<unsigned>((rows + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, stream(), x.data_ptr<double>(), coefs.data_ptr<double>(), rows, len,
                     static_cast<int>(coefs.size(0)), static_cast<int>(coefs.size(1)), static_cast<int>(rep),
                     clamp ? 1 : 0, y.data_ptr<double>());
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("biquad_cascade(Tensor x, Tensor coefs, Tensor(a!) y, int rep, bool clamp) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("biquad_cascade", &biquad_cascade); }

}  // namespace tm_amd
