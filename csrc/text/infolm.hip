// InfoLM on the device: the masked-LM distribution accumulation and the information measure.
//
// segment_softmax_sum -- reference F/text/infolm.py:300-330: per position a softmax over the vocabulary, a multiply by
// the (idf) token weight, then sums over the positions of each sentence (here: `softmax`, `mul`, `zeros`, `index_add`
// and `add` per chunk).  Here two launches per chunk: one block per masked row finds max(l / T) and sum exp(l / T - max)
// (one pass, online rescaling); then one thread per (sentence, vocabulary entry) walks the sentence's rows (sorted by
// sentence, `seg` offsets) and adds sum_r w_r exp(l_r / T - max_r) / sum_r into the sentence's distribution in place --
// no [rows, V] probability tensor, no atomics (rows of one sentence are summed in a fixed order).
//
// info_measure -- reference F/text/infolm.py:60-215 (`_InformationMeasure`): per pair of sentence distributions
// [N, V] the KL / alpha / beta / AB / Renyi divergences, L1 / L2 / L-inf distances or the Fisher-Rao distance.  The
// reference evaluates each as 3-6 full [N, V] elementwise ops plus reductions; here one block per sentence pair reads
// both rows once and accumulates every sum the measure needs in fp64, then applies the closed form and the reference's
// `nan_to_num` (NaN -> 0, +-inf -> +-FLT_MAX).
#include <cfloat>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 512;

template <typename T>
__global__ void __launch_bounds__(kThreads) row_softmax_stats_kernel(const T* __restrict__ logits, int V, float inv_t,
                                                                     float* __restrict__ stats) {
  const T* row = logits + static_cast<long long>(blockIdx.x) * V;
  float m = -INFINITY, s = 0.f;
  for (int v = threadIdx.x; v < V; v += kThreads) {
    const float x = to_f32(row[v]) * inv_t;
    if (x == -INFINITY) continue;  // exp(-inf) = 0
    if (x > m) {
      s = s * expf(m - x) + 1.f;
      m = x;
    } else {
      s += expf(x - m);
    }
  }
  // combine (m, s) pairs: wave, then block
  for (int off = 32; off > 0; off >>= 1) {
    const float mo = __shfl_xor(m, off, 64), so = __shfl_xor(s, off, 64);
    const float mn = fmaxf(m, mo);
    s = (m == -INFINITY ? 0.f : s * expf(m - mn)) + (mo == -INFINITY ? 0.f : so * expf(mo - mn));
    m = mn;
  }
  __shared__ float sm[kThreads / 64], ss[kThreads / 64];
  if ((threadIdx.x & 63) == 0) {
    sm[threadIdx.x >> 6] = m;
    ss[threadIdx.x >> 6] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float mm = -INFINITY;
    for (int w = 0; w < kThreads / 64; ++w) mm = fmaxf(mm, sm[w]);
    float tot = 0.f;
    for (int w = 0; w < kThreads / 64; ++w) tot += sm[w] == -INFINITY ? 0.f : ss[w] * expf(sm[w] - mm);
    stats[2 * blockIdx.x] = mm;
    stats[2 * blockIdx.x + 1] = tot;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) segment_prob_sum_kernel(const T* __restrict__ logits, int V, float inv_t,
                                                               const float* __restrict__ stats,
                                                               const float* __restrict__ w,
                                                               const int64_t* __restrict__ seg,
                                                               const int64_t* __restrict__ sent,
                                                               float* __restrict__ acc) {
  const int s = blockIdx.y;
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= V) return;
  const long long r0 = seg[s], r1 = seg[s + 1];
  if (r0 == r1) return;
  float sum = 0.f;
  for (long long r = r0; r < r1; ++r) {
    const float x = to_f32(logits[r * V + v]) * inv_t;
    sum += w[r] * (expf(x - stats[2 * r]) / stats[2 * r + 1]);
  }
  acc[sent[s] * V + v] += sum;
}

enum Measure : int { kKL = 0, kAlpha = 1, kBeta = 2, kAB = 3, kRenyi = 4, kL1 = 5, kL2 = 6, kLinf = 7, kFisher = 8 };

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < kThreads / 64; ++i) s += red[i];
  return s;
}

__global__ void __launch_bounds__(kThreads) info_measure_kernel(const float* __restrict__ p,
                                                                const float* __restrict__ t, int V, int measure,
                                                                float alpha, float beta, float* __restrict__ out) {
  __shared__ double red[kThreads / 64];
  const float* pr = p + static_cast<long long>(blockIdx.x) * V;
  const float* tr = t + static_cast<long long>(blockIdx.x) * V;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  double mx = 0.0;
  bool nan_seen = false;
  for (int v = threadIdx.x; v < V; v += kThreads) {
    const float a = pr[v], b = tr[v];
    switch (measure) {
      case kKL: s0 += static_cast<double>(b * logf(a / b)); break;
      case kAlpha:
      case kRenyi: s0 += static_cast<double>(powf(b, alpha) * powf(a, 1.f - alpha)); break;
      case kBeta:
      case kAB: {
        s0 += static_cast<double>(powf(b, beta + alpha));
        s1 += static_cast<double>(powf(a, beta + alpha));
        s2 += static_cast<double>(powf(b, alpha) * powf(a, beta));
        break;
      }
      case kL1: s0 += static_cast<double>(fabsf(b - a)); break;
      case kL2: s0 += static_cast<double>((b - a) * (b - a)); break;
      case kLinf: {
        const double d = static_cast<double>(fabsf(b - a));
        nan_seen |= d != d;
        mx = fmax(mx, d);
        break;
      }
      default: s0 += static_cast<double>(sqrtf(a * b)); break;
    }
  }
  s0 = block_sum(s0, red);
  if (measure == kBeta || measure == kAB) {
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
  }
  if (measure == kLinf) {
    // max over the block (fmax drops NaN operands: a NaN seen anywhere is carried separately, torch's max keeps it)
    __shared__ int any_nan;
    if (threadIdx.x == 0) any_nan = 0;
    __syncthreads();
    if (nan_seen) any_nan = 1;
    for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
      double m = 0.0;
      for (int i = 0; i < kThreads / 64; ++i) m = fmax(m, red[i]);
      s0 = any_nan ? NAN : m;
    }
  }
  if (threadIdx.x != 0) return;
  const double a = alpha, b = beta;
  double r;
  switch (measure) {
    case kKL: r = s0; break;
    case kAlpha: r = (1.0 - s0) / (a * (a - 1.0)); break;
    case kBeta:
    case kAB: {
      const double aa = measure == kBeta ? 1.0 : a;
      r = log(s0) / (b * (b + aa)) + log(s1) / (aa * (b + aa)) - log(s2) / (aa * b);
      break;
    }
    case kRenyi: r = log(s0) / (a - 1.0); break;
    case kL1:
    case kLinf: r = s0; break;
    case kL2: r = sqrt(s0); break;
    default: {
      double c = s0 < 0.0 ? 0.0 : (s0 > 1.0 ? 1.0 : s0);
      if (s0 != s0) c = s0;
      r = 2.0 * acos(c);
    }
  }
  float f = static_cast<float>(r);
  if (f != f) f = 0.f;                      // nan_to_num: NaN -> 0
  else if (f == INFINITY) f = FLT_MAX;      // +inf -> largest finite
  else if (f == -INFINITY) f = -FLT_MAX;    // -inf -> most negative finite
  out[blockIdx.x] = f;
}

}  // namespace

// logits [R, V] (fp32 / bf16 / fp16) rows sorted by sentence; w fp32 [R]; seg int64 [S + 1] row offsets of S segments;
// sent int64 [S] destination sentence per segment; acc fp32 [N, V] (accumulated in place).
void infolm_accumulate(const at::Tensor& logits, double temperature, const at::Tensor& w, const at::Tensor& seg,
                       const at::Tensor& sent, at::Tensor acc) {
  TM_CHECK_CUDA(logits);
  TM_SAME_DEVICE(logits, w);
  TM_SAME_DEVICE(logits, seg);
  TM_SAME_DEVICE(logits, sent);
  TM_SAME_DEVICE(logits, acc);
  TM_CHECK_CONTIG(logits);
  TORCH_CHECK(logits.dim() == 2, "infolm_accumulate: logits [rows, V]");
  const long long R = logits.size(0), V = logits.size(1), S = sent.numel();
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == R, "infolm_accumulate: w fp32 [rows]");
  TORCH_CHECK(seg.scalar_type() == at::kLong && seg.is_contiguous() && seg.numel() == S + 1,
              "infolm_accumulate: seg int64 [S + 1]");
  TORCH_CHECK(sent.scalar_type() == at::kLong && sent.is_contiguous(), "infolm_accumulate: sent int64 [S]");
  TORCH_CHECK(acc.scalar_type() == at::kFloat && acc.is_contiguous() && acc.dim() == 2 && acc.size(1) == V,
              "infolm_accumulate: acc fp32 [N, V]");
  TORCH_CHECK(temperature > 0, "infolm_accumulate: temperature must be positive");
  TORCH_CHECK(V < (1LL << 31) && S < 65536, "infolm_accumulate: sizes");
  if (R == 0 || S == 0) return;
  // host-side contract (checked by the caller's construction): seg is non-decreasing in [0, R], sent in [0, N)
  at::Tensor stats = at::empty({R, 2}, logits.options().dtype(at::kFloat));
  const float inv_t = static_cast<float>(1.0 / temperature);
  TM_DISPATCH_FLOAT(logits.scalar_type(), "infolm_accumulate", [&] {
    hipLaunchKernelGGL((row_softmax_stats_kernel<scalar_t>), dim3(static_cast<unsigned>(R)), dim3(kThreads), 0,
                       stream(), logits.data_ptr<scalar_t>(), static_cast<int>(V), inv_t, stats.data_ptr<float>());
    hipLaunchKernelGGL((segment_prob_sum_kernel<scalar_t>), dim3(static_cast<unsigned>((V + 255) / 256),
                       static_cast<unsigned>(S)), dim3(256), 0, stream(), logits.data_ptr<scalar_t>(),
                       static_cast<int>(V), inv_t, stats.data_ptr<float>(), w.data_ptr<float>(),
                       seg.data_ptr<int64_t>(), sent.data_ptr<int64_t>(), acc.data_ptr<float>());
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// p, t fp32 [N, V] -> out fp32 [N]; measure: 0 kl, 1 alpha, 2 beta, 3 ab, 4 renyi, 5 l1, 6 l2, 7 linf, 8 fisher-rao
// (beta: the caller passes alpha = 1, the reference's `_ab_divergence(alpha=1)`)
void info_measure(const at::Tensor& p, const at::Tensor& t, int64_t measure, double alpha, double beta, at::Tensor out) {
  TM_CHECK_CUDA(p);
  TM_SAME_DEVICE(p, t);
  TM_SAME_DEVICE(p, out);
  TM_CHECK_CONTIG(p);
  TM_CHECK_CONTIG(t);
  TORCH_CHECK(p.scalar_type() == at::kFloat && t.scalar_type() == at::kFloat && p.dim() == 2 && p.sizes() == t.sizes(),
              "info_measure: p / t must be fp32 [N, V]");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == p.size(0),
              "info_measure: out fp32 [N]");
  TORCH_CHECK(measure >= 0 && measure <= 8, "info_measure: unknown measure ", measure);
  TORCH_CHECK(p.size(1) < (1LL << 31), "info_measure: V too large");
  if (p.size(0) == 0) return;
  hipLaunchKernelGGL(info_measure_kernel, dim3(static_cast<unsigned>(p.size(0))), dim3(kThreads), 0, stream(),
                     p.data_ptr<float>(), t.data_ptr<float>(), static_cast<int>(p.size(1)), static_cast<int>(measure),
                     static_cast<float>(alpha), static_cast<float>(beta), out.data_ptr<float>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("infolm_accumulate(Tensor logits, float temperature, Tensor w, Tensor seg, Tensor sent, Tensor(a!) acc) -> ()");
  m.def("info_measure(Tensor p, Tensor t, int measure, float alpha, float beta, Tensor(a!) out) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("infolm_accumulate", &infolm_accumulate);
  m.impl("info_measure", &info_measure);
}

}  // namespace tm_amd
