// Fused token negative log-likelihood for Perplexity (K26 in SURVEY.md).
//
// The reference materialises softmax(preds) over the whole [B*S, V] logits tensor, gathers the target column and
// takes the log (F/text/perplexity.py:82-96): two full passes over the logits plus a [B*S, V] probability tensor.
// Here one 256-thread block owns one row: a single streaming pass over the V logits keeps a per-thread online
// (max, sum-exp) pair, 16-byte vector loads when the row is aligned, a wave/LDS reduction merges the pairs, and
// lane 0 writes  nll = log(sum exp(x - max)) + max - x[target]  (0 for ignored rows).  Accumulation is fp32 (fp64 for
// fp64 logits) whatever the storage type, so bf16/fp16 logits never see a half-precision softmax.  Rows write their
// own slot, and the host sums the [rows] vector -> deterministic.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;

template <typename A>
struct OnlineLse {
  A m, s;
  __device__ __forceinline__ void init() {
    m = -INFINITY;
    s = A(0);
  }
  __device__ __forceinline__ void add(A x) {
    if (x > m) {
      s = s * exp(m - x) + A(1);
      m = x;
    } else {
      s += exp(x - m);
    }
  }
  __device__ __forceinline__ void merge(A om, A os) {
    if (om == -INFINITY) return;
    if (m == -INFINITY) {
      m = om;
      s = os;
      return;
    }
    const A nm = m > om ? m : om;
    s = s * exp(m - nm) + os * exp(om - nm);
    m = nm;
  }
};

template <typename T, typename A>
__device__ __forceinline__ A ld(const T* p) {
  if constexpr (std::is_same<A, double>::value)
    return static_cast<double>(*p);
  else
    return to_f32<T>(*p);
}

template <typename T, typename A>
__global__ void __launch_bounds__(kThreads) token_nll_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                             long long rows, int vocab, long long ignore_index,
                                                             int use_ignore, int vec_ok, float* __restrict__ nll,
                                                             A* __restrict__ lse, int* __restrict__ flag) {
  __shared__ A sm[kThreads / kWave], ss[kThreads / kWave];
  for (long long row = blockIdx.x; row < rows; row += gridDim.x) {
    const int64_t t = target[row];
    const bool ignored = use_ignore && t == ignore_index;
    if (ignored) {  // uniform across the block
      if (threadIdx.x == 0) {
        nll[row] = 0.f;
        lse[row] = A(0);
      }
      continue;
    }
    const T* x = logits + row * static_cast<long long>(vocab);
    OnlineLse<A> acc;
    acc.init();
    constexpr int kVec = 16 / sizeof(T);
    if (vec_ok) {
      const int nvec = vocab / kVec;
      for (int v = threadIdx.x; v < nvec; v += kThreads) {
        const u32x4 raw = *reinterpret_cast<const u32x4*>(x + static_cast<long long>(v) * kVec);
        const T* e = reinterpret_cast<const T*>(&raw);
        A lm = ld<T, A>(e);
#pragma unroll
        for (int k = 1; k < kVec; ++k) lm = fmax(lm, ld<T, A>(e + k));
        A ls = A(0);
#pragma unroll
        for (int k = 0; k < kVec; ++k) ls += exp(ld<T, A>(e + k) - lm);
        acc.merge(lm, ls);
      }
      for (int v = nvec * kVec + threadIdx.x; v < vocab; v += kThreads) acc.add(ld<T, A>(x + v));
    } else {
      for (int v = threadIdx.x; v < vocab; v += kThreads) acc.add(ld<T, A>(x + v));
    }
    // wave merge
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
      const A om = __shfl_xor(acc.m, off, kWave);
      const A os = __shfl_xor(acc.s, off, kWave);
      acc.merge(om, os);
    }
    const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    if (lane == 0) {
      sm[wave] = acc.m;
      ss[wave] = acc.s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      OnlineLse<A> tot;
      tot.init();
      for (int w = 0; w < kThreads / kWave; ++w) tot.merge(sm[w], ss[w]);
      const A l = log(tot.s) + tot.m;
      lse[row] = l;
      if (t < 0 || t >= vocab) {
        raise_flag(flag, kErrTargetOutOfRange);
        nll[row] = NAN;
      } else {
        nll[row] = static_cast<float>(l - ld<T, A>(x + t));
      }
    }
    __syncthreads();
  }
}

}  // namespace

// nll[r] = -log softmax(logits[r])[target[r]]  (0 where target == ignore_index)
// lse[r] = logsumexp(logits[r]) (fp64 for fp64 logits, else fp32) is kept for the autograd backward.
void token_nll(const at::Tensor& logits, const at::Tensor& target, at::Tensor nll, at::Tensor lse, at::Tensor flag,
               int64_t ignore_index, bool use_ignore) {
  TM_CHECK_CUDA(logits);
  TM_CHECK_CONTIG(logits);
  TM_CHECK_CONTIG(target);
  TM_CHECK_CONTIG(nll);
  TORCH_CHECK(logits.dim() == 2, "token_nll: logits must be [rows, vocab]");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == logits.size(0), "token_nll: bad target");
  TORCH_CHECK(nll.scalar_type() == at::kFloat && nll.numel() == logits.size(0), "token_nll: bad nll buffer");
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "token_nll: bad flag");
  TORCH_CHECK(lse.numel() == logits.size(0) && lse.is_contiguous() &&
                  lse.scalar_type() == (logits.scalar_type() == at::kDouble ? at::kDouble : at::kFloat),
              "token_nll: bad lse buffer");
  const long long rows = logits.size(0);
  const int vocab = static_cast<int>(logits.size(1));
  if (rows == 0) return;
  TORCH_CHECK(vocab > 0, "token_nll: empty vocabulary");
  const int grid = static_cast<int>(rows < 65536 ? rows : 65536);
  TM_DISPATCH_FLOAT(logits.scalar_type(), "token_nll", [&] {
    const bool vec_ok = (reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0) &&
                        ((static_cast<long long>(vocab) * sizeof(scalar_t)) % 16 == 0);
    if constexpr (std::is_same<scalar_t, double>::value)
      hipLaunchKernelGGL((token_nll_kernel<double, double>), dim3(grid), dim3(kThreads), 0, stream(),
                         logits.data_ptr<double>(), target.data_ptr<int64_t>(), rows, vocab,
                         static_cast<long long>(ignore_index), use_ignore ? 1 : 0, vec_ok ? 1 : 0,
                         nll.data_ptr<float>(), lse.data_ptr<double>(), flag.data_ptr<int>());
    else
      hipLaunchKernelGGL((token_nll_kernel<scalar_t, float>), dim3(grid), dim3(kThreads), 0, stream(),
                         logits.data_ptr<scalar_t>(), target.data_ptr<int64_t>(), rows, vocab,
                         static_cast<long long>(ignore_index), use_ignore ? 1 : 0, vec_ok ? 1 : 0,
                         nll.data_ptr<float>(), lse.data_ptr<float>(), flag.data_ptr<int>());
  });
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "token_nll(Tensor logits, Tensor target, Tensor(a!) nll, Tensor(b!) lse, Tensor(c!) flag, int ignore_index, "
      "bool use_ignore) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("token_nll", &token_nll); }

}  // namespace tm_amd
