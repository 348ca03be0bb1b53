// CLIP metric math on the embeddings (reference F/multimodal/clip_score.py:60-96, F/multimodal/clip_iqa.py:171-178).
//
// CLIPScore: the reference L2-normalises both [N, D] embedding tensors (two norm + two divide launches, two [N, D]
// temporaries) and reduces their product.  ``paired_cosine_kernel``: one 64-lane wave per pair streams both rows
// once with 16-byte loads and keeps the three sums (a.b, a.a, b.b) in registers -- scale * a.b / (|a| |b|).
// CLIP-IQA: logits = 100 * img @ anchors^T followed by a softmax over each (positive, negative) prompt pair.
// ``prompt_pair_prob_kernel``: anchors staged through LDS in groups of 32, each wave computing two images' 32 dot
// products in registers, then each pair's softmax probability of the positive prompt,
// 1 / (1 + exp(l_neg - l_pos)), without the [N, 2P] logits tensor.
// Sums are fp32 (fp64 for fp64 embeddings), reduced across the wave in a fixed order (deterministic).
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;
constexpr int kWavesPerBlock = kThreads / kWave;

template <typename T>
using acc_t = typename std::conditional<std::is_same<T, double>::value, double, float>::type;

template <typename T>
__device__ __forceinline__ acc_t<T> ldx(const T* p) {
  if constexpr (std::is_same<T, double>::value) return *p;
  else return to_f32<T>(*p);
}

// a.b, a.a, b.b of two length-D rows (both 16-byte aligned when vec is set)
template <typename T, bool kSelfA, bool kSelfB>
__device__ __forceinline__ void row_dots(const T* __restrict__ a, const T* __restrict__ b, int D, bool vec,
                                         acc_t<T>& ab, acc_t<T>& aa, acc_t<T>& bb) {
  using A = acc_t<T>;
  const int lane = threadIdx.x & (kWave - 1);
  A s_ab = A(0), s_aa = A(0), s_bb = A(0);
  constexpr int kVec = 16 / sizeof(T);
  int d0 = 0;
  if (vec) {
    const int nvec = D / kVec;
    for (int v = lane; v < nvec; v += kWave) {
      const u32x4 ra = *reinterpret_cast<const u32x4*>(a + static_cast<long long>(v) * kVec);
      const u32x4 rb = *reinterpret_cast<const u32x4*>(b + static_cast<long long>(v) * kVec);
      const T* ea = reinterpret_cast<const T*>(&ra);
      const T* eb = reinterpret_cast<const T*>(&rb);
#pragma unroll
      for (int k = 0; k < kVec; ++k) {
        const A x = ldx<T>(ea + k), y = ldx<T>(eb + k);
        s_ab += x * y;
        if (kSelfA) s_aa += x * x;
        if (kSelfB) s_bb += y * y;
      }
    }
    d0 = nvec * kVec;
  }
  for (int d = d0 + lane; d < D; d += kWave) {
    const A x = ldx<T>(a + d), y = ldx<T>(b + d);
    s_ab += x * y;
    if (kSelfA) s_aa += x * x;
    if (kSelfB) s_bb += y * y;
  }
  ab = wave_sum(s_ab);
  if (kSelfA) aa = wave_sum(s_aa);
  if (kSelfB) bb = wave_sum(s_bb);
}

template <typename T>
__global__ void __launch_bounds__(kThreads) paired_cosine_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                                 long long n, int D, bool vec, float scale,
                                                                 float* __restrict__ out) {
  using A = acc_t<T>;
  const long long wave = (blockIdx.x * (long long)kThreads + threadIdx.x) / kWave;
  const long long nwaves = (long long)gridDim.x * kWavesPerBlock;
  for (long long r = wave; r < n; r += nwaves) {
    A ab, aa, bb;
    row_dots<T, true, true>(a + r * D, b + r * D, D, vec, ab, aa, bb);
    if ((threadIdx.x & (kWave - 1)) == 0)
      out[r] = static_cast<float>(static_cast<A>(scale) * (ab / (sqrt(aa) * sqrt(bb))));
  }
}

// Block = 8 waves, 16 images (2 per wave).  The anchors are staged through LDS in groups of 32 (16 prompt pairs,
// 32 x D values, <= 128 KB: every CLIP prompt set in one group); a wave holds its two image rows in registers
// (16 values per lane per chunk, all loads in flight), keeps the 2 x 32 dot products in registers, reduces them
// across the wave and writes the pair probabilities.  Images are read from HBM once, anchors from L2 once per block.
constexpr int kPairThreads = 512, kAncGroup = 32, kImgPerWave = 2, kRegPerLane = 16;
constexpr int kImgPerBlock = (kPairThreads / kWave) * kImgPerWave;

template <typename T>
__global__ void __launch_bounds__(kPairThreads) prompt_pair_prob_kernel(const T* __restrict__ img,
                                                                    const T* __restrict__ anchors, long long n,
                                                                    int n_anc, int D, float scale,
                                                                    float* __restrict__ out) {
  using A = acc_t<T>;
  extern __shared__ unsigned char smem_raw[];
  A* s_anc = reinterpret_cast<A*>(smem_raw);  // [kAncGroup][D]
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int pairs = n_anc / 2;
  const long long img0 = static_cast<long long>(blockIdx.x) * kImgPerBlock + wave * kImgPerWave;
  for (int g0 = 0; g0 < n_anc; g0 += kAncGroup) {
    __syncthreads();  // the previous group's readers are done with s_anc
    for (int d = threadIdx.x; d < D; d += kPairThreads) {
#pragma unroll
      for (int a = 0; a < kAncGroup; ++a)  // 32 independent loads in flight per thread
        s_anc[a * D + d] = (g0 + a < n_anc) ? ldx<T>(anchors + static_cast<long long>(g0 + a) * D + d) : A(0);
    }
    __syncthreads();
    // both images' rows in registers, 16 values per lane per chunk: 32 independent loads in flight per lane
    A acc[kImgPerWave][kAncGroup];
#pragma unroll
    for (int w = 0; w < kImgPerWave; ++w)
#pragma unroll
      for (int j = 0; j < kAncGroup; ++j) acc[w][j] = A(0);
    for (int c0 = 0; c0 < D; c0 += kRegPerLane * kWave) {
      A xr[kImgPerWave][kRegPerLane];
#pragma unroll
      for (int w = 0; w < kImgPerWave; ++w)
#pragma unroll
        for (int r = 0; r < kRegPerLane; ++r) {
          const int d = c0 + r * kWave + lane;
          const long long gi = img0 + w;
          xr[w][r] = (gi < n && d < D) ? ldx<T>(img + gi * D + d) : A(0);
        }
#pragma unroll
      for (int r = 0; r < kRegPerLane; ++r) {
        const int d = c0 + r * kWave + lane;
        if (d < D) {
#pragma unroll
          for (int j = 0; j < kAncGroup; ++j) {
            const A a = s_anc[j * D + d];
#pragma unroll
            for (int w = 0; w < kImgPerWave; ++w) acc[w][j] += xr[w][r] * a;
          }
        }
      }
    }
#pragma unroll
    for (int w = 0; w < kImgPerWave; ++w) {
      const long long gi = img0 + w;
#pragma unroll
      for (int j = 0; j < kAncGroup; ++j) acc[w][j] = wave_sum(acc[w][j]);
      // lane p writes pair g0/2 + p of this group
      A lp = A(0), ln = A(0);
#pragma unroll
      for (int p = 0; p < kAncGroup / 2; ++p) {
        if (lane == p) {
          lp = acc[w][2 * p];
          ln = acc[w][2 * p + 1];
        }
      }
      const int pp = g0 / 2 + lane;
      if (gi < n && lane < kAncGroup / 2 && pp < pairs) {
        const A s = static_cast<A>(scale);
        out[gi * pairs + pp] = static_cast<float>(A(1) / (A(1) + exp(s * ln - s * lp)));
      }
    }
  }
}

constexpr size_t kMaxPromptLds = 128 * 1024;

bool aligned16(const at::Tensor& t, int D, size_t elem) {
  return (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0) && ((static_cast<size_t>(D) * elem) % 16 == 0);
}

}  // namespace

// a, b: [N, D] floating, same dtype, contiguous -> scale * cos(a_i, b_i) as fp32 [N]
at::Tensor paired_cosine(const at::Tensor& a, const at::Tensor& b, double scale) {
  TM_CHECK_CUDA(a);
  TM_SAME_DEVICE(a, b);
  TORCH_CHECK(a.dim() == 2 && b.sizes() == a.sizes(), "paired_cosine: [N, D] inputs of equal shape expected");
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "paired_cosine: dtypes differ");
  TM_CHECK_CONTIG(a);
  TM_CHECK_CONTIG(b);
  const long long n = a.size(0);
  const int D = static_cast<int>(a.size(1));
  auto out = at::empty({n}, a.options().dtype(at::kFloat));
  if (n == 0) return out;
  const int grid = grid_cap((n + kWavesPerBlock - 1) / kWavesPerBlock, cu_count(a.get_device()) * 8);
  TM_DISPATCH_FLOAT(a.scalar_type(), "paired_cosine", [&] {
    const bool vec = aligned16(a, D, sizeof(scalar_t)) && aligned16(b, D, sizeof(scalar_t));
    hipLaunchKernelGGL((paired_cosine_kernel<scalar_t>), dim3(grid), dim3(kThreads), 0, stream(),
                       a.data_ptr<scalar_t>(), b.data_ptr<scalar_t>(), n, D, vec, static_cast<float>(scale),
                       out.data_ptr<float>());
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// img: [N, D], anchors: [2P, D] (positive, negative per prompt) -> softmax(scale * img @ anchors^T) over each pair,
// probability of the positive prompt: fp32 [N, P]
at::Tensor prompt_pair_prob(const at::Tensor& img, const at::Tensor& anchors, double scale) {
  TM_CHECK_CUDA(img);
  TM_SAME_DEVICE(img, anchors);
  TORCH_CHECK(img.dim() == 2 && anchors.dim() == 2 && anchors.size(1) == img.size(1) && anchors.size(0) % 2 == 0,
              "prompt_pair_prob: img [N, D] and anchors [2P, D] expected");
  TORCH_CHECK(img.scalar_type() == anchors.scalar_type(), "prompt_pair_prob: dtypes differ");
  TM_CHECK_CONTIG(img);
  TM_CHECK_CONTIG(anchors);
  const long long n = img.size(0);
  const int pairs = static_cast<int>(anchors.size(0) / 2);
  const int D = static_cast<int>(img.size(1));
  auto out = at::empty({n, pairs}, img.options().dtype(at::kFloat));
  if (n == 0 || pairs == 0) return out;
  const long long blocks = (n + kImgPerBlock - 1) / kImgPerBlock;
  TORCH_CHECK(blocks < (1LL << 31), "prompt_pair_prob: too many images");
  TM_DISPATCH_FLOAT(img.scalar_type(), "prompt_pair_prob", [&] {
    using A = acc_t<scalar_t>;
    const size_t lds = static_cast<size_t>(kAncGroup) * D * sizeof(A);
    TORCH_CHECK(lds <= kMaxPromptLds, "prompt_pair_prob: embedding dim too large for the LDS anchor group");
    TORCH_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&prompt_pair_prob_kernel<scalar_t>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) == hipSuccess,
                "prompt_pair_prob: LDS attribute");
    hipLaunchKernelGGL((prompt_pair_prob_kernel<scalar_t>), dim3(static_cast<unsigned>(blocks)), dim3(kPairThreads), lds,
                       stream(), img.data_ptr<scalar_t>(), anchors.data_ptr<scalar_t>(), n,
                       static_cast<int>(anchors.size(0)), D, static_cast<float>(scale), out.data_ptr<float>());
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("paired_cosine(Tensor a, Tensor b, float scale) -> Tensor");
  m.def("prompt_pair_prob(Tensor img, Tensor anchors, float scale) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("paired_cosine", &tm_amd::paired_cosine);
  m.impl("prompt_pair_prob", &tm_amd::prompt_pair_prob);
}
