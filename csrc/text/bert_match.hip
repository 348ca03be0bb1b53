// BERTScore greedy matching for sentence-length token sets (P, R <= 128): row / column maxima of the token cosine
// similarities of every (candidate, reference) pair, without materialising the [pairs, P, R] similarity tensor.
//
// Reference: F/text/bert.py:134-167 (`torch.einsum("blpd, blrd -> blpr")` over the whole batch, then `max` over each
// axis).  The 128 x 128-tile MFMA GEMM with the same epilogue (csrc/pairwise/gemm_nt.hip, kRowColMax) fills its tiles
// only for long sequences; typical sentences (10-60 tokens) would use a few percent of a tile.  Here one block per
// pair walks 64 x 64 super-tiles of its P x R matrix:
//   * 256 threads = 4 waves as 2 x 2, each wave one 32 x 32 v_mfma_f32_32x32x2_f32 accumulator (exact fp32 products);
//   * K (the embedding dim) in chunks of 32: the 64-row slabs of both operands are staged in LDS with 16-byte
//     coalesced loads (rows padded to 33 floats: the 32 rows one MFMA operand read touches hit distinct banks);
//   * epilogue: the 64 x 64 tile goes through LDS once; each thread folds one row / one column into running maxima
//     over the valid R / P range (kept in LDS across super-tiles), then the pair's maxima are written out.
// Embeddings are read once per super-tile row / column: the pair's bytes (P + R) * D * 4 dominate, so the kernel runs
// at streaming speed.
// bf16 / fp16 embeddings (a 16-bit model -- the reference's einsum runs in the model's dtype) take the 16-bit form:
// v_mfma_f32_32x32x16_{bf16,f16} on the embeddings as they are (no fp32 upcast pass, half the bytes), K in chunks of
// 64 elements staged as 16-byte vectors into LDS rows padded to 144 B; fp32 accumulation; the maxima are rounded to
// the input dtype (the reference's similarity tensor is in that dtype, and rounding commutes with max).
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kT = 64, kKC = 32, kStride = kKC + 1, kMaxTok = 128;
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) bert_rowcol_max_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                              int P, int R, int D, bool vec,
                                                              float* __restrict__ rmax, float* __restrict__ cmax) {
  __shared__ float xs[kT * kStride];
  __shared__ float ys[kT * kStride];
  __shared__ float tile[kT][kT + 1];
  __shared__ float rm[kMaxTok], cm[kMaxTok];
  const int pair = blockIdx.x;
  const float* X = x + static_cast<long long>(pair) * P * D;
  const float* Y = y + static_cast<long long>(pair) * R * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;
  for (int i = tid; i < kMaxTok; i += 256) {
    rm[i] = -INFINITY;
    cm[i] = -INFINITY;
  }
  for (int ti = 0; ti * kT < P; ++ti) {
    for (int tj = 0; tj * kT < R; ++tj) {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      for (int k0 = 0; k0 < D; k0 += kKC) {
        __syncthreads();  // previous chunk (or previous tile's epilogue) is done with the LDS slabs
        // stage 64 rows x 32 k of each operand: 512 float4 per operand, 2 per thread
        for (int v = tid; v < kT * (kKC / 4); v += 256) {
          const int row = v / (kKC / 4), kq = (v % (kKC / 4)) * 4;
          const int gx = ti * kT + row, gy = tj * kT + row;
          float a[4], b[4];
          if (vec && k0 + kq + 4 <= D) {
            const float4 fa = gx < P ? *reinterpret_cast<const float4*>(X + static_cast<long long>(gx) * D + k0 + kq)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 fb = gy < R ? *reinterpret_cast<const float4*>(Y + static_cast<long long>(gy) * D + k0 + kq)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
            a[0] = fa.x; a[1] = fa.y; a[2] = fa.z; a[3] = fa.w;
            b[0] = fb.x; b[1] = fb.y; b[2] = fb.z; b[3] = fb.w;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int k = k0 + kq + e;
              a[e] = (gx < P && k < D) ? X[static_cast<long long>(gx) * D + k] : 0.f;
              b[e] = (gy < R && k < D) ? Y[static_cast<long long>(gy) * D + k] : 0.f;
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            xs[row * kStride + kq + e] = a[e];
            ys[row * kStride + kq + e] = b[e];
          }
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < kKC; ks += 2) {
          const float av = xs[(wr * 32 + r32) * kStride + ks + h];
          const float bv = ys[(wc * 32 + r32) * kStride + ks + h];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
      }
      // epilogue: accumulator -> LDS tile (row = (e & 3) + 8 (e >> 2) + 4 h, col = lane & 31 within the wave tile)
#pragma unroll
      for (int e = 0; e < 16; ++e) tile[wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * h][wc * 32 + r32] = acc[e];
      __syncthreads();
      const int rows = min(kT, P - ti * kT), cols = min(kT, R - tj * kT);
      if (tid < kT) {
        if (tid < rows) {
          float m = -INFINITY;
          for (int j = 0; j < cols; ++j) m = fmaxf(m, tile[tid][j]);
          rm[ti * kT + tid] = fmaxf(rm[ti * kT + tid], m);
        }
      } else if (tid < 2 * kT) {
        const int j = tid - kT;
        if (j < cols) {
          float m = -INFINITY;
          for (int i = 0; i < rows; ++i) m = fmaxf(m, tile[i][j]);
          cm[tj * kT + j] = fmaxf(cm[tj * kT + j], m);
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < P; i += 256) rmax[static_cast<long long>(pair) * P + i] = rm[i];
  for (int j = tid; j < R; j += 256) cmax[static_cast<long long>(pair) * R + j] = cm[j];
}

template <typename T>
struct Mma16;
template <>
struct Mma16<__bf16> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 run(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float round(float v) { return static_cast<float>(static_cast<__bf16>(v)); }
};
template <>
struct Mma16<_Float16> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 run(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float round(float v) { return static_cast<float>(static_cast<_Float16>(v)); }
};

constexpr int kKC16 = 64, kStride16 = kKC16 + 8;  // 16-bit elements per K chunk / per padded LDS row (144 B)

template <typename T>
__global__ void __launch_bounds__(256) bert_rowcol_max16_kernel(const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ y, int P, int R, int D,
                                                                bool vec, float* __restrict__ rmax,
                                                                float* __restrict__ cmax) {
  typedef typename Mma16<T>::v8 v8;
  __shared__ __attribute__((aligned(16))) uint16_t xs[kT * kStride16];
  __shared__ __attribute__((aligned(16))) uint16_t ys[kT * kStride16];
  __shared__ float tile[kT][kT + 1];
  __shared__ float rm[kMaxTok], cm[kMaxTok];
  const int pair = blockIdx.x;
  const uint16_t* X = x + static_cast<long long>(pair) * P * D;
  const uint16_t* Y = y + static_cast<long long>(pair) * R * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;
  for (int i = tid; i < kMaxTok; i += 256) {
    rm[i] = -INFINITY;
    cm[i] = -INFINITY;
  }
  for (int ti = 0; ti * kT < P; ++ti) {
    for (int tj = 0; tj * kT < R; ++tj) {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      for (int k0 = 0; k0 < D; k0 += kKC16) {
        __syncthreads();  // previous chunk (or previous tile's epilogue) is done with the LDS slabs
        // stage 64 rows x 64 k of each operand: 512 16-byte vectors per operand, 2 per thread
        for (int v = tid; v < kT * (kKC16 / 8); v += 256) {
          const int row = v / (kKC16 / 8), kq = (v % (kKC16 / 8)) * 8;
          const int gx = ti * kT + row, gy = tj * kT + row;
          uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
          if (vec && k0 + kq + 8 <= D) {
            if (gx < P) a = *reinterpret_cast<const uint4*>(X + static_cast<long long>(gx) * D + k0 + kq);
            if (gy < R) b = *reinterpret_cast<const uint4*>(Y + static_cast<long long>(gy) * D + k0 + kq);
          } else {
            uint16_t ea[8], eb[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int k = k0 + kq + e;
              ea[e] = (gx < P && k < D) ? X[static_cast<long long>(gx) * D + k] : uint16_t(0);
              eb[e] = (gy < R && k < D) ? Y[static_cast<long long>(gy) * D + k] : uint16_t(0);
            }
            a = __builtin_bit_cast(uint4, ea);
            b = __builtin_bit_cast(uint4, eb);
          }
          *reinterpret_cast<uint4*>(xs + row * kStride16 + kq) = a;
          *reinterpret_cast<uint4*>(ys + row * kStride16 + kq) = b;
        }
        __syncthreads();
#pragma unroll
        for (int s4 = 0; s4 < kKC16 / 16; ++s4) {
          const v8 av = *reinterpret_cast<const v8*>(xs + (wr * 32 + r32) * kStride16 + 16 * s4 + 8 * h);
          const v8 bv = *reinterpret_cast<const v8*>(ys + (wc * 32 + r32) * kStride16 + 16 * s4 + 8 * h);
          acc = Mma16<T>::run(av, bv, acc);
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) tile[wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * h][wc * 32 + r32] = acc[e];
      __syncthreads();
      const int rows = min(kT, P - ti * kT), cols = min(kT, R - tj * kT);
      if (tid < kT) {
        if (tid < rows) {
          float m = -INFINITY;
          for (int j = 0; j < cols; ++j) m = fmaxf(m, tile[tid][j]);
          rm[ti * kT + tid] = fmaxf(rm[ti * kT + tid], m);
        }
      } else if (tid < 2 * kT) {
        const int j = tid - kT;
        if (j < cols) {
          float m = -INFINITY;
          for (int i = 0; i < rows; ++i) m = fmaxf(m, tile[i][j]);
          cm[tj * kT + j] = fmaxf(cm[tj * kT + j], m);
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < P; i += 256) rmax[static_cast<long long>(pair) * P + i] = Mma16<T>::round(rm[i]);
  for (int j = tid; j < R; j += 256) cmax[static_cast<long long>(pair) * R + j] = Mma16<T>::round(cm[j]);
}

}  // namespace

// x [pairs, P, D], y [pairs, R, D] fp32 / bf16 / fp16 (one dtype) -> rmax [pairs, P], cmax [pairs, R] fp32
void bert_rowcol_max(const at::Tensor& x, const at::Tensor& y, at::Tensor rmax, at::Tensor cmax) {
  TM_CHECK_CUDA(x);
  TM_SAME_DEVICE(x, y);
  TM_SAME_DEVICE(x, rmax);
  TM_SAME_DEVICE(x, cmax);
  TM_CHECK_CONTIG(x);
  TM_CHECK_CONTIG(y);
  const auto dt = x.scalar_type();
  TORCH_CHECK((dt == at::kFloat || dt == at::kBFloat16 || dt == at::kHalf) && y.scalar_type() == dt,
              "bert_rowcol_max: fp32 / bf16 / fp16 embeddings of one dtype");
  TORCH_CHECK(x.dim() == 3 && y.dim() == 3 && x.size(0) == y.size(0) && x.size(2) == y.size(2),
              "bert_rowcol_max: x [pairs, P, D], y [pairs, R, D]");
  const int pairs = x.size(0), P = x.size(1), R = y.size(1), D = x.size(2);
  TORCH_CHECK(P <= kMaxTok && R <= kMaxTok, "bert_rowcol_max: at most ", kMaxTok, " tokens per side");
  TORCH_CHECK(rmax.scalar_type() == at::kFloat && rmax.is_contiguous() && rmax.numel() == static_cast<long long>(pairs) * P,
              "bert_rowcol_max: rmax must be fp32 [pairs, P]");
  TORCH_CHECK(cmax.scalar_type() == at::kFloat && cmax.is_contiguous() && cmax.numel() == static_cast<long long>(pairs) * R,
              "bert_rowcol_max: cmax must be fp32 [pairs, R]");
  if (pairs == 0 || P == 0 || R == 0) return;
  // 16-byte loads only when every row start is 16-byte aligned
  const bool aligned = reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                       reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0;
  if (dt == at::kFloat) {
    hipLaunchKernelGGL(bert_rowcol_max_kernel, dim3(pairs), dim3(256), 0, stream(), x.data_ptr<float>(),
                       y.data_ptr<float>(), P, R, D, aligned && D % 4 == 0, rmax.data_ptr<float>(),
                       cmax.data_ptr<float>());
  } else {
    const auto* xp = reinterpret_cast<const uint16_t*>(x.data_ptr());
    const auto* yp = reinterpret_cast<const uint16_t*>(y.data_ptr());
    const bool vec = aligned && D % 8 == 0;
    if (dt == at::kBFloat16)
      hipLaunchKernelGGL(bert_rowcol_max16_kernel<__bf16>, dim3(pairs), dim3(256), 0, stream(), xp, yp, P, R, D, vec,
                         rmax.data_ptr<float>(), cmax.data_ptr<float>());
    else
      hipLaunchKernelGGL(bert_rowcol_max16_kernel<_Float16>, dim3(pairs), dim3(256), 0, stream(), xp, yp, P, R, D,
                         vec, rmax.data_ptr<float>(), cmax.data_ptr<float>());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("bert_rowcol_max(Tensor x, Tensor y, Tensor(a!) rmax, Tensor(b!) cmax) -> ()"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("bert_rowcol_max", &bert_rowcol_max); }

}  // namespace tm_amd
