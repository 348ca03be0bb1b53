// FID / MiFID feature statistics: Σx (fp64) and XᵀX (fp64, symmetric) accumulated into metric states.
//
// Reference (S/image/fid.py:336-348) promotes the [N, D] features to fp64 and runs `features.t().mm(features)`
// (a full D x D fp64 GEMM, both triangles) plus `features.sum(0)`.  Here one SYRK kernel on the fp64 matrix cores
// (v_mfma_f64_16x16x4_f64 on gfx950) computes only the upper-triangle 128 x 128 tiles (half the FLOPs), keeps the
// staged panels in LDS in their input precision (fp32 for fp32/bf16/fp16 features: exact, half the LDS bytes of fp64)
// and widens to fp64 in registers right before each MFMA, folds the column sums into the diagonal tiles, and splits
// the sample (K) dimension across blocks so the ~136 upper tiles of a D = 2048 problem fill the 256 CUs.  A second
// kernel reduces the split-K partials in a fixed order (bitwise reproducible) and adds them into both triangles of
// the state, transposing the mirrored block through LDS so both writes are coalesced.
//
// Per block: 128 x 128 C tile, 8 waves as 2 x 4, each 64 x 32 = 4 x 2 MFMA 16x16 accumulators (f64x4): two waves per
// SIMD, so one wave's LDS waits and the chunk barrier hide under the other's MFMAs (the 4-wave 64 x 64 layout ran the
// f64 pipe ~8 % less busy, csrc/image/dgemm.hip).  K chunk = 32 samples, two LDS stages: chunk c+1 is written into the
// other stage while chunk c is consumed, chunk c+2 is in flight in registers, one barrier per chunk; inside a chunk the
// operands of k-step s+1 are read while the MFMAs of step s issue.  LDS rows are padded to 144 elements (≡ 16 mod 32
// words for b32 reads, ≡ 32 mod 64 for b64 reads) so the 4 k-rows read by one wave land on disjoint banks.
//
// Numerics: products and sums are fp64 exactly as in the reference (inputs are exactly representable in fp64).
#include <cstdlib>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 128;          // C tile edge
constexpr int kKC = 32;             // samples per K chunk (8 MFMA k-steps of 4)
constexpr int kLdsRow = kTile + 16; // padded LDS row (elements)
constexpr int kThreads = 512;       // 8 waves, 2 x 4 over the tile, 64 x 32 each
constexpr int kColsPerThread = 8;   // each thread stages 8 consecutive columns of one sample row per panel
constexpr int kThrPerRow = kTile / kColsPerThread;  // 16 threads stage one sample row
static_assert(kThrPerRow * kKC == kThreads, "staging covers the chunk exactly");

// LDS element type: fp32 for every input narrower than or equal to fp32 (exact), fp64 for fp64 inputs
template <typename T>
struct Stage {
  using type = float;
};
template <>
struct Stage<double> {
  using type = double;
};

template <typename T>
__device__ __forceinline__ typename Stage<T>::type to_stage(T v) {
  return to_f32(v);
}
template <>
__device__ __forceinline__ double to_stage<double>(double v) {
  return v;
}

__device__ __forceinline__ void tile_coords(int t, int ntile, int& ti, int& tj) {
  // t enumerates the upper triangle row by row: (0,0),(0,1)..(0,n-1),(1,1)..
  int row = 0;
  int rem = t;
  while (rem >= ntile - row) {
    rem -= ntile - row;
    ++row;
  }
  ti = row;
  tj = row + rem;
}

// Loads kColsPerThread consecutive features (columns c0..c0+15 of sample row `row`) in storage type, 16-byte loads when possible.
template <typename scalar_t>
__device__ __forceinline__ void load_cols(const scalar_t* __restrict__ x, long long n, int d, long long row, int c0,
                                       bool vec_ok, scalar_t (&out)[kColsPerThread]) {
  if (row < n && vec_ok && c0 + kColsPerThread <= d) {
    const scalar_t* p = x + row * d + c0;
    constexpr int kPer = 16 / sizeof(scalar_t);  // elements per 16-byte load
    static_assert(kColsPerThread % kPer == 0, "whole 16-byte loads");
#pragma unroll
    for (int v = 0; v < kColsPerThread / kPer; ++v) {
      const u32x4 raw = *reinterpret_cast<const u32x4*>(p + v * kPer);
      __builtin_memcpy(&out[v * kPer], &raw, 16);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kColsPerThread; ++j) {
      const int c = c0 + j;
      out[j] = (row < n && c < d) ? x[row * d + c] : scalar_t(0);
    }
  }
}

template <typename scalar_t>
__global__ void __launch_bounds__(kThreads, 2)
    syrk_f64_kernel(const scalar_t* __restrict__ x, long long n, int d, int ntile, int splits, bool vec_ok,
                    double* __restrict__ cov_part, double* __restrict__ sum_part) {
  using st_t = typename Stage<scalar_t>::type;
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  st_t* lds = reinterpret_cast<st_t*>(lds_raw);  // [2 stages][2 panels][kKC][kLdsRow]
  constexpr int kPanel = kKC * kLdsRow;
  const int tiles = ntile * (ntile + 1) / 2;
  const int tile = blockIdx.x % tiles;
  const int split = blockIdx.x / tiles;
  int ti, tj;
  tile_coords(tile, ntile, ti, tj);
  const int i0 = ti * kTile, j0 = tj * kTile;
  const bool diag = ti == tj;
  const long long chunks = (n + kKC - 1) / kKC;
  const long long per = (chunks + splits - 1) / splits;
  const long long c_beg = static_cast<long long>(split) * per;
  const long long c_end = min(chunks, c_beg + per);

  const int tid = threadIdx.x;
  const int lr = tid / kThrPerRow;                     // sample row (0..31) staged by this thread
  const int lc = (tid % kThrPerRow) * kColsPerThread;  // first of its panel columns
  const int wave = tid / kWave, lane = tid & (kWave - 1);
  const int wr = wave >> 2, wc = wave & 3;             // wave tile: rows wr*64.., cols wc*32..

  f64x4 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
  double colsum = 0.0;  // diagonal tiles: threads 0..127 own one column's running sum

  scalar_t ra[kColsPerThread], rb[kColsPerThread];
  auto load = [&](long long chunk) {
    const long long row = chunk * kKC + lr;
    load_cols(x, n, d, row, i0 + lc, vec_ok, ra);
    if (!diag) load_cols(x, n, d, row, j0 + lc, vec_ok, rb);
  };
  auto store = [&](int stage) {
    st_t* a = lds + (stage * 2) * kPanel + lr * kLdsRow + lc;
#pragma unroll
    for (int e = 0; e < kColsPerThread; ++e) a[e] = to_stage(ra[e]);
    if (!diag) {
      st_t* b = lds + (stage * 2 + 1) * kPanel + lr * kLdsRow + lc;
#pragma unroll
      for (int e = 0; e < kColsPerThread; ++e) b[e] = to_stage(rb[e]);
    }
  };

  if (c_beg < c_end) {
    load(c_beg);
    store(0);
    if (c_beg + 1 < c_end) load(c_beg + 1);
  }
  __syncthreads();
  int stage = 0;
  for (long long c = c_beg; c < c_end; ++c) {
    const st_t* As = lds + (stage * 2) * kPanel;
    const st_t* Bs = diag ? As : lds + (stage * 2 + 1) * kPanel;  // diagonal tiles read both operands from A
    if (diag && tid < kTile) {
#pragma unroll 8
      for (int r = 0; r < kKC; ++r) colsum += static_cast<double>(As[r * kLdsRow + tid]);
    }
    st_t av[2][4], bv[2][2];  // stage type in registers: widened right at the MFMA
    auto rd = [&](int buf, int ks) {
      const int k = ks * 4 + (lane >> 4);
#pragma unroll
      for (int m = 0; m < 4; ++m) av[buf][m] = As[k * kLdsRow + wr * 64 + m * 16 + (lane & 15)];
#pragma unroll
      for (int q = 0; q < 2; ++q) bv[buf][q] = Bs[k * kLdsRow + wc * 32 + q * 16 + (lane & 15)];
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < kKC / 4; ++ks) {
      if (ks + 1 < kKC / 4) rd((ks + 1) & 1, ks + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(static_cast<double>(av[ks & 1][m]),
                                                           static_cast<double>(bv[ks & 1][q]), acc[m][q], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 1 < c_end) {
      store(stage ^ 1);                    // the other stage was released by the previous iteration's barrier
      if (c + 2 < c_end) load(c + 2);      // in flight across the barrier and the next chunk's MFMAs
    }
    __syncthreads();
    stage ^= 1;
  }

  // partial tile -> workspace [split][tile][128][128]
  double* out = cov_part + (static_cast<long long>(split) * tiles + tile) * kTile * kTile;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + m * 16 + (lane >> 4) + 4 * r;  // f64 MFMA C/D layout
        const int col = wc * 32 + q * 16 + (lane & 15);
        out[row * kTile + col] = acc[m][q][r];
      }
  if (diag && tid < kTile) {
    const int col = i0 + tid;
    if (col < d) sum_part[static_cast<long long>(split) * d + col] = colsum;
  }
}

// One block per (tile, 32x32 sub-block): fixed-order split reduction, coalesced add into cov[i][j] and, through an
// LDS transpose, into the mirrored cov[j][i] of off-diagonal tiles.  Extra blocks reduce the column sums.
__global__ void __launch_bounds__(256) syrk_finalize_kernel(const double* __restrict__ cov_part,
                                                            const double* __restrict__ sum_part, int d, int ntile,
                                                            int splits, double* __restrict__ cov,
                                                            double* __restrict__ sum) {
  constexpr int kSub = 32;
  constexpr int kSubs = (kTile / kSub) * (kTile / kSub);
  const int tiles = ntile * (ntile + 1) / 2;
  const int bid = blockIdx.x;
  if (bid < tiles * kSubs) {
    __shared__ double t[kSub][kSub + 1];
    const int tile = bid / kSubs, sub = bid % kSubs;
    int ti, tj;
    tile_coords(tile, ntile, ti, tj);
    const int sr = (sub / (kTile / kSub)) * kSub, sc = (sub % (kTile / kSub)) * kSub;
    const int tx = threadIdx.x % kSub, ty = threadIdx.x / kSub;  // 32 x 8
    for (int r = ty; r < kSub; r += 8) {
      const int e = (sr + r) * kTile + sc + tx;
      double v = 0.0;
      for (int s = 0; s < splits; ++s) v += cov_part[(static_cast<long long>(s) * tiles + tile) * kTile * kTile + e];
      t[r][tx] = v;
      const int i = ti * kTile + sr + r, j = tj * kTile + sc + tx;
      if (i < d && j < d) cov[static_cast<long long>(i) * d + j] += v;
    }
    if (ti != tj) {
      __syncthreads();
      for (int r = ty; r < kSub; r += 8) {
        // mirrored element (j, i): row j = tj*128 + sc + r, col i = ti*128 + sr + tx  -> value t[tx][r]
        const int j = tj * kTile + sc + r, i = ti * kTile + sr + tx;
        if (i < d && j < d) cov[static_cast<long long>(j) * d + i] += t[tx][r];
      }
    }
  } else {
    const int first = bid - tiles * kSubs;
    const int nblk = gridDim.x - tiles * kSubs;
    for (int c = first * blockDim.x + threadIdx.x; c < d; c += nblk * blockDim.x) {
      double v = 0.0;
      for (int s = 0; s < splits; ++s) v += sum_part[static_cast<long long>(s) * d + c];
      sum[c] += v;
    }
  }
}

}  // namespace

// features [N, D] (f32/f16/bf16/f64, contiguous); sum f64[D] and cov f64[D, D] are accumulated in place.
void feature_moments_update(const at::Tensor& features, at::Tensor sum, at::Tensor cov) {
  TM_CHECK_CUDA(features);
  TM_CHECK_CONTIG(features);
  TORCH_CHECK(features.dim() == 2, "feature_moments_update: features must be [N, D]");
  const long long n = features.size(0);
  const int d = static_cast<int>(features.size(1));
  TORCH_CHECK(sum.scalar_type() == at::kDouble && sum.is_contiguous() && sum.numel() == d,
              "feature_moments_update: sum must be contiguous f64[D]");
  TORCH_CHECK(cov.scalar_type() == at::kDouble && cov.is_contiguous() && cov.numel() == static_cast<long long>(d) * d,
              "feature_moments_update: cov must be contiguous f64[D, D]");
  if (n == 0 || d == 0) return;
  const int ntile = (d + kTile - 1) / kTile;
  const int tiles = ntile * (ntile + 1) / 2;
  const long long chunks = (n + kKC - 1) / kKC;
  // Split-K count: the kernel is MFMA-bound, so its time is the busiest CU's share of the work.  With `slots`
  // co-resident blocks (2 per CU) a grid of tiles * s blocks runs in ceil(tiles * s / slots) rounds of 1/s of a tile
  // each; pick the s (<= 64, >= 4 chunks per split) minimising that, e.g. D = 2048 (136 tiles) on 256 CUs: s = 15
  // (2040 blocks ~ 8 full rounds) instead of s = 4 (544 blocks = 2 full rounds + a 32-block tail).
  const int slots = 2 * cu_count(features.get_device());
  const long long max_s = std::max<long long>(1, std::min<long long>(64, chunks / 4));
  int splits = 1;
  double best = 1e30;
  for (int s_try = 1; s_try <= max_s; ++s_try) {
    const double rounds = static_cast<double>((static_cast<long long>(tiles) * s_try + slots - 1) / slots);
    const double cost = rounds / s_try * 1.0 + 1e-3 * s_try;  // small per-split cost: partial-tile write-back
    if (cost < best) {
      best = cost;
      splits = s_try;
    }
  }
  if (const char* env = std::getenv("TM_AMD_SYRK_SPLITS")) {
    const int v = std::atoi(env);
    if (v > 0) splits = static_cast<int>(std::min<long long>(v, std::max<long long>(1, chunks)));
  }
  auto opts = features.options().dtype(at::kDouble);
  at::Tensor cov_part = at::empty({static_cast<long long>(splits) * tiles * kTile * kTile}, opts);
  at::Tensor sum_part = at::zeros({static_cast<long long>(splits) * d}, opts);
  const bool vec_ok = (d * features.element_size()) % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(features.data_ptr()) % 16 == 0;
  auto s = stream();
  TM_DISPATCH_FLOAT(features.scalar_type(), "feature_moments_update", [&] {
    const size_t lds = 2 * 2 * kKC * kLdsRow * sizeof(typename Stage<scalar_t>::type);
    hipLaunchKernelGGL((syrk_f64_kernel<scalar_t>), dim3(static_cast<unsigned>(splits) * tiles), dim3(kThreads), lds,
                       s, reinterpret_cast<const scalar_t*>(features.data_ptr()), n, d, ntile, splits, vec_ok,
                       cov_part.data_ptr<double>(), sum_part.data_ptr<double>());
  });
  const int sum_blocks = (d + 255) / 256;
  hipLaunchKernelGGL(syrk_finalize_kernel, dim3(tiles * 16 + sum_blocks), dim3(256), 0, s, cov_part.data_ptr<double>(),
                     sum_part.data_ptr<double>(), d, ntile, splits, cov.data_ptr<double>(), sum.data_ptr<double>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("feature_moments_update(Tensor features, Tensor(a!) sum, Tensor(b!) cov) -> ()");
}

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("feature_moments_update", &tm_amd::feature_moments_update); }
