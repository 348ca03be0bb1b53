// fp32 "NT" GEMM on the gfx950 matrix cores with fused metric epilogues: C[i, j] = sum_k X[i, k] * Y[j, k].
//
// Used by pairwise euclidean / cosine / linear (F/pairwise/{euclidean,cosine,linear}.py: fp64 GEMM + norm trick /
// normalise + mm), KID's polynomial-kernel MMD sums (S/image/kid.py:33-66: three Gram matrices per subset, then
// masked sums) and MiFID's memorisation distance (S/image/mifid.py:36-63: normalise, mm, row min).  Instead of a
// library GEMM followed by elementwise/reduction passes over the [N, M] result, the epilogue consumes the
// accumulator tile in registers:
//
//   * v_mfma_f32_32x32x2_f32 (exact fp32 products, k-ordered fma chain -- 64 FLOP/clk/SIMD, the fp32 peak);
//     block 256 threads = 4 waves, block tile 128 x 128, wave tile 64 x 64 (2 x 2 MFMA tiles), k-step 32;
//   * K is permuted per lane half (half h owns k in [16h, 16h+16) of each 32-chunk) so every operand fragment of a
//     k-chunk is 16 contiguous floats: 4 x ds_read_b128 from LDS rows padded to 144 B (conflict-free);
//   * global -> LDS staging is double buffered with the next chunk prefetched into registers during the MFMAs;
//   * block ids are remapped so each XCD works through a contiguous band of row tiles (L2 reuse of the X band);
//   * epilogues: STORE (scale), EUCLID (sqrt(|x|^2 + |y|^2 - 2 x.y) with an exact difference-form recompute when
//     cancellation could cost more than ~1e-6 relative, zero_diagonal), COSINE (scaled by inverse norms),
//     POLY_SUM (KID: (gamma x.y + c)^degree summed, diagonal optionally excluded, one fp64 partial per block),
//     ROW_MIN (MiFID: min over j of 1 - |cos|, one partial per (row, column tile)), ROW_SUM (reduction='sum'/'mean').
// Batched over blockIdx.z, with per-batch strides or per-batch row-index gathers (KID subsets are read straight from
// the feature matrix through their index draws: the [subsets, m, D] gathered copies are never materialised).
#include <cstdlib>

#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBM = 128, kBN = 128, kNT = 256;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum Epi : int { kStore = 0, kEuclid = 1, kCosine = 2, kPolySum = 3, kRowMin = 4, kRowSum = 5, kRowColMax = 6 };

struct EpiParams {
  const float* nx;  // |x_i|^2 (EUCLID) or 1/|x_i| (COSINE, ROW_MIN)
  const float* ny;
  float scale;      // STORE / COSINE scale, POLY gamma
  float coef;       // POLY c
  int degree;       // POLY degree
  bool zero_diag;   // EUCLID: zero the diagonal; POLY_SUM: skip it
  bool sqrt_out;    // EUCLID: sqrt (else squared distance)
  float* out;       // [N, M] (STORE / EUCLID / COSINE) or partials
  float* out2;      // ROW_COL_MAX column partials [batch][tiles_n][M]
  double* dpart;    // POLY_SUM partials [batch * blocks]
  const int32_t* ix;  // optional row gather: X row i of batch b is X[ix[b * N + i]] (KID subsets); else batch-strided
  const int32_t* iy;
  int ldo;          // leading dim of out
  int part_cols;    // ROW_MIN / ROW_SUM partial columns (= column tiles)
  uint16_t* out16;  // STORE / COSINE with a 16-bit output: [N, M] in bf16 (out_kind 1) or fp16 (2), else nullptr
  int out_kind;
};

__device__ __forceinline__ float ipow(float b, int d) {
  float r = 1.0f;
  while (d) {
    if (d & 1) r *= b;
    b *= b;
    d >>= 1;
  }
  return r;
}

// 16-bit output: round to nearest even (the rounding of a library GEMM writing bf16 / fp16 from its fp32 accumulator)
__device__ __forceinline__ void store_out(const EpiParams& ep, long long idx, float v) {
  if (ep.out_kind == 0) {
    ep.out[idx] = v;
  } else if (ep.out_kind == 1) {
    ep.out16[idx] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
  } else {
    ep.out16[idx] = __builtin_bit_cast(uint16_t, static_cast<_Float16>(v));
  }
}

// Element-wise epilogues (STORE / COSINE / EUCLID) of the 16-bit kernels run on the TRANSPOSED accumulator: those
// kernels issue mfma(Y fragment, X fragment), so lane r holds output row wr + 32 a + r and, for e = 4 g + q, column
// wc + 32 b + 8 g + 4 h + q -- four consecutive columns per group.  Each group leaves as ONE vector store (4 x 16-bit =
// 8 B, 4 x fp32 = 16 B) instead of four 2- / 4-byte stores, with a quarter of the address arithmetic.
template <int EPI>
__host__ __device__ __forceinline__ constexpr bool rows_in_lanes() {
  return EPI == 0 || EPI == 1 || EPI == 2;  // kStore, kEuclid, kCosine
}

// interior tile of STORE / COSINE with aligned rows and no diagonal: every group is one unconditional vector store
template <int EPI, int NA, int NB, int OK>
__device__ __forceinline__ void tile_store_full(f32x16 (&acc)[NA][NB], const EpiParams& ep, int batch, int N, int M,
                                                int i0, int j0w) {
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int i = i0 + 32 * a;
    float f = ep.scale;
    if constexpr (EPI == 2) f *= ep.nx[batch * (long long)N + i];
    const long long rowbase = batch * (long long)N * ep.ldo + (long long)i * ep.ldo;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j0 = j0w + 32 * b + 8 * g + 4 * h;
        float v[4];
        if constexpr (EPI == 2) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(ep.ny + batch * (long long)M + j0);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[a][b][4 * g + q] * (f * w[q]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[a][b][4 * g + q] * f;
        }
        if constexpr (OK == 0) {
          *reinterpret_cast<f32x4*>(ep.out + rowbase + j0) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          uint16_t u[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            u[q] = OK == 1 ? __builtin_bit_cast(uint16_t, static_cast<__bf16>(v[q]))
                           : __builtin_bit_cast(uint16_t, static_cast<_Float16>(v[q]));
          *reinterpret_cast<uint2*>(ep.out16 + rowbase + j0) =
              make_uint2(u[0] | (static_cast<uint32_t>(u[1]) << 16), u[2] | (static_cast<uint32_t>(u[3]) << 16));
        }
      }
    }
  }
}

template <int EPI, int NA, int WC, typename Dist2, int NB = 2>
__device__ __forceinline__ void tile_epilogue_t(f32x16 (&acc)[NA][NB], const EpiParams& ep, int batch, int N, int M,
                                                int row0, int col0, Dist2 dist2, int tile_rows = 0,
                                                int tile_cols = 0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave / WC) * 32 * NA, wc = (wave % WC) * 32 * NB;
  const int h = lane >> 5, r = lane & 31;
  const bool vec = (ep.ldo & 3) == 0 &&
                   ((ep.out_kind ? reinterpret_cast<uintptr_t>(ep.out16) : reinterpret_cast<uintptr_t>(ep.out)) &
                    (ep.out_kind ? 7 : 15)) == 0;
  if constexpr (EPI == 0 || EPI == 2) {
    // (the cosine multiplies scale * nx_i first, then ny_j: the order of the general path below up to rounding)
    const bool full = vec && !ep.zero_diag && row0 + tile_rows <= N && col0 + tile_cols <= M &&
                      (EPI == 0 || (((batch * (long long)M) & 3) == 0 &&
                                    (reinterpret_cast<uintptr_t>(ep.ny) & 15) == 0));
    if (full) {
      const int i0 = row0 + wr + r, j0w = col0 + wc;
      if (ep.out_kind == 0) tile_store_full<EPI, NA, NB, 0>(acc, ep, batch, N, M, i0, j0w);
      else if (ep.out_kind == 1) tile_store_full<EPI, NA, NB, 1>(acc, ep, batch, N, M, i0, j0w);
      else tile_store_full<EPI, NA, NB, 2>(acc, ep, batch, N, M, i0, j0w);
      return;
    }
  }
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int i = row0 + wr + 32 * a + r;
    if (i >= N) continue;
    float nxi = 0.f;
    if constexpr (EPI != 0) nxi = ep.nx[batch * (long long)N + i];
    const long long rowbase = batch * (long long)N * ep.ldo + (long long)i * ep.ldo;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j0 = col0 + wc + 32 * b + 8 * g + 4 * h;
        if (j0 >= M) continue;
        float v[4];
        float nyq[4] = {0.f, 0.f, 0.f, 0.f};  // the group's four column factors: one 16-byte load when aligned
        if constexpr (EPI != 0) {
          const long long o = batch * (long long)M + j0;
          if (j0 + 3 < M && (o & 3) == 0) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(ep.ny + o);
            nyq[0] = w[0], nyq[1] = w[1], nyq[2] = w[2], nyq[3] = w[3];
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (j0 + q < M) nyq[q] = ep.ny[o + q];
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = j0 + q;
          float x = acc[a][b][4 * g + q];
          if (j < M) {
            if constexpr (EPI == 0) {
              x = (ep.zero_diag && i == j) ? 0.f : x * ep.scale;
            } else if constexpr (EPI == 2) {
              x = (ep.zero_diag && i == j) ? 0.f : x * nxi * nyq[q] * ep.scale;
            } else {
              const float s2 = nxi + nyq[q];
              float d2 = s2 - 2.0f * x;
              if (d2 < s2 * (1.0f / 128.0f)) d2 = dist2(i, j);  // cancellation guard: exact difference form
              d2 = fmaxf(d2, 0.f);
              if (ep.zero_diag && i == j) d2 = 0.f;
              x = ep.sqrt_out ? sqrtf(d2) : d2;
            }
          }
          v[q] = x;
        }
        if (vec && j0 + 3 < M) {
          if (ep.out_kind == 0) {
            *reinterpret_cast<f32x4*>(ep.out + rowbase + j0) = f32x4{v[0], v[1], v[2], v[3]};
          } else {
            uint16_t u[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
              u[q] = ep.out_kind == 1 ? __builtin_bit_cast(uint16_t, static_cast<__bf16>(v[q]))
                                      : __builtin_bit_cast(uint16_t, static_cast<_Float16>(v[q]));
            const uint2 w = make_uint2(u[0] | (static_cast<uint32_t>(u[1]) << 16),
                                       u[2] | (static_cast<uint32_t>(u[3]) << 16));
            *reinterpret_cast<uint2*>(ep.out16 + rowbase + j0) = w;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (j0 + q < M) store_out(ep, rowbase + j0 + q, v[q]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ shared epilogue
// One implementation for every kernel of this file.  The block tile is TM x TM, NT threads = NT / 64 waves laid out as
// (NT / 64 / WC) wave rows x WC wave columns; a wave owns NA x 2 MFMA 32 x 32 tiles: acc[a][b][e] holds
// row wr + 32 a + (e & 3) + 8 (e >> 2) + 4 h, column wc + 32 b + r (the C/D map of every 32x32 MFMA form used here:
// f32 32x32x2, bf16 / f16 32x32x16).  Reduction scratch reuses the staging LDS (`smem`), after a barrier.
// `dist2(i, j)`: the exact difference-form squared distance of rows i, j (EUCLID's cancellation recompute).
template <int EPI, int NA, int WC, int TM, int NT, typename Dist2>
__device__ __forceinline__ void tile_epilogue(f32x16 (&acc)[NA][2], float* smem, const EpiParams& ep, int batch, int N,
                                              int M, int row0, int col0, int ti, int tj, int tiles_n, int tile,
                                              Dist2 dist2) {
  constexpr int NWR = NT / 64 / WC;  // wave rows
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave / WC) * 32 * NA, wc = (wave % WC) * 64;
  const int h = lane >> 5, r = lane & 31;
  __syncthreads();
  if constexpr (EPI == kStore || EPI == kEuclid || EPI == kCosine) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int j = col0 + wc + 32 * b + r;
        if (j >= M) continue;
        float nyj = 0.f;
        if constexpr (EPI != kStore) nyj = ep.ny[batch * (long long)M + j];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int i = row0 + wr + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (i >= N) continue;
          float v = acc[a][b][e];
          if constexpr (EPI == kStore) {
            v = (ep.zero_diag && i == j) ? 0.f : v * ep.scale;
          } else if constexpr (EPI == kCosine) {
            v = (ep.zero_diag && i == j) ? 0.f : v * ep.nx[batch * (long long)N + i] * nyj * ep.scale;
          } else {
            const float s2 = ep.nx[batch * (long long)N + i] + nyj;
            float d2 = s2 - 2.0f * v;
            if (d2 < s2 * (1.0f / 128.0f)) d2 = dist2(i, j);  // cancellation guard: exact difference form
            d2 = fmaxf(d2, 0.f);
            if (ep.zero_diag && i == j) d2 = 0.f;
            v = ep.sqrt_out ? sqrtf(d2) : d2;
          }
          store_out(ep, batch * (long long)N * ep.ldo + (long long)i * ep.ldo + j, v);
        }
      }
  } else if constexpr (EPI == kPolySum) {
    double part = 0.0;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int j = col0 + wc + 32 * b + r;
        if (j >= M) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int i = row0 + wr + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (i >= N || (ep.zero_diag && i == j)) continue;
          part += static_cast<double>(ipow(fmaf(acc[a][b][e], ep.scale, ep.coef), ep.degree));
        }
      }
    part = wave_sum(part);
    double* red = reinterpret_cast<double*>(smem);
    if (lane == 0) red[wave] = part;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int w = 0; w < NT / 64; ++w) t += red[w];
      ep.dpart[(long long)batch * gridDim.x + tile] = t;
    }
  } else if constexpr (EPI == kRowColMax) {
    // row maxima over this block's TM columns and column maxima over its TM rows (scaled dot)
    float* redr = smem;            // [WC wave columns][TM]
    float* redc = smem + WC * TM;  // [NWR wave rows][TM]
#pragma unroll
    for (int a = 0; a < NA; ++a) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int il = wr + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int i = row0 + il;
        float v = -3.0e38f;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int j = col0 + wc + 32 * b + r;
          if (j < M && i < N) v = fmaxf(v, acc[a][b][e] * ep.scale);
        }
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
        if (r == 0) redr[(wave % WC) * TM + il] = v;
      }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int jl = wc + 32 * b + r;
      float v = -3.0e38f;
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int i = row0 + wr + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (i < N && col0 + jl < M) v = fmaxf(v, acc[a][b][e] * ep.scale);
        }
      v = fmaxf(v, __shfl_xor(v, 32, 64));  // the two lane halves hold interleaved row groups
      if (h == 0) redc[(wave / WC) * TM + jl] = v;
    }
    __syncthreads();
    for (int t = tid; t < 2 * TM; t += NT) {
      if (t < TM) {
        const int i = row0 + t;
        if (i < N) {
          float v = redr[t];
#pragma unroll
          for (int w = 1; w < WC; ++w) v = fmaxf(v, redr[w * TM + t]);
          ep.out[(long long)batch * N * ep.part_cols + (long long)i * ep.part_cols + tj] = v;
        }
      } else {
        const int jl = t - TM, j = col0 + jl;
        if (j < M) {
          float v = redc[jl];
#pragma unroll
          for (int w = 1; w < NWR; ++w) v = fmaxf(v, redc[w * TM + jl]);
          ep.out2[((long long)batch * tiles_n + ti) * M + j] = v;
        }
      }
    }
  } else {
    // ROW_MIN of (1 - |cos|) or ROW_SUM of the (scaled) dot: per row over this block's TM columns
    float* red = smem;  // [WC][TM]
#pragma unroll
    for (int a = 0; a < NA; ++a) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int il = wr + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int i = row0 + il;
        float v = EPI == kRowMin ? 3.0e38f : 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int j = col0 + wc + 32 * b + r;
          if (j >= M || i >= N) continue;
          float x = acc[a][b][e];
          if constexpr (EPI == kRowMin) {
            x = 1.0f - fabsf(x * ep.nx[batch * (long long)N + i] * ep.ny[batch * (long long)M + j]);
            v = fminf(v, x);
          } else {
            v += x * ep.scale;
          }
        }
        // reduce over the 32 columns held by this lane half (lanes r = 0..31)
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) {
          const float o = __shfl_xor(v, off, 64);
          v = EPI == kRowMin ? fminf(v, o) : v + o;
        }
        if (r == 0) red[(wave % WC) * TM + il] = v;
      }
    }
    __syncthreads();
    for (int t = tid; t < TM; t += NT) {
      const int i = row0 + t;
      if (i < N) {
        float v = red[t];
#pragma unroll
        for (int w = 1; w < WC; ++w) v = EPI == kRowMin ? fminf(v, red[w * TM + t]) : v + red[w * TM + t];
        ep.out[(long long)batch * N * ep.part_cols + (long long)i * ep.part_cols + tj] = v;
      }
    }
  }
}

template <int EPI, int STAGES, int kBK>
__global__ __launch_bounds__(kNT) void gemm_nt_kernel(const float* __restrict__ X, const float* __restrict__ Y, int N,
                                                       int M, int D, long long bx, long long by, int tiles_m,
                                                       EpiParams ep) {
  // LDS row: kBK floats + 4 pad (conflict-free ds_read_b128 of a lane half's slab); kQ f32x4 per lane-half slab;
  // kLd float4 loads per thread per operand and k-chunk
  constexpr int kRowF = kBK + 4, kQ = kBK / 8, kLd = kBM * (kBK / 4) / kNT, kC4 = kBK / 4;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sa = smem;                          // [STAGES][kBM][kRowF]
  float* sb = smem + STAGES * kBM * kRowF;   // [STAGES][kBN][kRowF]
  const int batch = blockIdx.z;
  const int32_t* gix = ep.ix ? ep.ix + (long long)batch * N : nullptr;
  const int32_t* giy = ep.iy ? ep.iy + (long long)batch * M : nullptr;
  if (!gix) X += batch * bx;
  if (!giy) Y += batch * by;
  auto xrow = [&](int i) -> const float* { return X + (long long)(gix ? gix[i] : i) * D; };
  auto yrow = [&](int j) -> const float* { return Y + (long long)(giy ? giy[j] : j) * D; };
  // XCD-aware tile order: hardware deals consecutive block ids round-robin over 8 XCDs; give each XCD a contiguous
  // band of (row-major) tiles
  const int tiles_n = (N + kBM - 1) / kBM;
  const int total = tiles_n * tiles_m;
  const int bid = blockIdx.x;
  const int per = (total + 7) / 8;
  const int tile = (bid % 8) * per + bid / 8;
  if (tile >= total) return;
  const int ti = tile / tiles_m, tj = tile - ti * tiles_m;
  const int row0 = ti * kBM, col0 = tj * kBN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;  // wave tile origin inside the block tile
  const int h = lane >> 5, r = lane & 31;

  // staging: 128 rows x 8 float4 per operand = 1024 float4 = 4 per thread.  Row pointers (gathered or strided) and
  // row validity are resolved ONCE per tile, so the k-loop's prefetch is 8 independent float4 loads with no index
  // loads or waits in between.  D % 4 == 0 (host check): a float4 is either wholly inside K or wholly past it.
  float4 ra[kLd], rb[kLd];
  const float* pa_row[kLd];
  const float* pb_row[kLd];
  bool va_row[kLd], vb_row[kLd];
  int c4_of[kLd];
#pragma unroll
  for (int q = 0; q < kLd; ++q) {
    const int idx = tid + q * kNT;
    const int rr = idx / kC4;
    c4_of[q] = (idx % kC4) * 4;
    const int gi = row0 + rr, gj = col0 + rr;
    va_row[q] = gi < N;
    vb_row[q] = gj < M;
    pa_row[q] = va_row[q] ? xrow(gi) : X;
    pb_row[q] = vb_row[q] ? yrow(gj) : Y;
  }
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < kLd; ++q) {
      const int gk = k0 + c4_of[q];
      const bool kin = gk < D;
      float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
      if (kin && va_row[q]) va = *reinterpret_cast<const float4*>(pa_row[q] + gk);
      if (kin && vb_row[q]) vb = *reinterpret_cast<const float4*>(pb_row[q] + gk);
      ra[q] = va;
      rb[q] = vb;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < kLd; ++q) {
      const int idx = tid + q * kNT;
      const int rr = idx / kC4, c4 = (idx % kC4) * 4;
      *reinterpret_cast<float4*>(sa + (buf * kBM + rr) * kRowF + c4) = ra[q];
      *reinterpret_cast<float4*>(sb + (buf * kBN + rr) * kRowF + c4) = rb[q];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int nk = (D + kBK - 1) / kBK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = STAGES == 2 ? (kc & 1) : 0;
    if (kc + 1 < nk) gload((kc + 1) * kBK);
    // fragments: lane (r, h) -> rows wr + 32a + r, k in [h kBK/2, (h + 1) kBK/2), read one float4 (4 k-steps) at a
    // time and software-pipelined: the ds_reads of quarter q + 1 are in flight while the 16 MFMAs of quarter q issue
    const float* pa0 = sa + (buf * kBM + wr + r) * kRowF + (kBK / 2) * h;
    const float* pb0 = sb + (buf * kBN + wc + r) * kRowF + (kBK / 2) * h;
    f32x4 ca[2], cb[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      ca[a] = *reinterpret_cast<const f32x4*>(pa0 + 32 * a * kRowF);
      cb[a] = *reinterpret_cast<const f32x4*>(pb0 + 32 * a * kRowF);
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      f32x4 na[2], nb[2];
      if (q < kQ - 1) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          na[a] = *reinterpret_cast<const f32x4*>(pa0 + 32 * a * kRowF + 4 * (q + 1));
          nb[a] = *reinterpret_cast<const f32x4*>(pb0 + 32 * a * kRowF + 4 * (q + 1));
        }
      }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[a][s4], cb[b][s4], acc[a][b], 0, 0, 0);
      }
      if (q < kQ - 1) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          ca[a] = na[a];
          cb[a] = nb[a];
        }
      }
    }
    if (kc + 1 < nk) {
      if constexpr (STAGES == 1) __syncthreads();  // every wave is done reading the single buffer
      sstore(STAGES == 2 ? (buf ^ 1) : 0);
      __syncthreads();
    }
  }

  // ----------------------------------------------------------------------------------------------- epilogue
  tile_epilogue<EPI, 2, 2, kBM, kNT>(acc, smem, ep, batch, N, M, row0, col0, ti, tj, tiles_n, tile,
                                     [&](int i, int j) {
                                       const float* xr = xrow(i);
                                       const float* yr = yrow(j);
                                       float t = 0.f;
                                       for (int k = 0; k < D; ++k) {
                                         const float d = xr[k] - yr[k];
                                         t = fmaf(d, d, t);
                                       }
                                       return t;
                                     });
}

// ------------------------------------------------------------------------------------------------ 256 x 256 tiles
// Large problems (D % 32 == 0, both sides >= 256): block tile 256 x 256, 8 waves as 2 (rows) x 4 (columns), wave tile
// 128 x 64 = 4 x 2 MFMA 32x32 tiles (128 accumulators per lane), k-step 32.  Versus the 128 x 128 kernel above this
// halves the LDS traffic and the barriers per MFMA, and stages global -> LDS with global_load_lds_dwordx4 (no VGPR
// round trip, no write pass): two 64 KiB LDS stages, the next k-chunk's DMAs in flight while the current one is
// multiplied, ONE barrier per k-chunk (the barrier that publishes chunk k also proves every wave finished chunk k-1,
// so chunk k+1 may be staged into that buffer right after it).  The 128 x 128 kernel's waves spent 84 % of their
// cycles in s_waitcnt at 4096^2 x 2048 (profiles/r03_gemm_vs_hipblaslt.md).
//
// LDS image: per operand 256 rows x 8 16-byte chunks (128 B rows, unpadded: a DMA instruction writes 1 KiB = 8 rows
// lane-linearly), chunk c of row r stored at c ^ ((r >> 1) & 7) -- the swizzle is applied on the global SOURCE
// address of each lane, and makes the fragment reads (32 rows x one chunk per lane half) bank-conflict free.
constexpr int kGM = 256, kGN = 256, kGT = 512, kGK = 32;

template <int EPI>
__global__ __launch_bounds__(kGT) void gemm_nt_big_kernel(const float* __restrict__ X, const float* __restrict__ Y,
                                                          int N, int M, int D, long long bx, long long by, int tiles_m,
                                                          EpiParams ep, bool pipe) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [2 stages][A 256 x 32 | B 256 x 32]
  constexpr int kStage = (kGM + kGN) * kGK;                    // floats per stage
  const int batch = blockIdx.z;
  const int32_t* gix = ep.ix ? ep.ix + (long long)batch * N : nullptr;
  const int32_t* giy = ep.iy ? ep.iy + (long long)batch * M : nullptr;
  if (!gix) X += batch * bx;
  if (!giy) Y += batch * by;
  auto xrow = [&](int i) -> const float* { return X + (long long)(gix ? gix[i] : i) * D; };
  auto yrow = [&](int j) -> const float* { return Y + (long long)(giy ? giy[j] : j) * D; };
  const int tiles_n = (N + kGM - 1) / kGM;
  const int total = tiles_n * tiles_m;
  const int bid = blockIdx.x;
  const int per = (total + 7) / 8;
  const int tile = (bid % 8) * per + bid / 8;  // XCD-aware: each XCD takes a contiguous band of row-major tiles
  if (tile >= total) return;
  const int ti = tile / tiles_m, tj = tile - ti * tiles_m;
  const int row0 = ti * kGM, col0 = tj * kGN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 2) * 128, wc = (wave & 3) * 64;
  const int h = lane >> 5, r = lane & 31;

  // DMA sources: wave w moves rows [32 w, 32 w + 32) of each operand tile, 8 rows (1 KiB) per instruction; lane l
  // of instruction q covers row 32 w + 8 q + l / 8, LDS chunk l % 8 = logical chunk (l % 8) ^ ((row >> 1) & 7).
  // Rows past N / M read a valid row (their products are never stored).
  const float* srcA[4];
  const float* srcB[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = 32 * wave + 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ ((rr >> 1) & 7);
    const int gi = min(row0 + rr, N - 1), gj = min(col0 + rr, M - 1);
    srcA[q] = xrow(gi) + 4 * c;
    srcB[q] = yrow(gj) + 4 * c;
  }
  typedef __attribute__((address_space(3))) void lds_t;
  typedef __attribute__((address_space(1))) void glb_t;
  auto stage = [&](int kc, int buf) {
    float* sa = smem + buf * kStage;
    float* sb = sa + kGM * kGK;
    const int k0 = kc * kGK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_global_load_lds((glb_t*)(srcA[q] + k0), (lds_t*)(sa + (32 * wave + 8 * q) * kGK), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((glb_t*)(srcB[q] + k0), (lds_t*)(sb + (32 * wave + 8 * q) * kGK), 16, 0, 0);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  // fragment addresses: lane (r, h) reads row wr + 32 a + r (A) / wc + 32 b + r (B), logical chunk 4 h + q
  const int swz_a = ((wr + r) >> 1) & 7;  // (32 a keeps (row >> 1) & 7: 32 rows shift it by 16)
  const int swz_b = ((wc + r) >> 1) & 7;
  const int nk = D / kGK;
  // fragment slice q (k columns 8q .. 8q + 7 of the chunk, as 4 x 2 f32x4) of LDS stage `buf`
  auto frag = [&](int buf, int q, f32x4* fa, f32x4* fb) {
    const float* sa = smem + buf * kStage + (wr + r) * kGK;
    const float* sb = smem + buf * kStage + kGM * kGK + (wc + r) * kGK;
#pragma unroll
    for (int a = 0; a < 4; ++a) fa[a] = *reinterpret_cast<const f32x4*>(sa + 32 * a * kGK + 4 * ((4 * h + q) ^ swz_a));
#pragma unroll
    for (int b = 0; b < 2; ++b) fb[b] = *reinterpret_cast<const f32x4*>(sb + 32 * b * kGK + 4 * ((4 * h + q) ^ swz_b));
  };
  auto mfma16 = [&](const f32x4* fa, const f32x4* fb) {
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a][s4], fb[b][s4], acc[a][b], 0, 0, 0);
  };
  f32x4 ca[4], cb[2], na[4], nb[2];
  if (pipe) {
    // The barrier of chunk kc+1 sits INSIDE chunk kc: after the last LDS read of chunk kc (slice 3, loaded during
    // slice 2's MFMAs) and before slice 3's MFMAs, so the matrix pipe still holds slice 2's MFMAs while waves meet
    // there, and chunk kc+1's first slice is read while slice 3 multiplies -- the pipe never drains at a chunk
    // boundary.  The barrier also proves every wave is done reading stage kc & 1: chunk kc+2's DMAs go there next.
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (nk > 1) stage(1, 1);
    frag(0, 0, ca, cb);
    for (int kc = 0; kc < nk; ++kc) {
      const int buf = kc & 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool more = q < 3 || kc + 1 < nk;
        if (q < 3) {
          frag(buf, q + 1, na, nb);
        } else if (kc + 1 < nk) {
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // chunk kc+1 DMAs; chunk kc reads landed
          __builtin_amdgcn_s_barrier();
          if (kc + 2 < nk) stage(kc + 2, buf);
          frag(buf ^ 1, 0, na, nb);
        }
        mfma16(ca, cb);
        if (more) {
#pragma unroll
          for (int a = 0; a < 4; ++a) ca[a] = na[a];
#pragma unroll
          for (int b = 0; b < 2; ++b) cb[b] = nb[b];
        }
      }
    }
  } else {
    stage(0, 0);
    for (int kc = 0; kc < nk; ++kc) {
      const int buf = kc & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs of chunk kc (the only ones in flight)
      __builtin_amdgcn_s_barrier();                     // ... and every other wave's; all done with chunk kc - 1
      if (kc + 1 < nk) stage(kc + 1, buf ^ 1);          // in flight during this chunk's MFMAs
      frag(buf, 0, ca, cb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q < 3) frag(buf, q + 1, na, nb);
        mfma16(ca, cb);
        if (q < 3) {
#pragma unroll
          for (int a = 0; a < 4; ++a) ca[a] = na[a];
#pragma unroll
          for (int b = 0; b < 2; ++b) cb[b] = nb[b];
        }
      }
    }
  }

  // ----------------------------------------------------------------------------------------------- epilogue
  // (no DMA is in flight: the last chunk issued none)
  tile_epilogue<EPI, 4, 4, kGM, kGT>(acc, smem, ep, batch, N, M, row0, col0, ti, tj, tiles_n, tile,
                                     [&](int i, int j) {
                                       const float* xr = xrow(i);
                                       const float* yr = yrow(j);
                                       float t = 0.f;
                                       for (int k = 0; k < D; ++k) {
                                         const float d = xr[k] - yr[k];
                                         t = fmaf(d, d, t);
                                       }
                                       return t;
                                     });
}

// ------------------------------------------------------------------------------------------ 16-bit operands
// bf16 / fp16 operands on the 16-bit matrix cores: v_mfma_f32_32x32x16_{bf16,f16} (fp32 accumulate; 16x the rate of the
// fp32 MFMA above), read straight from the caller's 16-bit tensors -- no fp32 upcast copy.  The structure is the
// 256 x 256 kernel's (the 128 x 128 form for small problems): a k-chunk of 64 elements is a 128-byte LDS row, exactly
// the fp32 kernel's 32-float chunk, staged by global_load_lds_dwordx4 into two swizzled stages (chunk c of row r at
// c ^ ((r >> 1) & 7)), one barrier per chunk placed inside its last k-step.  A chunk is 4 MFMA k-steps of 16: lane
// (r, h) of step s reads logical chunk 2 s + h of its row = A[row][16 s + 8 h + j] / B[k][col] for j = 0..7 (the
// operand map of the 32x32x16 forms), one ds_read_b128 per fragment.  K need not be a multiple of 64: a 16-byte
// source chunk at or past D (D % 8 == 0) is redirected to a zero block, so the DMA itself writes the zero padding.
template <typename T>
struct Mfma16;
template <>
struct Mfma16<__bf16> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 run(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float to_f32(uint16_t v) { return static_cast<float>(__builtin_bit_cast(__bf16, v)); }
};
template <>
struct Mfma16<_Float16> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 run(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float to_f32(uint16_t v) {
    return static_cast<float>(__builtin_bit_cast(_Float16, v));
  }
};

__device__ __attribute__((aligned(16))) uint32_t g_zero_chunk[4];  // the DMA source of K padding (never written)

// Measured and dropped (profiles/r05_bench_gemm16_ring_sweep_last.jsonl, r05_bench_gemm16_v2_ring*.jsonl and the
// round-5 log): a 4-deep / 2-deep ring of 32-wide k-chunks (no faster; at 165 VGPRs two 512-thread blocks never share
// a CU), four waves of 128 x 128 per wave (512 VGPRs, spills: 10-20 % slower), and a persistent grid-stride form that
// overlaps a tile's stores with the next tile's DMA (within 5 %).
// Round 6 (profiles/r06_gemm16_loop_probes.txt, r06_bench_gemm16_pingpong.jsonl): a phased "ping-pong" loop after
// cdna_hip_programming.md §5 (32-deep K pieces through a 4-slot LDS ring, counted vmcnt across barriers, the two wave rows
// one barrier apart so one wave per SIMD issues MFMAs while the other reads) ran 925-960 TFLOP/s at 4096^2 x 2048 against
// 951-961 for this loop; its timing probes put the ceiling in the MFMA-and-barrier skeleton itself (no DMA: 1193, no DMA
// and no barriers: 1222), not in the staging.
// Also measured and dropped in round 6 (profiles/r06_bench_gemm16_w4_variant.jsonl): the library's own shape at this
// tile, four waves of 128 x 128 (acc[4][4], 512 registers per lane, no spill; half the LDS reads per MFMA): 903 vs 956
// TFLOP/s at 4096^2 x 2048, slower on every shape -- one wave per SIMD leaves the chunk barrier and the first fragment
// reads after it exposed.
// GRAN: bytes per DMA lane.  16 (the fast form) needs 16-byte aligned rows (D % 8 == 0, 16-byte aligned bases);
// rows of any other width are staged in place into the SAME swizzled LDS layout, the K tail zero-filled element by
// element -- no padded copy and no fp32 upcast of the operands: 4-byte DMA lanes for even widths (4x the
// instructions), register staging of whole 16-byte slots for odd ones (GRAN 2).
template <int EPI, typename T, int TM, int GRAN = 16>
__global__ __launch_bounds__(TM == 256 ? 512 : 256) void gemm_nt_h16_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ Y, int N, int M, int D, long long bx, long long by,
    int tiles_m, EpiParams ep) {
  constexpr int NT = TM == 256 ? 512 : 256, WC = TM == 256 ? 4 : 2, NA = TM == 256 ? 4 : 2, KC = 64;
  typedef typename Mfma16<T>::v8 v8;
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [2 stages][A TM x 64 | B TM x 64] 16-bit elements
  uint16_t* sh = reinterpret_cast<uint16_t*>(smem);
  constexpr int kStage = 2 * TM * KC;  // elements per stage
  const int batch = blockIdx.z;
  const int32_t* gix = ep.ix ? ep.ix + (long long)batch * N : nullptr;
  const int32_t* giy = ep.iy ? ep.iy + (long long)batch * M : nullptr;
  if (!gix) X += batch * bx;
  if (!giy) Y += batch * by;
  auto xrow = [&](int i) -> const uint16_t* { return X + (long long)(gix ? gix[i] : i) * D; };
  auto yrow = [&](int j) -> const uint16_t* { return Y + (long long)(giy ? giy[j] : j) * D; };
  const int tiles_n = (N + TM - 1) / TM;
  const int total = tiles_n * tiles_m;
  const int bid = blockIdx.x;
  const int per = (total + 7) / 8;
  const int tile = (bid % 8) * per + bid / 8;  // XCD-aware: each XCD takes a contiguous band of row-major tiles
  if (tile >= total) return;
  const int ti = tile / tiles_m, tj = tile - ti * tiles_m;
  const int row0 = ti * TM, col0 = tj * TM;
  // the wave index as an SGPR value: the DMA's LDS destinations (M0) are then scalar arithmetic, not a
  // v_readfirstlane per instruction
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = (wave / WC) * 32 * NA, wc = (wave % WC) * 64;
  const int h = lane >> 5, r = lane & 31;

  // DMA: wave w moves rows [32 w, 32 w + 32) of each operand tile (TM / waves = 32 for both tile sizes), 8 rows
  // (1 KiB) per instruction; lane l of instruction q covers row 32 w + 8 q + l / 8, LDS slot l % 8 = logical chunk
  // (l % 8) ^ ((row >> 1) & 7).  Rows past N / M read a valid row (their products are never stored).
  const uint16_t* srcA[4];
  const uint16_t* srcB[4];
  int kof[4];  // element offset of the lane's logical chunk inside a k-chunk
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = 32 * wave + 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ ((rr >> 1) & 7);
    kof[q] = 8 * c;
    srcA[q] = xrow(min(row0 + rr, N - 1)) + 8 * c;
    srcB[q] = yrow(min(col0 + rr, M - 1)) + 8 * c;
  }
  typedef __attribute__((address_space(3))) void lds_t;
  typedef __attribute__((address_space(1))) void glb_t;
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_chunk);
  auto stage = [&](int kc, int buf) {
    uint16_t* sa = sh + buf * kStage;
    uint16_t* sb = sa + TM * KC;
    const int k0 = kc * KC;
    if constexpr (GRAN == 16) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool in = k0 + kof[q] < D;
        __builtin_amdgcn_global_load_lds((glb_t*)(in ? srcA[q] + k0 : zero), (lds_t*)(sa + (32 * wave + 8 * q) * KC),
                                         16, 0, 0);
        __builtin_amdgcn_global_load_lds((glb_t*)(in ? srcB[q] + k0 : zero), (lds_t*)(sb + (32 * wave + 8 * q) * KC),
                                         16, 0, 0);
      }
    } else if constexpr (GRAN == 2) {
      // odd widths: 2-byte rows.  The LDS-DMA forms below 4 bytes do not pack lanes 2 bytes apart, so these rows
      // are register-staged: each lane assembles whole 16-byte slots (8 elements, element-wise K bound) and writes
      // them to their swizzled LDS place; the barrier protocol is unchanged (the writes land before the barrier
      // that precedes the reads)
      constexpr int kSlots = TM * (KC / 8) / NT;  // slots per thread and operand
#pragma unroll
      for (int v = 0; v < kSlots; ++v) {
        const int id = tid + v * NT;
        const int rr = id >> 3, slot = id & 7;
        const int k = k0 + 8 * (slot ^ ((rr >> 1) & 7));
        const uint16_t* pa = xrow(min(row0 + rr, N - 1)) + k;
        const uint16_t* pb = yrow(min(col0 + rr, M - 1)) + k;
        uint16_t ea[8], eb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool in = k + e < D;
          ea[e] = in ? pa[e] : uint16_t(0);
          eb[e] = in ? pb[e] : uint16_t(0);
        }
        *reinterpret_cast<uint4*>(sa + rr * KC + 8 * slot) = __builtin_bit_cast(uint4, ea);
        *reinterpret_cast<uint4*>(sb + rr * KC + 8 * slot) = __builtin_bit_cast(uint4, eb);
      }
    } else {
      // E elements per lane, LPR lanes per 64-element LDS row, RPI rows per instruction: lane l of instruction q
      // fills element slot (l % LPR) * E of row 32 w + RPI q + l / LPR, i.e. logical chunk slot ^ swizzle(row)
      constexpr int E = GRAN / 2, LPR = KC / E, RPI = 64 / LPR;
      const int le = (lane % LPR) * E;
      const int slot = le >> 3, within = le & 7;
#pragma unroll 4
      for (int q = 0; q < 32 / RPI; ++q) {
        const int rr = 32 * wave + RPI * q + lane / LPR;
        const int k = k0 + 8 * (slot ^ ((rr >> 1) & 7)) + within;
        const bool in = k < D;  // (E = 2 only with D even: k and k + 1 are both inside or both past D)
        const uint16_t* pa = in ? xrow(min(row0 + rr, N - 1)) + k : zero;
        const uint16_t* pb = in ? yrow(min(col0 + rr, M - 1)) + k : zero;
        __builtin_amdgcn_global_load_lds((glb_t*)pa, (lds_t*)(sa + (32 * wave + RPI * q) * KC), 4, 0, 0);
        __builtin_amdgcn_global_load_lds((glb_t*)pb, (lds_t*)(sb + (32 * wave + RPI * q) * KC), 4, 0, 0);
      }
    }
  };

  f32x16 acc[NA][2];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int swz_a = ((wr + r) >> 1) & 7;  // (32 a keeps (row >> 1) & 7)
  const int swz_b = ((wc + r) >> 1) & 7;
  const int nk = (D + KC - 1) / KC;
  // fragments of k-step s of LDS stage `buf`: logical chunk 2 s + h of rows wr + 32 a + r / wc + 32 b + r
  auto frag = [&](int buf, int s, v8* fa, v8* fb) {
    const uint16_t* sa = sh + buf * kStage + (wr + r) * KC;
    const uint16_t* sb = sh + buf * kStage + TM * KC + (wc + r) * KC;
#pragma unroll
    for (int a = 0; a < NA; ++a) fa[a] = *reinterpret_cast<const v8*>(sa + 32 * a * KC + 8 * ((2 * s + h) ^ swz_a));
#pragma unroll
    for (int b = 0; b < 2; ++b) fb[b] = *reinterpret_cast<const v8*>(sb + 32 * b * KC + 8 * ((2 * s + h) ^ swz_b));
  };
  auto mma = [&](const v8* fa, const v8* fb) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if constexpr (rows_in_lanes<EPI>())
          acc[a][b] = Mfma16<T>::run(fb[b], fa[a], acc[a][b]);  // transposed tile: output rows in lanes
        else
          acc[a][b] = Mfma16<T>::run(fa[a], fb[b], acc[a][b]);
      }
  };
  // two fragment sets used in turn: k-step s multiplies set s & 1 while set (s + 1) & 1 loads (4 k-steps per chunk,
  // so the parity carries across chunks) -- no register copies between steps (the copying form spent ~3 v_mov per
  // MFMA)
  v8 fa[2][NA], fb[2][2];
  // chunk kc+1's barrier sits inside chunk kc, after its last LDS read (step 3's fragments, loaded during step 2's
  // MFMAs) and before step 3's MFMAs: the matrix pipe still holds step 2's work while the waves meet there
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (nk > 1) stage(1, 1);
  frag(0, 0, fa[0], fb[0]);
  // the last chunk is peeled off (no barrier, no next fragments): the loop body has one path, so the 128
  // accumulators are not shuffled between registers at control-flow joins
  auto chunk = [&](int kc, auto last_c) {
    constexpr bool kLast = decltype(last_c)::value;
    const int buf = kc & 1;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int cur = s4 & 1, nxt = cur ^ 1;
      if (s4 < 3) {
        frag(buf, s4 + 1, fa[nxt], fb[nxt]);
      } else if constexpr (!kLast) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // chunk kc+1 DMAs; chunk kc reads landed
        __builtin_amdgcn_s_barrier();
        if (kc + 2 < nk) stage(kc + 2, buf);
        frag(buf ^ 1, 0, fa[nxt], fb[nxt]);
      }
      mma(fa[cur], fb[cur]);
    }
  };
  for (int kc = 0; kc + 1 < nk; ++kc) chunk(kc, std::false_type{});
  chunk(nk - 1, std::true_type{});
  // (no DMA is in flight: the last chunk issued none)
  auto dist2 = [&](int i, int j) {
    const uint16_t* xr = xrow(i);
    const uint16_t* yr = yrow(j);
    float t = 0.f;
    for (int k = 0; k < D; ++k) {
      const float d = Mfma16<T>::to_f32(xr[k]) - Mfma16<T>::to_f32(yr[k]);
      t = fmaf(d, d, t);
    }
    return t;
  };
  if constexpr (rows_in_lanes<EPI>())
    tile_epilogue_t<EPI, NA, WC>(acc, ep, batch, N, M, row0, col0, dist2, TM, TM);
  else
    tile_epilogue<EPI, NA, WC, TM, NT>(acc, smem, ep, batch, N, M, row0, col0, ti, tj, tiles_n, tile, dist2);
}

// The 256 x 256 kernel for large problems: D a multiple of its k-step, both sides at least one tile, enough tiles to
// fill the chip once; TM_AMD_GEMM_BIG=0|1 forces it off / on (where it applies).
bool big_choice(int N, int M, int D, int batches) {
  static const int forced = [] {
    const char* e = std::getenv("TM_AMD_GEMM_BIG");
    return e ? (e[0] == '0' ? 0 : 1) : -1;
  }();
  if (D % kGK != 0 || N < kGM || M < kGN || forced == 0) return false;
  if (forced == 1) return true;
  const long long tiles = static_cast<long long>((N + kGM - 1) / kGM) * ((M + kGN - 1) / kGN) * batches;
  return tiles >= 128 && static_cast<long long>(N) * M * D * batches >= (1LL << 30);
}

// LDS stages: double buffering (74 KB, 2 blocks/CU) pays for long K loops; for short ones the single buffer's higher
// occupancy (37 KB, 3 blocks/CU: the next tile's loads overlap this tile's epilogue) wins (benchmarks/bench_gemm.py).
// TM_AMD_GEMM_STAGES=1|2 overrides.
int stages_choice(int D) {
  static int forced = [] {
    const char* e = std::getenv("TM_AMD_GEMM_STAGES");
    return e ? (e[0] == '1' ? 1 : 2) : 0;
  }();
  return forced ? forced : (D >= 1024 ? 2 : 1);
}

// K chunk per LDS stage: TM_AMD_GEMM_BK=32|64 overrides
int bk_choice(int D) {
  static int forced = [] {
    const char* e = std::getenv("TM_AMD_GEMM_BK");
    return e ? (e[0] == '6' ? 64 : 32) : 0;
  }();
  return forced ? forced : 32;
}

template <int EPI, int STAGES, int BK>
void launch_one(const at::Tensor& x, const at::Tensor& y, dim3 grid, int N, int M, int D, long long bx, long long by,
                int tiles_m, const EpiParams& ep) {
  const size_t lds = static_cast<size_t>(STAGES) * (kBM + kBN) * (BK + 4) * sizeof(float);
  hipLaunchKernelGGL((gemm_nt_kernel<EPI, STAGES, BK>), grid, dim3(kNT), lds, stream(), x.data_ptr<float>(),
                     y.data_ptr<float>(), N, M, D, bx, by, tiles_m, ep);
}

template <int EPI>
void launch(const at::Tensor& x, const at::Tensor& y, int batches, long long bx, long long by, int N, int M, int D,
            const EpiParams& ep) {
  if (big_choice(N, M, D, batches)) {
    const int tiles_n = (N + kGM - 1) / kGM, tiles_m = (M + kGN - 1) / kGN;
    const int per = (tiles_n * tiles_m + 7) / 8;
    const size_t lds = 2ull * (kGM + kGN) * kGK * sizeof(float);
    static const bool pipe = [] {  // TM_AMD_GEMM_PIPE=0: the barrier at the chunk boundary (A/B knob)
      const char* e = std::getenv("TM_AMD_GEMM_PIPE");
      return !(e && e[0] == '0');
    }();
    hipLaunchKernelGGL((gemm_nt_big_kernel<EPI>), dim3(per * 8, 1, batches), dim3(kGT), lds, stream(),
                       x.data_ptr<float>(), y.data_ptr<float>(), N, M, D, bx, by, tiles_m, ep, pipe);
    return;
  }
  const int tiles_n = (N + kBM - 1) / kBM, tiles_m = (M + kBN - 1) / kBN;
  const int total = tiles_n * tiles_m;
  const int per = (total + 7) / 8;
  const dim3 grid(per * 8, 1, batches);
  const int st = stages_choice(D), bk = bk_choice(D);
  if (bk == 64) {
    if (st == 1) launch_one<EPI, 1, 64>(x, y, grid, N, M, D, bx, by, tiles_m, ep);
    else launch_one<EPI, 2, 64>(x, y, grid, N, M, D, bx, by, tiles_m, ep);
  } else {
    if (st == 1) launch_one<EPI, 1, 32>(x, y, grid, N, M, D, bx, by, tiles_m, ep);
    else launch_one<EPI, 2, 32>(x, y, grid, N, M, D, bx, by, tiles_m, ep);
  }
}


// 16-bit operands: the 256 x 256 tile where it fills the chip (the fp32 kernel's rule), else 128 x 128
template <int EPI, typename T>
void launch_h16(const at::Tensor& x, const at::Tensor& y, int batches, long long bx, long long by, int N, int M, int D,
                const EpiParams& ep, bool big) {
  // DMA granularity from the rows' alignment (D and the base addresses): 16-byte rows take the fast form
  const uintptr_t align = reinterpret_cast<uintptr_t>(x.data_ptr()) | reinterpret_cast<uintptr_t>(y.data_ptr());
  const int gran = (D % 8 == 0 && align % 16 == 0) ? 16 : ((D % 2 == 0 && align % 4 == 0) ? 4 : 2);
  if (gran != 16) {  // (odd widths: the 128 x 128 tile)
    const int tiles_n = (N + 127) / 128, tiles_m = (M + 127) / 128;
    const int per = (tiles_n * tiles_m + 7) / 8;
    const size_t lds = 2ull * 2 * 128 * 64 * sizeof(uint16_t);
    const auto* xp = reinterpret_cast<const uint16_t*>(x.data_ptr());
    const auto* yp = reinterpret_cast<const uint16_t*>(y.data_ptr());
    if (gran == 4)
      hipLaunchKernelGGL((gemm_nt_h16_kernel<EPI, T, 128, 4>), dim3(per * 8, 1, batches), dim3(256), lds, stream(),
                         xp, yp, N, M, D, bx, by, tiles_m, ep);
    else
      hipLaunchKernelGGL((gemm_nt_h16_kernel<EPI, T, 128, 2>), dim3(per * 8, 1, batches), dim3(256), lds, stream(),
                         xp, yp, N, M, D, bx, by, tiles_m, ep);
    return;
  }
  const int tm = big ? 256 : 128;
  const int tiles_n = (N + tm - 1) / tm, tiles_m = (M + tm - 1) / tm;
  const int per = (tiles_n * tiles_m + 7) / 8;
  const size_t lds = 2ull * 2 * tm * 64 * sizeof(uint16_t);
  const auto* xp = reinterpret_cast<const uint16_t*>(x.data_ptr());
  const auto* yp = reinterpret_cast<const uint16_t*>(y.data_ptr());
  if (big)
    hipLaunchKernelGGL((gemm_nt_h16_kernel<EPI, T, 256>), dim3(per * 8, 1, batches), dim3(512), lds, stream(), xp, yp,
                       N, M, D, bx, by, tiles_m, ep);
  else
    hipLaunchKernelGGL((gemm_nt_h16_kernel<EPI, T, 128>), dim3(per * 8, 1, batches), dim3(256), lds, stream(), xp, yp,
                       N, M, D, bx, by, tiles_m, ep);
}

template <int EPI>
void launch_any(const at::Tensor& x, const at::Tensor& y, int batches, long long bx, long long by, int N, int M, int D,
                const EpiParams& ep, bool big16) {
  if (x.scalar_type() == at::kBFloat16) launch_h16<EPI, __bf16>(x, y, batches, bx, by, N, M, D, ep, big16);
  else if (x.scalar_type() == at::kHalf) launch_h16<EPI, _Float16>(x, y, batches, bx, by, N, M, D, ep, big16);
  else launch<EPI>(x, y, batches, bx, by, N, M, D, ep);
}

}  // namespace

// x: [B, N, D] or [N, D]; y: [B, M, D] or [M, D] (fp32, contiguous).  kind: 0 store, 1 euclid, 2 cosine,
// 3 poly-sum, 4 row-min(1 - cos), 5 row-sum, 6 row-and-column max of the scaled dot.  aux_x / aux_y: per-row squared norms (euclid) or inverse norms.
// Returns the output tensor ([B] dims only for batched operands): [B, N, M] fp32 (0-2), fp64 partials [B, blocks]
// (3), fp32 partials [B, N, tiles_m] (4-5), flat fp32 [B*N*tiles_m row partials | B*tiles_n*M column partials] (6).
at::Tensor gemm_nt(const at::Tensor& x, const at::Tensor& y, int64_t kind, const c10::optional<at::Tensor>& aux_x,
                   const c10::optional<at::Tensor>& aux_y, double scale, double coef, int64_t degree, bool zero_diag,
                   bool sqrt_out, const c10::optional<at::Tensor>& idx_x, const c10::optional<at::Tensor>& idx_y,
                   int64_t out_kind) {
  TM_CHECK_CUDA(x);
  TM_SAME_DEVICE(x, y);
  const auto dt = x.scalar_type();
  const bool h16 = dt == at::kBFloat16 || dt == at::kHalf;
  TORCH_CHECK((dt == at::kFloat || h16) && y.scalar_type() == dt, "gemm_nt: fp32 / bf16 / fp16 operands of one dtype");
  TORCH_CHECK(out_kind == 0 || (out_kind == 1 && h16), "gemm_nt: out_kind 1 (16-bit output) needs 16-bit operands");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous(), "gemm_nt: contiguous operands");
  TORCH_CHECK(x.dim() == y.dim() && (x.dim() == 2 || x.dim() == 3), "gemm_nt: [N, D] / [B, N, D] operands");
  const bool gathered = idx_x.has_value();
  TORCH_CHECK(gathered == idx_y.has_value(), "gemm_nt: give both index sets or neither");
  const bool batched = x.dim() == 3 || gathered;
  TORCH_CHECK(!(gathered && x.dim() == 3), "gemm_nt: gathered rows come from 2-D operands");
  const int B = gathered ? static_cast<int>(idx_x->size(0)) : (batched ? static_cast<int>(x.size(0)) : 1);
  TORCH_CHECK(gathered || !batched || y.size(0) == B, "gemm_nt: batch mismatch");
  int N = static_cast<int>(x.size(-2)), M = static_cast<int>(y.size(-2));
  const int D = static_cast<int>(x.size(-1));
  EpiParams ep{};
  if (gathered) {
    for (const auto* t : {&(*idx_x), &(*idx_y)}) {
      TM_SAME_DEVICE(x, (*t));
      TORCH_CHECK(t->scalar_type() == at::kInt && t->is_contiguous() && t->dim() == 2 && t->size(0) == B,
                  "gemm_nt: index sets must be contiguous int32 [B, rows]");
    }
    // host-side bound check of the draws is the caller's contract (indices < rows of x / y); N, M = subset sizes
    N = static_cast<int>(idx_x->size(1));
    M = static_cast<int>(idx_y->size(1));
    ep.ix = idx_x->data_ptr<int32_t>();
    ep.iy = idx_y->data_ptr<int32_t>();
  }
  TORCH_CHECK(y.size(-1) == D, "gemm_nt: inner dimension mismatch");
  // fp32 operands: 16-byte rows (the fp32 kernels' vector staging); 16-bit operands: any width / 2-byte alignment
  // (launch_h16 picks the DMA granularity)
  TORCH_CHECK(h16 || (reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0 && D % 4 == 0),
              "gemm_nt: fp32 operands need 16-byte aligned rows (D % 4 == 0)");
  TORCH_CHECK(D > 0 && N > 0 && M > 0, "gemm_nt: empty operands");
  TORCH_CHECK(static_cast<long long>(N) * M * B < (1LL << 40), "gemm_nt: output too large");
  // 16-bit operands: the 256 x 256 tile once it alone fills the chip (256 tiles), else 128 x 128
  static const int big16_env = [] {  // TM_AMD_GEMM16_BIG=0|1 forces the 128 / 256 tile (measurement)
    const char* e = std::getenv("TM_AMD_GEMM16_BIG");
    return e ? std::atoi(e) : -1;
  }();
  // (rows that are not 16-byte aligned run the 128 x 128 tile with narrower DMA lanes: launch_h16)
  const bool rows16 = D % 8 == 0 && ((reinterpret_cast<uintptr_t>(x.data_ptr()) |
                                      reinterpret_cast<uintptr_t>(y.data_ptr())) % 16) == 0;
  const bool big16 = rows16 && (big16_env >= 0 ? big16_env == 1
                                               : static_cast<long long>((N + 255) / 256) * ((M + 255) / 256) * B >= 256);
  const bool big = h16 ? big16 : big_choice(N, M, D, B);
  const int tbm = big ? kGM : kBM, tbn = big ? kGN : kBN;
  const int tiles_n = (N + tbm - 1) / tbm, tiles_m = (M + tbn - 1) / tbn;
  const int blocks = ((tiles_n * tiles_m + 7) / 8) * 8;
  auto f32 = x.options().dtype(at::kFloat);
  ep.scale = static_cast<float>(scale);
  ep.coef = static_cast<float>(coef);
  ep.degree = static_cast<int>(degree);
  ep.zero_diag = zero_diag;
  ep.sqrt_out = sqrt_out;
  if (aux_x.has_value()) {
    TM_SAME_DEVICE(x, (*aux_x));
    TORCH_CHECK(aux_x->scalar_type() == at::kFloat && aux_x->numel() == static_cast<int64_t>(B) * N, "gemm_nt: aux_x");
    ep.nx = aux_x->data_ptr<float>();
  }
  if (aux_y.has_value()) {
    TM_SAME_DEVICE(x, (*aux_y));
    TORCH_CHECK(aux_y->scalar_type() == at::kFloat && aux_y->numel() == static_cast<int64_t>(B) * M, "gemm_nt: aux_y");
    ep.ny = aux_y->data_ptr<float>();
  }
  if ((kind == kEuclid || kind == kCosine || kind == kRowMin) && (!ep.nx || !ep.ny))
    TORCH_CHECK(false, "gemm_nt: this epilogue needs aux_x and aux_y");
  const long long bx = (batched && !gathered) ? static_cast<long long>(N) * D : 0;
  const long long by = (batched && !gathered) ? static_cast<long long>(M) * D : 0;
  at::Tensor out;
  switch (kind) {
    case kStore:
    case kEuclid:
    case kCosine:
      out = batched ? at::empty({B, N, M}, out_kind ? x.options() : f32) : at::empty({N, M}, out_kind ? x.options() : f32);
      if (out_kind) {
        ep.out16 = reinterpret_cast<uint16_t*>(out.data_ptr());
        ep.out_kind = dt == at::kBFloat16 ? 1 : 2;
      } else {
        ep.out = out.data_ptr<float>();
      }
      ep.ldo = M;
      if (kind == kStore) launch_any<kStore>(x, y, B, bx, by, N, M, D, ep, big);
      else if (kind == kEuclid) launch_any<kEuclid>(x, y, B, bx, by, N, M, D, ep, big);
      else launch_any<kCosine>(x, y, B, bx, by, N, M, D, ep, big);
      break;
    case kPolySum:
      out = batched ? at::zeros({B, blocks}, x.options().dtype(at::kDouble))
                    : at::zeros({blocks}, x.options().dtype(at::kDouble));
      ep.dpart = out.data_ptr<double>();
      launch_any<kPolySum>(x, y, B, bx, by, N, M, D, ep, big);
      break;
    case kRowColMax: {
      // row partials [B, N, tiles_m] then column partials [B, tiles_n, M] in one allocation
      const long long nrow = static_cast<long long>(B) * N * tiles_m, ncol = static_cast<long long>(B) * tiles_n * M;
      out = at::empty({nrow + ncol}, f32);
      ep.out = out.data_ptr<float>();
      ep.out2 = ep.out + nrow;
      ep.part_cols = tiles_m;
      launch_any<kRowColMax>(x, y, B, bx, by, N, M, D, ep, big);
      break;
    }
    case kRowMin:
    case kRowSum:
      out = batched ? at::empty({B, N, tiles_m}, f32) : at::empty({N, tiles_m}, f32);
      ep.out = out.data_ptr<float>();
      ep.part_cols = tiles_m;
      if (kind == kRowMin) launch_any<kRowMin>(x, y, B, bx, by, N, M, D, ep, big);
      else launch_any<kRowSum>(x, y, B, bx, by, N, M, D, ep, big);
      break;
    default:
      TORCH_CHECK(false, "gemm_nt: unknown epilogue ", kind);
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

namespace {
// one wave per row: fp32 sum of squares of a [rows, D] fp32 / bf16 / fp16 operand (16-byte loads when D allows),
// then the squared norm (mode 0) or the inverse norm 1 / sqrt (mode 1) -- the epilogue factors of EUCLID / COSINE
template <typename T>
__global__ void __launch_bounds__(256) row_norms_kernel(const T* __restrict__ x, long long rows, int D, int mode,
                                                        float* __restrict__ out, const T* __restrict__ x2,
                                                        long long rows2, float* __restrict__ out2) {
  const int lane = threadIdx.x & 63;
  long long row = (static_cast<long long>(blockIdx.x) * 256 + threadIdx.x) / 64;
  if (row >= rows) {  // the second operand's rows (one launch for both sides of a GEMM)
    row -= rows;
    if (row >= rows2) return;  // (whole waves)
    x = x2;
    out = out2;
  }
  const T* r = x + row * D;
  float s = 0.f;
  constexpr int kVec = 16 / sizeof(T);
  if (D % kVec == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    for (int c = lane * kVec; c < D; c += 64 * kVec) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(r + c);
      const T* e = reinterpret_cast<const T*>(&w);
#pragma unroll
      for (int k = 0; k < kVec; ++k) {
        const float v = to_f32(e[k]);
        s = fmaf(v, v, s);
      }
    }
  } else {
    for (int c = lane; c < D; c += 64) {
      const float v = to_f32(r[c]);
      s = fmaf(v, v, s);
    }
  }
  s = wave_sum(s);
  if (lane == 0) out[row] = mode ? 1.f / sqrtf(s) : s;
}
}  // namespace

// x (and optionally y): [..., D] contiguous fp32 / bf16 / fp16 of one dtype and D -> fp32 [rows] each: squared row
// norms (mode 0) or inverse norms (mode 1), both operands in one launch
std::vector<at::Tensor> row_norms(const at::Tensor& x, const c10::optional<at::Tensor>& y, int64_t mode) {
  TM_CHECK_CUDA(x);
  TM_CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() >= 1 && (mode == 0 || mode == 1), "row_norms: [..., D] operand, mode 0 / 1");
  const int D = static_cast<int>(x.size(-1));
  const long long rows = D > 0 ? x.numel() / D : 0;
  at::Tensor out = at::empty({rows}, x.options().dtype(at::kFloat));
  long long rows2 = 0;
  at::Tensor out2;
  if (y.has_value()) {
    TM_SAME_DEVICE(x, (*y));
    TM_CHECK_CONTIG((*y));
    TORCH_CHECK(y->scalar_type() == x.scalar_type() && y->size(-1) == D, "row_norms: operands of one dtype and D");
    rows2 = D > 0 ? y->numel() / D : 0;
    out2 = at::empty({rows2}, x.options().dtype(at::kFloat));
  }
  std::vector<at::Tensor> res{out};
  if (y.has_value()) res.push_back(out2);
  if (rows + rows2 == 0) return res;
  const dim3 grid(static_cast<unsigned>((rows + rows2 + 3) / 4));
  auto go = [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((row_norms_kernel<T>), grid, dim3(256), 0, stream(), reinterpret_cast<const T*>(x.data_ptr()),
                       rows, D, static_cast<int>(mode), out.data_ptr<float>(),
                       y.has_value() ? reinterpret_cast<const T*>(y->data_ptr()) : nullptr, rows2,
                       y.has_value() ? out2.data_ptr<float>() : nullptr);
  };
  switch (x.scalar_type()) {
    case at::kFloat: go(float{}); break;
    case at::kBFloat16: go(c10::BFloat16{}); break;
    case at::kHalf: go(c10::Half{}); break;
    default: TORCH_CHECK(false, "row_norms: fp32 / bf16 / fp16 operand");
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return res;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("row_norms(Tensor x, Tensor? y, int mode) -> Tensor[]");
  m.def(
      "gemm_nt(Tensor x, Tensor y, int kind, Tensor? aux_x, Tensor? aux_y, float scale, float coef, int degree, "
      "bool zero_diag, bool sqrt_out, Tensor? idx_x=None, Tensor? idx_y=None, int out_kind=0) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("gemm_nt", &tm_amd::gemm_nt);
  m.impl("row_norms", &tm_amd::row_norms);
}
