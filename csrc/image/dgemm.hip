// fp64 matrix-core GEMM and power-iteration GEMV for FID's compute() (tr sqrt(Σ1 Σ2) by Newton-Schulz).
//
// Reference site: S/image/fid.py:159-179 (`_compute_fid`: `eigvals(sigma1 @ sigma2)` on a non-symmetric D x D fp64
// matrix).  Our compute runs the coupled Newton-Schulz iteration (torchmetrics_amd/image/generative.py) -- three
// D x D fp64 GEMMs per step -- entirely on these kernels, so no vendor GEMM (Tensile / rocBLAS) runs in compute().
//
// dgemm_nn_kernel: C_p = alpha_p * A_p B_p + beta_p * Cin_p + diag_p * I for up to kMaxBatch problems of one shape in
// ONE launch (the Newton-Schulz update Y' = a Y W + b Y and Z' = a W Z + b Z are two GEMMs sharing W: batching them
// gives 2 tiles per CU instead of 1 at D = 2048).  Row-major operands, M x K times K x N.
//   * C tile per block 128 x 128 (8 waves as 2 x 4, 64 x 32 each) once the grid covers every CU, else 64 x 64 (4 waves
//     of 32 x 32, four blocks per CU: D = 1024 runs at 30 instead of 14 TFLOP/s); see the note at the kernel.
//   * K chunk of 16, two LDS stages; chunk c+1 staged while chunk c is consumed, chunk c+2 in flight in registers;
//     within a chunk the operands of k-step s+1 are read from LDS while the MFMAs of step s issue.
//     A is stored m-major (row stride 17 doubles: the 16 rows a wave reads at one k land on distinct banks), B k-major
//     (row stride kTN + 16 doubles: consecutive k rows start 32 banks apart).
//   * XCD-aware tile order: block b runs on XCD b % 8 (observed dispatch), so the tile id is remapped to give each XCD
//     a contiguous range of tile ids, and tile ids walk groups of 4 tile rows column by column: the 32 tiles one XCD
//     holds at D = 2048 are a 4 x 8 patch (A panels read by 8 tiles, B panels by 4, out of that XCD's L2).
//   * Epilogue in registers (f64 C/D layout: col = lane & 15, row = (lane >> 4) + 4 r), coalesced 128-byte rows.
// Numerics: fp64 products and fp64 accumulation in a fixed order (bitwise reproducible run to run).
//
// dgemv4_resid_kernel: one power-iteration step on 4 vectors, W = V - A V with V = Wprev / ||Wprev|| (column norms from
// the previous step's fixed-order per-block partials, so every block normalises identically), and this step's
// per-block partial squared norms.  One wave per row, four 16-byte loads of A in flight per lane, V read from L1/L2.
#include <cstdlib>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kT = 128;        // C tile edge
constexpr int kKC = 16;        // K chunk
constexpr int kAStride = kKC + 1;
constexpr int kMaxBatch = 2;
constexpr int kGroupRows = 4;  // tile-row group of the L2-friendly order

struct GemmProblem {
  const double* a;
  const double* b;
  const double* cin;  // may be null (beta ignored)
  double* c;
  double alpha, beta, diag;
  // euclidean epilogue (out32 != null): out32[i, j] = f32(rowv[i] + colv[j] + alpha * acc), clamped at 0, sqrt'ed
  // when sqrt_out, 0 on the diagonal when zero_diag -- the reference's fp64 formula (F/pairwise/euclidean.py:35-44)
  const double* rowv;
  const double* colv;
  float* out32;
  bool sqrt_out, zero_diag;
};

struct GemmBatch {
  GemmProblem p[kMaxBatch];
};

__device__ __forceinline__ void tile_of(int t, int nti, int ntj, int& ti, int& tj) {
  const int per_group = kGroupRows * ntj;
  const int g = t / per_group;
  const int r = t - g * per_group;
  const int rows_in_group = min(kGroupRows, nti - g * kGroupRows);
  tj = r / rows_in_group;
  ti = g * kGroupRows + r % rows_in_group;
}

// C tile kTM x kTN per block, kWR x kWC waves, each wave (kTM / kWR) x (kTN / kWC) as 16 x 16 f64 MFMA tiles:
//   * 128 x 128, 2 x 4 waves of 64 x 32 (8 accumulators; two waves per SIMD at one block per CU);
//   * 64 x 64, 2 x 2 waves of 32 x 32 (4 accumulators, 38 KB of LDS): four blocks per CU, for grids smaller than the
//     CU count.
//   Measured at D = 2048 (profiles/r06_dgemm_pmc_*.txt, SQ_VALU_MFMA_BUSY_CYCLES over SIMD cycles): 128 x 128 / 8 waves
//   keeps the f64 pipe 75-79 % busy, 64 x 64 / 4 blocks per CU 73 %, Tensile's MT64x64x16 90 % at a higher clock; at
//   D = 4096 ours is within 3-6 % of Tensile (profiles/r06_bench_dgemm.jsonl).
// kBT: B given as [N, K] row-major (C = A B^T), staged like A and transposed into the k-major LDS slab.
template <int kTM, int kTN, int kWR, int kWC, int kOcc, bool kBT, bool kPipeLds = true>
__global__ void __launch_bounds__(kWave * kWR * kWC, kOcc)
    dgemm_nn_kernel(GemmBatch batch, int nprob, int M, int N, int K, bool vec_ok) {
  constexpr int kThr = kWave * kWR * kWC;
  constexpr int kWaveRows = kTM / kWR;
  constexpr int kMW = kWaveRows / 16;         // 16-row MFMA tiles per wave
  constexpr int kWaveCols = kTN / kWC;
  constexpr int kQ = kWaveCols / 16;          // 16-col MFMA tiles per wave (4 or 2)
  constexpr int kPerA = kTM * kKC / kThr;     // A doubles staged per thread
  constexpr int kPerB = kKC * kTN / kThr;     // B doubles staged per thread
  constexpr int kBStr = kTN + 16;             // consecutive k rows of the B slab start 32 banks apart
  static_assert(kMW >= 1 && kQ >= 1 && kPerA % 2 == 0 && kPerB % 2 == 0 && kTM * kKC == kThr * kPerA &&
                    kKC * kTN == kThr * kPerB, "dgemm tile shape");
  __shared__ __attribute__((aligned(16))) double As[2][kTM * kAStride];
  __shared__ __attribute__((aligned(16))) double Bs[2][kKC * kBStr];
  const int nti = (M + kTM - 1) / kTM, ntj = (N + kTN - 1) / kTN;
  const int per = nti * ntj;
  const int total = per * nprob;
  // XCD-aware remap: contiguous tile ids per XCD (when the grid divides evenly over 8 XCDs)
  int t = blockIdx.x;
  if (total % 8 == 0) t = (blockIdx.x % 8) * (total / 8) + blockIdx.x / 8;
  const int pi = t / per;
  int ti, tj;
  tile_of(t - pi * per, nti, ntj, ti, tj);
  const GemmProblem& pr = batch.p[pi];
  const double* __restrict__ A = pr.a;
  const double* __restrict__ B = pr.b;
  const int i0 = ti * kTM, j0 = tj * kTN;

  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid & (kWave - 1);
  const int wr = wave / kWC, wc = wave % kWC;
  // staging: A chunk kTM rows x 16 k (thread: one row, kPerA consecutive k); B chunk 16 k x kTN cols (thread: one k
  // row, kPerB consecutive cols)
  constexpr int kAThrPerRow = kKC / kPerA;
  constexpr int kBThrPerRow = kTN / kPerB;
  const int ar = tid / kAThrPerRow, ak = (tid % kAThrPerRow) * kPerA;
  const int bk = tid / kBThrPerRow, bc = (tid % kBThrPerRow) * kPerB;
  constexpr int kBTThrPerRow = kKC / kPerB;  // kBT: thread -> one B row (output column), kPerB consecutive k
  const int btn = tid / kBTThrPerRow, btk = (tid % kBTThrPerRow) * kPerB;
  double ra[kPerA], rb[kPerB];
  auto load = [&](int k0) {
    const int row = i0 + ar;
    if (vec_ok && row < M && k0 + ak + kPerA <= K) {
      const double* p = A + static_cast<long long>(row) * K + k0 + ak;
#pragma unroll
      for (int v = 0; v < kPerA / 2; ++v) {
        const double2 x = *reinterpret_cast<const double2*>(p + 2 * v);
        ra[2 * v] = x.x;
        ra[2 * v + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int e = 0; e < kPerA; ++e) {
        const int k = k0 + ak + e;
        ra[e] = (row < M && k < K) ? A[static_cast<long long>(row) * K + k] : 0.0;
      }
    }
    if constexpr (kBT) {
      const int n = j0 + btn;
      if (vec_ok && n < N && k0 + btk + kPerB <= K) {
        const double* p = B + static_cast<long long>(n) * K + k0 + btk;
#pragma unroll
        for (int v = 0; v < kPerB / 2; ++v) {
          const double2 x = *reinterpret_cast<const double2*>(p + 2 * v);
          rb[2 * v] = x.x;
          rb[2 * v + 1] = x.y;
        }
      } else {
#pragma unroll
        for (int e = 0; e < kPerB; ++e) {
          const int k = k0 + btk + e;
          rb[e] = (n < N && k < K) ? B[static_cast<long long>(n) * K + k] : 0.0;
        }
      }
      return;
    }
    const int kr = k0 + bk;
    if (vec_ok && kr < K && j0 + bc + kPerB <= N) {
      const double* p = B + static_cast<long long>(kr) * N + j0 + bc;
#pragma unroll
      for (int v = 0; v < kPerB / 2; ++v) {
        const double2 x = *reinterpret_cast<const double2*>(p + 2 * v);
        rb[2 * v] = x.x;
        rb[2 * v + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int e = 0; e < kPerB; ++e) {
        const int c = j0 + bc + e;
        rb[e] = (kr < K && c < N) ? B[static_cast<long long>(kr) * N + c] : 0.0;
      }
    }
  };
  auto store = [&](int s) {
    double* a = &As[s][ar * kAStride + ak];
#pragma unroll
    for (int e = 0; e < kPerA; ++e) a[e] = ra[e];
    if constexpr (kBT) {
#pragma unroll
      for (int e = 0; e < kPerB; ++e) Bs[s][(btk + e) * kBStr + btn] = rb[e];
    } else {
      double* b = &Bs[s][bk * kBStr + bc];
#pragma unroll
      for (int e = 0; e < kPerB; ++e) b[e] = rb[e];
    }
  };

  f64x4 acc[kMW][kQ];
#pragma unroll
  for (int m = 0; m < kMW; ++m)
#pragma unroll
    for (int q = 0; q < kQ; ++q) acc[m][q] = f64x4{0.0, 0.0, 0.0, 0.0};

  const int chunks = (K + kKC - 1) / kKC;
  load(0);
  store(0);
  if (chunks > 1) load(kKC);
  __syncthreads();
  int s = 0;
  for (int c = 0; c < chunks; ++c) {
    const double* as = As[s];
    const double* bs = Bs[s];
    // operands of k-step ks + 1 are read while the MFMAs of k-step ks issue (two register sets), so a wave never
    // waits on LDS between its own MFMAs; the scheduling barriers keep the compiler from sinking the reads back
    double av[2][kMW], bv[2][kQ];
    auto rd = [&](int buf, int ks) {
      const int k = ks * 4 + (lane >> 4);
#pragma unroll
      for (int m = 0; m < kMW; ++m) av[buf][m] = as[(wr * kWaveRows + m * 16 + (lane & 15)) * kAStride + k];
#pragma unroll
      for (int q = 0; q < kQ; ++q) bv[buf][q] = bs[k * kBStr + wc * kWaveCols + q * 16 + (lane & 15)];
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < kKC / 4; ++ks) {
      if (kPipeLds) {
        if (ks + 1 < kKC / 4) rd((ks + 1) & 1, ks + 1);
        __builtin_amdgcn_sched_barrier(0);
      } else if (ks > 0) {
        rd(ks & 1, ks);
      }
#pragma unroll
      for (int m = 0; m < kMW; ++m)
#pragma unroll
        for (int q = 0; q < kQ; ++q)
          acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks & 1][m], bv[ks & 1][q], acc[m][q], 0, 0, 0);
      if (kPipeLds) __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 1 < chunks) {
      store(s ^ 1);  // the other stage was released by the previous iteration's barrier
      if (c + 2 < chunks) load((c + 2) * kKC);
    }
    __syncthreads();
    s ^= 1;
  }

  double* __restrict__ C = pr.c;
  const double* __restrict__ Cin = pr.cin;
  const double alpha = pr.alpha, beta = pr.beta, dg = pr.diag;
  const bool euclid = pr.out32 != nullptr;
  const int col0 = j0 + wc * kWaveCols + (lane & 15);
  // one 16-row slice of accumulators at a time: its Cin values (or norms) are loaded together, all in flight at once,
  // before any of its stores -- not one dependent load per element
#pragma unroll
  for (int m = 0; m < kMW; ++m) {
    const int row0 = i0 + wr * kWaveRows + m * 16 + (lane >> 4);
    double cv[kQ][4];
    double rv[4], colv[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * r, col = col0 + q * 16;
        cv[q][r] = (!euclid && Cin != nullptr && row < M && col < N) ? Cin[static_cast<long long>(row) * N + col] : 0.0;
      }
    if (euclid) {
#pragma unroll
      for (int r = 0; r < 4; ++r) rv[r] = row0 + 4 * r < M ? pr.rowv[row0 + 4 * r] : 0.0;
#pragma unroll
      for (int q = 0; q < kQ; ++q) colv[q] = col0 + q * 16 < N ? pr.colv[col0 + q * 16] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * r, col = col0 + q * 16;
        if (row < M && col < N) {
          const long long e = static_cast<long long>(row) * N + col;
          double v = alpha * acc[m][q][r];
          if (euclid) {
            float d2 = static_cast<float>(v + rv[r] + colv[q]);
            d2 = d2 > 0.f ? d2 : 0.f;
            if (pr.zero_diag && row == col) d2 = 0.f;
            pr.out32[e] = pr.sqrt_out ? sqrtf(d2) : d2;
            continue;
          }
          if (Cin != nullptr) v += beta * cv[q][r];
          if (row == col) v += dg;
          C[e] = v;
        }
      }
  }
}

// ----------------------------------------------------------------------------------------------- power iteration
constexpr int kGemvThreads = 512;
constexpr int kGemvRowsPerWave = 1;

// w_out[i][c] = v[i][c] - sum_k A[i][k] v[k][c],  v = w_in / ||w_in[:, c]||  (normalize=false: v = w_in)
// part_in: [nb_in][4] per-block partial squared norms of w_in; part_out: [gridDim.x][4] of w_out.
__global__ void __launch_bounds__(kGemvThreads)
    dgemv4_resid_kernel(const double* __restrict__ A, const double* __restrict__ w_in,
                        const double* __restrict__ part_in, int nb_in, bool normalize, int d,
                        double* __restrict__ w_out, double* __restrict__ part_out) {
  // (A (s * v))_j = s_j (A v)_j: the previous step's normalisation is applied after the dot products, so the raw
  // vectors are read straight from global memory (64 KB at d = 2048: L1 / L2 resident, every wave of a block reads the
  // same k at the same time) -- no LDS copy of V before the A stream starts
  __shared__ double scale[4];
  __shared__ double wsum[kGemvThreads / kWave][4];
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid & (kWave - 1);
  if (normalize) {
    // column norms from the previous step's per-block partials: the whole block sums them as a fixed-shape tree
    // (thread t: partials t, t + 512, ...; then wave shuffles and the 8 wave sums in order), so every block gets
    // bit-identical norms -- and no single thread walks all partials in a dependent chain
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    const f64x4* P = reinterpret_cast<const f64x4*>(part_in);
    for (int b = tid; b < nb_in; b += kGemvThreads) {
      const f64x4 v = P[b];
      acc[0] += v[0];
      acc[1] += v[1];
      acc[2] += v[2];
      acc[3] += v[3];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = wave_sum(acc[j]);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) wsum[wave][j] = acc[j];
    }
    __syncthreads();
    if (tid < 4) {
      double tot = 0.0;
      for (int w = 0; w < kGemvThreads / kWave; ++w) tot += wsum[w][tid];
      const double n = sqrt(tot);
      scale[tid] = 1.0 / (n > 1e-300 ? n : 1e-300);
    }
  } else if (tid < 4) {
    scale[tid] = 1.0;
  }
  __syncthreads();
  double sq[4] = {0.0, 0.0, 0.0, 0.0};
  const int row0 = (blockIdx.x * (kGemvThreads / kWave) + wave) * kGemvRowsPerWave;
  const f64x4* V = reinterpret_cast<const f64x4*>(w_in);  // [d][4]
  for (int rr = 0; rr < kGemvRowsPerWave; ++rr) {
    const int row = row0 + rr;
    if (row >= d) break;  // wave-uniform
    const double* ar = A + static_cast<long long>(row) * d;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if ((d & 1) == 0) {
      // 4 independent 16-byte loads of A in flight per lane per iteration
      int k = lane * 2;
      for (; k + 3 * 2 * kWave < d; k += 4 * 2 * kWave) {
        double2 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const double2*>(ar + k + u * 2 * kWave);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f64x4 va = V[k + u * 2 * kWave], vb = V[k + u * 2 * kWave + 1];
          s0 += x[u].x * va[0] + x[u].y * vb[0];
          s1 += x[u].x * va[1] + x[u].y * vb[1];
          s2 += x[u].x * va[2] + x[u].y * vb[2];
          s3 += x[u].x * va[3] + x[u].y * vb[3];
        }
      }
      for (; k < d; k += 2 * kWave) {
        const double2 x = *reinterpret_cast<const double2*>(ar + k);
        const f64x4 va = V[k], vb = V[k + 1];
        s0 += x.x * va[0] + x.y * vb[0];
        s1 += x.x * va[1] + x.y * vb[1];
        s2 += x.x * va[2] + x.y * vb[2];
        s3 += x.x * va[3] + x.y * vb[3];
      }
    } else {
      for (int k = lane; k < d; k += kWave) {
        const double a0 = ar[k];
        const f64x4 va = V[k];
        s0 += a0 * va[0];
        s1 += a0 * va[1];
        s2 += a0 * va[2];
        s3 += a0 * va[3];
      }
    }
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
      s0 += __shfl_xor(s0, off, kWave);
      s1 += __shfl_xor(s1, off, kWave);
      s2 += __shfl_xor(s2, off, kWave);
      s3 += __shfl_xor(s3, off, kWave);
    }
    if (lane < 4) {
      const double s = lane == 0 ? s0 : lane == 1 ? s1 : lane == 2 ? s2 : s3;
      const double w = scale[lane] * (w_in[row * 4 + lane] - s);
      w_out[row * 4 + lane] = w;
      sq[lane] += w * w;
    }
  }
  if (lane < 4) wsum[wave][lane] = sq[lane];
  __syncthreads();
  if (tid < 4) {
    double acc = 0.0;
    for (int w = 0; w < kGemvThreads / kWave; ++w) acc += wsum[w][tid];
    part_out[blockIdx.x * 4 + tid] = acc;
  }
}

}  // namespace

// C_i = alpha_i * A_i @ B_i + beta_i * Cin_i + diag_i * I  (fp64, row-major, all problems [M,K] x [K,N]);
// a cin entry with no elements means "no Cin" (beta ignored); an empty list means none for every problem.
void dgemm_nn(at::TensorList a, at::TensorList b, at::TensorList c, at::TensorList cin, at::ArrayRef<double> alpha,
              at::ArrayRef<double> beta, at::ArrayRef<double> diag) {
  const int np = static_cast<int>(a.size());
  TORCH_CHECK(np >= 1 && np <= kMaxBatch, "dgemm_nn: 1..", kMaxBatch, " problems per launch");
  TORCH_CHECK(static_cast<int>(b.size()) == np && static_cast<int>(c.size()) == np &&
                  static_cast<int>(alpha.size()) == np && static_cast<int>(beta.size()) == np &&
                  static_cast<int>(diag.size()) == np && (cin.empty() || static_cast<int>(cin.size()) == np),
              "dgemm_nn: argument lists must have one entry per problem");
  TM_CHECK_CUDA(a[0]);
  const int M = static_cast<int>(a[0].size(0)), K = static_cast<int>(a[0].size(1));
  const int N = static_cast<int>(b[0].size(1));
  bool vec_ok = (K % 2 == 0) && (N % 2 == 0);
  GemmBatch gb{};
  for (int i = 0; i < np; ++i) {
    for (const at::Tensor* t : {&a[i], &b[i], &c[i]}) {
      TM_SAME_DEVICE(a[0], *t);
      TM_CHECK_CONTIG(*t);
      TORCH_CHECK(t->scalar_type() == at::kDouble && t->dim() == 2, "dgemm_nn: operands must be 2-D fp64");
    }
    TORCH_CHECK(a[i].size(0) == M && a[i].size(1) == K && b[i].size(0) == K && b[i].size(1) == N &&
                    c[i].size(0) == M && c[i].size(1) == N,
                "dgemm_nn: shape mismatch in problem ", i);
    const double* cinp = nullptr;
    if (!cin.empty() && cin[i].defined() && cin[i].numel() > 0) {
      TM_SAME_DEVICE(a[0], cin[i]);
      TM_CHECK_CONTIG(cin[i]);
      TORCH_CHECK(cin[i].scalar_type() == at::kDouble && cin[i].numel() == static_cast<long long>(M) * N,
                  "dgemm_nn: cin must be fp64 [M, N]");
      cinp = cin[i].data_ptr<double>();
    }
    gb.p[i] = GemmProblem{a[i].data_ptr<double>(), b[i].data_ptr<double>(), cinp, c[i].data_ptr<double>(),
                          alpha[i], beta[i], diag[i], nullptr, nullptr, nullptr, false, false};
    vec_ok = vec_ok && reinterpret_cast<uintptr_t>(gb.p[i].a) % 16 == 0 &&
             reinterpret_cast<uintptr_t>(gb.p[i].b) % 16 == 0;
  }
  if (M == 0 || N == 0) return;
  static const int variant = [] {
    // tuning knob: 8 = 128 x 128 tile / 8 waves, 4 = 128 x 128 / 4 waves, 64 = 128 x 64 / 4 waves, 44 = 64 x 64 / 4
    // waves; 0 = by shape
    const char* e = std::getenv("TM_AMD_DGEMM_VARIANT");
    return e ? std::atoi(e) : 0;
  }();
  // by shape: 128 x 128 tiles once they cover every CU (MFMA busy 79 % vs 73 % for 64 x 64 at D = 2048), 64 x 64
  // below that (D = 1024: 29 vs 14 TFLOP/s)
  const int t128 = ((M + kT - 1) / kT) * ((N + kT - 1) / kT) * np;
  const int v = variant != 0 ? variant : (t128 < cu_count(a[0].get_device()) ? 44 : 8);
  auto grid = [&](int tm, int tn) { return dim3(((M + tm - 1) / tm) * ((N + tn - 1) / tn) * np); };
  auto s = stream();
  switch (v) {
    case 44:
      hipLaunchKernelGGL((dgemm_nn_kernel<64, 64, 2, 2, 4, false>), grid(64, 64), dim3(256), 0, s, gb, np, M, N, K, vec_ok);
      break;
    case -44:
      hipLaunchKernelGGL((dgemm_nn_kernel<64, 64, 2, 2, 4, false, false>), grid(64, 64), dim3(256), 0, s, gb, np, M, N, K,
                         vec_ok);
      break;
    case 64:
      hipLaunchKernelGGL((dgemm_nn_kernel<128, 64, 2, 2, 2, false>), grid(128, 64), dim3(256), 0, s, gb, np, M, N, K,
                         vec_ok);
      break;
    case 4:
      hipLaunchKernelGGL((dgemm_nn_kernel<128, 128, 2, 2, 2, false>), grid(128, 128), dim3(256), 0, s, gb, np, M, N, K,
                         vec_ok);
      break;
    case -8:
      hipLaunchKernelGGL((dgemm_nn_kernel<128, 128, 2, 4, 2, false, false>), grid(128, 128), dim3(512), 0, s, gb, np, M, N,
                         K, vec_ok);
      break;
    default:
      hipLaunchKernelGGL((dgemm_nn_kernel<128, 128, 2, 4, 2, false>), grid(128, 128), dim3(512), 0, s, gb, np, M, N, K,
                         vec_ok);
  }
}

// Pairwise euclidean distances with the reference's fp64 formula (F/pairwise/euclidean.py:35-44): x [N, K] and y [M, K]
// fp64, nx [N] / ny [M] their squared row norms (fp64) -> out fp32 [N, M] = sqrt(max(f32(nx_i + ny_j - 2 x_i.y_j), 0)),
// all in one fp64-MFMA launch (y read as rows: no transposed copy).
void euclid_f64(const at::Tensor& x, const at::Tensor& y, const at::Tensor& nx, const at::Tensor& ny, bool zero_diag,
                bool sqrt_out, at::Tensor out) {
  TM_CHECK_CUDA(x);
  for (const at::Tensor* t : {&y, &nx, &ny}) {
    TM_SAME_DEVICE(x, *t);
    TM_CHECK_CONTIG(*t);
    TORCH_CHECK(t->scalar_type() == at::kDouble, "euclid_f64: fp64 operands");
  }
  TM_CHECK_CONTIG(x);
  TM_SAME_DEVICE(x, out);
  TORCH_CHECK(x.scalar_type() == at::kDouble && x.dim() == 2 && y.dim() == 2 && x.size(1) == y.size(1),
              "euclid_f64: x [N, K], y [M, K]");
  const int M = static_cast<int>(x.size(0)), N = static_cast<int>(y.size(0)), K = static_cast<int>(x.size(1));
  TORCH_CHECK(nx.numel() == M && ny.numel() == N, "euclid_f64: norm sizes");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == static_cast<long long>(M) * N,
              "euclid_f64: out must be contiguous fp32 [N, M]");
  if (M == 0 || N == 0) return;
  GemmBatch gb{};
  gb.p[0] = GemmProblem{x.data_ptr<double>(), y.data_ptr<double>(), nullptr, nullptr, -2.0, 0.0, 0.0,
                        nx.data_ptr<double>(), ny.data_ptr<double>(), out.data_ptr<float>(), sqrt_out, zero_diag};
  const bool vec_ok = K % 2 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0;
  const int tiles = ((M + kT - 1) / kT) * ((N + kT - 1) / kT);
  hipLaunchKernelGGL((dgemm_nn_kernel<128, 128, 2, 4, 2, true>), dim3(tiles), dim3(512), 0, stream(), gb, 1, M, N, K, vec_ok);
}

// One power-iteration step (see dgemv4_resid_kernel); returns nothing, writes w_out [d, 4] and part_out [blocks, 4].
int64_t dgemv4_blocks(int64_t d) {
  const int rows_per_block = (kGemvThreads / kWave) * kGemvRowsPerWave;
  return (d + rows_per_block - 1) / rows_per_block;
}

void dgemv4_resid(const at::Tensor& a, const at::Tensor& w_in, const at::Tensor& part_in, bool normalize,
                  at::Tensor w_out, at::Tensor part_out) {
  TM_CHECK_CUDA(a);
  for (const at::Tensor* t : {&w_in, &part_in, const_cast<const at::Tensor*>(&w_out),
                              const_cast<const at::Tensor*>(&part_out)}) {
    TM_SAME_DEVICE(a, *t);
    TM_CHECK_CONTIG(*t);
    TORCH_CHECK(t->scalar_type() == at::kDouble, "dgemv4_resid: fp64 operands");
  }
  TM_CHECK_CONTIG(a);
  const int d = static_cast<int>(a.size(0));
  TORCH_CHECK(a.dim() == 2 && a.size(1) == d && a.scalar_type() == at::kDouble, "dgemv4_resid: A must be fp64 [d, d]");
  TORCH_CHECK(w_in.numel() == 4LL * d && w_out.numel() == 4LL * d, "dgemv4_resid: vectors must be [d, 4]");
  const int nb = static_cast<int>(dgemv4_blocks(d));
  TORCH_CHECK(part_out.numel() == 4LL * nb, "dgemv4_resid: part_out must be [", nb, ", 4]");
  TORCH_CHECK(!normalize || part_in.numel() % 4 == 0, "dgemv4_resid: part_in must be [blocks, 4]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w_in.data_ptr()) % 32 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(part_in.data_ptr()) % 32 == 0,
              "dgemv4_resid: 32-byte aligned vectors / partials, 16-byte aligned matrix");
  hipLaunchKernelGGL(dgemv4_resid_kernel, dim3(nb), dim3(kGemvThreads), 0, stream(), a.data_ptr<double>(),
                     w_in.data_ptr<double>(), part_in.data_ptr<double>(), static_cast<int>(part_in.numel() / 4),
                     normalize, d, w_out.data_ptr<double>(), part_out.data_ptr<double>());
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "dgemm_nn(Tensor[] a, Tensor[] b, Tensor(a!)[] c, Tensor[] cin, float[] alpha, float[] beta, float[] diag) -> ()");
  m.def("dgemv4_blocks(int d) -> int", &dgemv4_blocks);
  m.def("euclid_f64(Tensor x, Tensor y, Tensor nx, Tensor ny, bool zero_diag, bool sqrt_out, Tensor(a!) out) -> ()");
  m.def("dgemv4_resid(Tensor a, Tensor w_in, Tensor part_in, bool normalize, Tensor(a!) w_out, Tensor(b!) part_out) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("dgemm_nn", &dgemm_nn);
  m.impl("dgemv4_resid", &dgemv4_resid);
  m.impl("euclid_f64", &euclid_f64);
}

}  // namespace tm_amd
