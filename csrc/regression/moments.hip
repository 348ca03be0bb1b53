// Streaming regression moments: one pass over (preds, target) computing any subset of 19 per-output sums
// (SSE, SAE, Σp, Σt, Σp², Σt², Σpt, MAPE/SMAPE/WMAPE terms, MSLE, log-cosh, Minkowski, count), accumulated in fp64.
//
// This one kernel backs every streaming regression metric (reference F/regression/{mse,mae,mape,symmetric_mape,
// wmape,log_mse,log_cosh,r2,rse,explained_variance,pearson,concordance,minkowski}.py) and, through
// MetricCollection, a whole group of them in a single launch.  Stage 1 writes per-block partials (no float atomics:
// bitwise-reproducible), stage 2 reduces them in fixed order and adds the results straight into the metric state
// tensors (f32 / f64 / i64) given as a tensor list, so an update is exactly two launches whatever the metric set.
//
// Pearson-style metrics pass per-column shifts (the running means) so the sums are of centred values, which keeps
// the single-pass variance/covariance update stable (Σ(x-s)² instead of Σx² - n·mean²).
#include <map>
#include <mutex>

#include "../common/tm_common.h"

#include <vector>

namespace tm_amd {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxSums = 19;

enum SumId : int {
  kSSE = 0,     // Σ (p - t)^2
  kSAE = 1,     // Σ |p - t|
  kSP = 2,      // Σ p~      (p~ = p - shift_p)
  kST = 3,      // Σ t~
  kSPP = 4,     // Σ p~^2
  kSTT = 5,     // Σ t~^2
  kSPT = 6,     // Σ p~ t~
  kMAPE = 7,    // Σ |p - t| / max(|t|, eps)
  kSMAPE = 8,   // Σ 2|p - t| / max(|p| + |t|, eps)
  kSABST = 9,   // Σ |t|
  kMSLE = 10,   // Σ (log1p(p) - log1p(t))^2
  kLOGCOSH = 11,// Σ log(cosh(p - t))
  kMINK = 12,   // Σ |p - t|^P
  kCOUNT = 13,  // number of observations per column
  // the same five sums UNSHIFTED (p, t themselves): a Pearson fold (centred sums) and plain R^2 / explained-variance
  // destinations (raw sums) on the same inputs then share ONE pass (ops.run_moments_plans)
  kSP0 = 14,
  kST0 = 15,
  kSPP0 = 16,
  kSTT0 = 17,
  kSPT0 = 18,
};
constexpr int kUnshifted = (1 << kSP0) | (1 << kST0) | (1 << kSPP0) | (1 << kSTT0) | (1 << kSPT0);

// Destinations of one update: up to kMaxDests plain "state += sum" targets (a whole MetricCollection's worth of
// streaming regression metrics on the same inputs) plus, optionally, one Pearson fold block.
constexpr int kMaxDests = 32;
struct DestSpec {
  void* ptr[kMaxDests];
  int sum_id[kMaxDests];   // dest += sum[sum_id]
  int sub_id[kMaxDests];   // ... - sum[sub_id] when >= 0 (e.g. Σ(t - p) = Σt - Σp for explained variance)
  int dtype[kMaxDests];    // 0 = f32, 1 = f64, 2 = i64
  int per_col[kMaxDests];  // 1: dest has k elements, 0: dest is a scalar (sum over columns)
  int n;
  int fold;                // kFoldPearson: fptr = running (mean_x, mean_y, m2_x, m2_y, c_xy, n) folded in place
  void* fptr[6];
  int fdtype[6];
};

// Pearson / concordance running-moment fold (Chan et al. merge of a centred batch into the running state, the
// update of reference F/regression/pearson.py:25-78 without its host-side branching):
//   tot = n0 + n;  dx = Σx~ / tot;  mean_x += dx;  m2_x += Σx~² - dx Σx~;  c_xy += Σx~y~ - dx Σy~;  n0 = tot
// where x~ = x - mean_x(old) are the shifted sums of the partial kernel.  Each state is updated in its own dtype
// with the increment rounded to that dtype first, exactly like the host formulation.
constexpr int kFoldNone = 0;
constexpr int kFoldPearson = 1;
constexpr int kColParMin = 256;  // above this many outputs: moments_colpar_kernel

__device__ __forceinline__ double ld_state(const DestSpec& spec, int j, int c) {
  return spec.fdtype[j] == 0 ? static_cast<double>(reinterpret_cast<const float*>(spec.fptr[j])[c])
                             : reinterpret_cast<const double*>(spec.fptr[j])[c];
}

// The fold of one column: all six states are loaded before the first store (load-after-possibly-aliasing-store
// kept the compiler from hoisting them: six dependent HBM round trips, ~1 us each, at the tail of every launch).
__device__ __forceinline__ void pearson_fold(const DestSpec& spec, int c, double sd, double se, double sdd, double see,
                                             double sde, double n) {
  double old[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) old[j] = ld_state(spec, j, c);
  const double tot = old[5] + n;
  const double dx = sd / tot, dy = se / tot;
  const double inc[6] = {dx, dy, sdd - dx * sd, see - dy * se, sde - dx * se, n};
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    if (spec.fdtype[j] == 0)
      reinterpret_cast<float*>(spec.fptr[j])[c] = static_cast<float>(old[j]) + static_cast<float>(inc[j]);
    else
      reinterpret_cast<double*>(spec.fptr[j])[c] = old[j] + inc[j];
  }
}

__device__ void finalize_column(const double* __restrict__ partial, int nblocks, int k, int c,
                                const DestSpec& spec, double* __restrict__ out_sums, int mask);

template <typename scalar_t>
__device__ __forceinline__ void accumulate_pair(double* acc, scalar_t pv, scalar_t tv, float sp, float st, int mask,
                                                double eps, double pw) {
  const float p = to_f32(pv);
  const float t = to_f32(tv);
  const float d = p - t;
  const float ad = fabsf(d);
  if (mask & (1 << kSSE)) acc[kSSE] += static_cast<double>(d) * d;
  if (mask & (1 << kSAE)) acc[kSAE] += ad;
  if (mask & ((1 << kSP) | (1 << kSPP) | (1 << kSPT) | (1 << kST) | (1 << kSTT))) {
    const double pc = static_cast<double>(p) - sp, tc = static_cast<double>(t) - st;
    acc[kSP] += pc;
    acc[kST] += tc;
    acc[kSPP] += pc * pc;
    acc[kSTT] += tc * tc;
    acc[kSPT] += pc * tc;
  }
  if (mask & kUnshifted) {
    const double pd = p, td = t;
    acc[kSP0] += pd;
    acc[kST0] += td;
    acc[kSPP0] += pd * pd;
    acc[kSTT0] += td * td;
    acc[kSPT0] += pd * td;
  }
  if (mask & (1 << kMAPE)) acc[kMAPE] += ad / fmax(static_cast<double>(fabsf(t)), eps);
  if (mask & (1 << kSMAPE)) acc[kSMAPE] += 2.0 * ad / fmax(static_cast<double>(fabsf(p) + fabsf(t)), eps);
  if (mask & (1 << kSABST)) acc[kSABST] += fabsf(t);
  if (mask & (1 << kMSLE)) {
    const double l = log1p(static_cast<double>(p)) - log1p(static_cast<double>(t));
    acc[kMSLE] += l * l;
  }
  if (mask & (1 << kLOGCOSH)) {
    // log(cosh(x)) = |x| + log1p(exp(-2|x|)) - log(2)  (overflow-free)
    const double x = fabs(static_cast<double>(d));
    acc[kLOGCOSH] += x + log1p(exp(-2.0 * x)) - 0.69314718055994530942;
  }
  if (mask & (1 << kMINK)) acc[kMINK] += pow(static_cast<double>(ad), pw);
  acc[kCOUNT] += 1.0;
}

template <typename scalar_t>
__global__ void __launch_bounds__(kBlock) moments_partial_kernel(const scalar_t* __restrict__ preds,
                                                                 const scalar_t* __restrict__ target, long long n_rows,
                                                                 int k, int mask, double eps, double pw,
                                                                 const float* __restrict__ shift_p,
                                                                 const float* __restrict__ shift_t,
                                                                 double* __restrict__ partial, int fuse,
                                                                 DestSpec spec, double* __restrict__ out_sums,
                                                                 unsigned int* __restrict__ ticket) {
  // every thread keeps one column: total threads is a multiple of k (host guarantees blockDim % k == 0 or k > block)
  const long long tid = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long nthreads = static_cast<long long>(gridDim.x) * blockDim.x;
  const long long total = n_rows * k;
  double acc[kMaxSums];
#pragma unroll
  for (int s = 0; s < kMaxSums; ++s) acc[s] = 0.0;
  const int col = static_cast<int>(tid % k);
  const float sp = shift_p ? shift_p[col] : 0.f;
  const float st = shift_t ? shift_t[col] : 0.f;
  // stride is a multiple of k -> the column of this thread never changes
  for (long long i = tid; i < total; i += nthreads) {
    accumulate_pair(acc, preds[i], target[i], sp, st, mask, eps, pw);
  }
  if ((kWave % k) == 0) {
    // k divides the wave: lanes l and l ^ off (off >= k) share a column -> xor-shuffle tree inside the wave, then a
    // 4-wave fold in LDS (the generic path below walks the block serially per column: ~25 us for k = 1)
    __shared__ double wred[kBlock / kWave][kWave][kMaxSums];
    const int wid = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    wave_colsum_f64(acc, k);
#pragma unroll
    for (int s = 0; s < kMaxSums; ++s)
      if ((((mask >> s) & 1) || s == kCOUNT) && lane < k) wred[wid][lane][s] = acc[s];
    __syncthreads();
    for (int i = threadIdx.x; i < k * kMaxSums; i += blockDim.x) {
      const int c = i / kMaxSums, s = i % kMaxSums;
      double v = 0.0;
      if (((mask >> s) & 1) || s == kCOUNT)
        for (int w = 0; w < kBlock / kWave; ++w) v += wred[w][c][s];
      // lane l of every wave holds column (block_base + l) % k; block_base is a multiple of k here
      partial[(static_cast<long long>(blockIdx.x) * k + c) * kMaxSums + s] = v;
    }
  } else {
  // block reduction per (column, sum): threads with equal tid % k hold the same column
  __shared__ double red[kBlock][kMaxSums + 1];
#pragma unroll
  for (int s = 0; s < kMaxSums; ++s) red[threadIdx.x][s] = acc[s];
  __syncthreads();
  // rows of the partial buffer: [block][column][sum]
  for (int c = threadIdx.x; c < k; c += blockDim.x) {
    double out[kMaxSums];
#pragma unroll
    for (int s = 0; s < kMaxSums; ++s) out[s] = 0.0;
    // threads t with (blockIdx*blockDim + t) % k == c
    const int first = static_cast<int>(((c - (static_cast<long long>(blockIdx.x) * blockDim.x) % k) % k + k) % k);
    for (int t = first; t < static_cast<int>(blockDim.x); t += k) {
#pragma unroll
      for (int s = 0; s < kMaxSums; ++s) out[s] += red[t][s];
    }
    double* dst = partial + (static_cast<long long>(blockIdx.x) * k + c) * kMaxSums;
#pragma unroll
    for (int s = 0; s < kMaxSums; ++s) dst[s] = out[s];
  }
  }
  if (fuse) {  // single-block launch: this block also folds its sums into the states (one launch per update)
    __threadfence_block();
    __syncthreads();
    for (int c = 0; c < k; ++c) finalize_column(partial, 1, k, c, spec, out_sums, mask);
  } else if (ticket != nullptr) {
    // a few blocks (mid-size batches): the LAST block to finish folds every block's partials -- one launch instead
    // of this pass + moments_finalize_kernel; it re-arms the ticket for the next launch on this stream
    __shared__ bool last;
    __threadfence();  // this block's partials are visible device-wide before its ticket
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last) {
      __threadfence();
      for (int c = 0; c < k; ++c) finalize_column(partial, static_cast<int>(gridDim.x), k, c, spec, out_sums, mask);
      if (threadIdx.x == 0) *ticket = 0u;
    }
  }
}

// fixed-order reduction of one column's partials over blocks, then add / fold into the destination states;
// called by every thread of a block
__device__ void finalize_column(const double* __restrict__ partial, int nblocks, int k, int c, const DestSpec& spec,
                                double* __restrict__ out_sums, int mask) {
  __shared__ double red[kMaxSums][kBlock / kWave];
  double acc[kMaxSums];
#pragma unroll
  for (int s = 0; s < kMaxSums; ++s) acc[s] = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) {
    const double* src = partial + (static_cast<long long>(b) * k + c) * kMaxSums;
#pragma unroll
    for (int s = 0; s < kMaxSums; ++s) acc[s] += src[s];
  }
  const int wid = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  wave_colsum_f64(acc, 1);
#pragma unroll
  for (int s = 0; s < kMaxSums; ++s)
    if (lane == 0) red[s][wid] = (((mask >> s) & 1) || s == kCOUNT) ? acc[s] : 0.0;
  __syncthreads();
  if (threadIdx.x < kMaxSums) {
    double v = 0.0;
    for (int w = 0; w < static_cast<int>(blockDim.x / kWave); ++w) v += red[threadIdx.x][w];
    if (out_sums) out_sums[c * kMaxSums + threadIdx.x] = v;
    red[threadIdx.x][0] = v;
  }
  __syncthreads();
  if (spec.fold == kFoldPearson) {
    if (threadIdx.x == kWave) {  // a lane of the second wave: the first wave's lanes own the plain dests below
      const double sd = red[kSP][0], se = red[kST][0], sdd = red[kSPP][0], see = red[kSTT][0], sde = red[kSPT][0];
      const double n = red[kCOUNT][0];
      pearson_fold(spec, c, sd, se, sdd, see, sde, n);
    }
  }
  if (threadIdx.x < spec.n) {
    const int j = threadIdx.x;
    const double v = red[spec.sum_id[j]][0] - (spec.sub_id[j] >= 0 ? red[spec.sub_id[j]][0] : 0.0);
    const int idx = spec.per_col[j] ? c : 0;
    // per-column destination, or a scalar destination fed from column 0 (counts are equal in every column)
    if (spec.per_col[j] || c == 0) {
      if (spec.dtype[j] == 0) reinterpret_cast<float*>(spec.ptr[j])[idx] += static_cast<float>(v);
      else if (spec.dtype[j] == 1) reinterpret_cast<double*>(spec.ptr[j])[idx] += v;
      else reinterpret_cast<int64_t*>(spec.ptr[j])[idx] += static_cast<int64_t>(llrint(v));
    }
  }
  __syncthreads();  // red[] is reused by the next column of a fused single-block launch
}

// one block per column
// Many outputs (k > kColParMin): one thread per column walks a chunk of rows (reads of a row are coalesced across
// the block's consecutive columns); grid.y splits the rows so k * chunks threads fill the GPU.  Partials use the same
// [chunk][column][sum] layout as moments_partial_kernel, so moments_finalize_kernel folds both.
template <typename scalar_t>
__global__ void __launch_bounds__(kBlock) moments_colpar_kernel(const scalar_t* __restrict__ preds,
                                                                const scalar_t* __restrict__ target,
                                                                long long n_rows, int k, long long rows_per_chunk,
                                                                int mask, double eps, double pw,
                                                                const float* __restrict__ shift_p,
                                                                const float* __restrict__ shift_t,
                                                                double* __restrict__ partial) {
  const long long col = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (col >= k) return;
  double acc[kMaxSums];
#pragma unroll
  for (int s = 0; s < kMaxSums; ++s) acc[s] = 0.0;
  const float sp = shift_p ? shift_p[col] : 0.f;
  const float st = shift_t ? shift_t[col] : 0.f;
  const long long r0 = static_cast<long long>(blockIdx.y) * rows_per_chunk;
  const long long r1 = r0 + rows_per_chunk < n_rows ? r0 + rows_per_chunk : n_rows;
  long long r = r0;
  for (; r + 4 <= r1; r += 4) {  // four rows' loads in flight before the dependent accumulation
    scalar_t pv[4], tv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pv[q] = preds[(r + q) * k + col];
      tv[q] = target[(r + q) * k + col];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) accumulate_pair(acc, pv[q], tv[q], sp, st, mask, eps, pw);
  }
  for (; r < r1; ++r) accumulate_pair(acc, preds[r * k + col], target[r * k + col], sp, st, mask, eps, pw);
  double* dst = partial + (static_cast<long long>(blockIdx.y) * k + col) * kMaxSums;
#pragma unroll
  for (int s = 0; s < kMaxSums; ++s) dst[s] = acc[s];
}

__global__ void __launch_bounds__(kBlock) moments_finalize_kernel(const double* __restrict__ partial, int nblocks,
                                                                  int k, DestSpec spec, double* __restrict__ out_sums,
                                                                  int mask) {
  finalize_column(partial, nblocks, k, blockIdx.x, spec, out_sums, mask);
}


// Small batches (n_rows * k <= kSmallMax, k dividing the wave): ONE 512-thread block does the pass and the fold -- one
// launch, no partials buffer, no grid-wide fence or ticket.  Every thread keeps one column (k | 64 | 1024, so the
// stride never changes a thread's column) and issues up to kSmallUnroll pairs' loads before accumulating them; wave
// xor-trees then a 16-wave LDS fold give the per-column sums, and (column, destination) threads apply them.
constexpr int kSmallThreads = 512;  // 1024 capped VGPRs at 128 and spilled the fp64 accumulators to scratch
constexpr int kSmallUnroll = 8;
constexpr long long kSmallMax = 65536;

__device__ __forceinline__ void apply_sums(const double* __restrict__ v, int c, int j, const DestSpec& spec) {
  // j < spec.n: plain destination j of column c; j == spec.n: the Pearson fold of column c
  if (j < spec.n) {
    const double x = v[spec.sum_id[j]] - (spec.sub_id[j] >= 0 ? v[spec.sub_id[j]] : 0.0);
    const int idx = spec.per_col[j] ? c : 0;
    if (spec.per_col[j] || c == 0) {
      if (spec.dtype[j] == 0) reinterpret_cast<float*>(spec.ptr[j])[idx] += static_cast<float>(x);
      else if (spec.dtype[j] == 1) reinterpret_cast<double*>(spec.ptr[j])[idx] += x;
      else reinterpret_cast<int64_t*>(spec.ptr[j])[idx] += static_cast<int64_t>(llrint(x));
    }
  } else if (spec.fold == kFoldPearson) {
    const double sd = v[kSP], se = v[kST], sdd = v[kSPP], see = v[kSTT], sde = v[kSPT], n = v[kCOUNT];
    pearson_fold(spec, c, sd, se, sdd, see, sde, n);
  }
}

// The same application with every load hoisted to the kernel's start: the (column, destination) item's spec fields
// and the destination's old value(s) are loaded while the pass's own loads are in flight, so the tail is arithmetic
// and stores.  (Applied after the sums, the field loads -- dynamically indexed kernel arguments -- then the pointer,
// then the old value were three dependent round trips, ~1 us each, at the end of every small launch.)  Valid because
// nothing else writes the destinations while the launch runs (one stream), and only one block applies.
struct ApplyPre {
  unsigned long long raw[6];  // old values, as stored (f32 in the low word / f64 / i64)
  void* ptr;
  int sum_id, sub_id, dtype, idx, live;
};

__device__ __forceinline__ unsigned long long ld_raw(const void* p, int dtype, int idx) {
  if (dtype == 0) return __float_as_uint(reinterpret_cast<const float*>(p)[idx]);
  return reinterpret_cast<const unsigned long long*>(p)[idx];
}

__device__ __forceinline__ ApplyPre apply_prefetch(int c, int j, const DestSpec& spec) {
  ApplyPre a{};
  if (j < spec.n) {
    a.live = spec.per_col[j] || c == 0;
    a.ptr = spec.ptr[j];
    a.sum_id = spec.sum_id[j];
    a.sub_id = spec.sub_id[j];
    a.dtype = spec.dtype[j];
    a.idx = spec.per_col[j] ? c : 0;
    if (a.live) a.raw[0] = ld_raw(a.ptr, a.dtype, a.idx);
  } else if (spec.fold == kFoldPearson) {
    a.live = 1;
#pragma unroll
    for (int q = 0; q < 6; ++q) a.raw[q] = ld_raw(spec.fptr[q], spec.fdtype[q], c);
  }
  return a;
}

__device__ __forceinline__ void apply_sums_pre(const double* __restrict__ v, int c, int j, const DestSpec& spec,
                                               const ApplyPre& a) {
  if (!a.live) return;
  if (j < spec.n) {
    const double x = v[a.sum_id] - (a.sub_id >= 0 ? v[a.sub_id] : 0.0);
    const int idx = a.idx;
    if (a.dtype == 0)
      reinterpret_cast<float*>(a.ptr)[idx] = __uint_as_float(static_cast<unsigned>(a.raw[0])) + static_cast<float>(x);
    else if (a.dtype == 1)
      reinterpret_cast<double*>(a.ptr)[idx] = __longlong_as_double(static_cast<long long>(a.raw[0])) + x;
    else
      reinterpret_cast<int64_t*>(a.ptr)[idx] = static_cast<int64_t>(a.raw[0]) + static_cast<int64_t>(llrint(x));
    return;
  }
  const double sd = v[kSP], se = v[kST], sdd = v[kSPP], see = v[kSTT], sde = v[kSPT], n = v[kCOUNT];
  double old[6];
#pragma unroll
  for (int q = 0; q < 6; ++q)
    old[q] = spec.fdtype[q] == 0 ? static_cast<double>(__uint_as_float(static_cast<unsigned>(a.raw[q])))
                                 : __longlong_as_double(static_cast<long long>(a.raw[q]));
  const double tot = old[5] + n;
  const double dx = sd / tot, dy = se / tot;
  const double inc[6] = {dx, dy, sdd - dx * sd, see - dy * se, sde - dx * se, n};
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    if (spec.fdtype[q] == 0)
      reinterpret_cast<float*>(spec.fptr[q])[c] = static_cast<float>(old[q]) + static_cast<float>(inc[q]);
    else
      reinterpret_cast<double*>(spec.fptr[q])[c] = old[q] + inc[q];
  }
}

template <typename scalar_t>
__global__ void __launch_bounds__(kSmallThreads) moments_small_kernel(
    const scalar_t* __restrict__ preds, const scalar_t* __restrict__ target, long long total, int k, int mask,
    double eps, double pw, const float* __restrict__ shift_p, const float* __restrict__ shift_t, DestSpec spec,
    double* __restrict__ out_sums) {
  extern __shared__ double wsum[];  // [16 waves][k][kMaxSums], then [k][kMaxSums] block totals
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  constexpr int kWaves = kSmallThreads / kWave;
  // measurement-only ablation (TM_AMD_MOMENTS_ABLATE, bits 27..29 of mask): 1 no pass, 2 no apply, 4 no prefetch
  const int abl = (mask >> 27) & 7;
  mask &= (1 << 27) - 1;
  if (abl & 1) total = 0;
  double acc[kMaxSums];
#pragma unroll
  for (int q = 0; q < kMaxSums; ++q) acc[q] = 0.0;
  const int col = tid % k;
  const float sp = shift_p ? shift_p[col] : 0.f;
  const float st = shift_t ? shift_t[col] : 0.f;
  const int items = k * (spec.n + 1);
  const bool pre = items <= kSmallThreads;  // uniform: one (column, destination) item per thread
  ApplyPre ap{};
  if (pre && tid < items && !(abl & 4)) ap = apply_prefetch(tid / (spec.n + 1), tid % (spec.n + 1), spec);
  for (long long base = tid; base < total; base += static_cast<long long>(kSmallThreads) * kSmallUnroll) {
    scalar_t pv[kSmallUnroll], tv[kSmallUnroll];
#pragma unroll
    for (int u = 0; u < kSmallUnroll; ++u) {  // all loads in flight before the dependent fp64 accumulation
      const long long i = base + static_cast<long long>(u) * kSmallThreads;
      pv[u] = i < total ? preds[i] : scalar_t(0);
      tv[u] = i < total ? target[i] : scalar_t(0);
    }
#pragma unroll
    for (int u = 0; u < kSmallUnroll; ++u)
      if (base + static_cast<long long>(u) * kSmallThreads < total) accumulate_pair(acc, pv[u], tv[u], sp, st, mask, eps, pw);
  }
  // VALU (DPP / permlane) column sums of the requested sums: LDS-pipe shuffles were most of this kernel
  wave_colsum_f64_masked(acc, k, (mask & ((1 << kMaxSums) - 1)) | (1 << kCOUNT));
#pragma unroll
  for (int q = 0; q < kMaxSums; ++q)
    if ((((mask >> q) & 1) || q == kCOUNT) && lane < k) wsum[(wid * k + lane) * kMaxSums + q] = acc[q];
  __syncthreads();
  double* tot = wsum + kWaves * k * kMaxSums;
  for (int i = tid; i < k * kMaxSums; i += kSmallThreads) {
    const int c = i / kMaxSums, q = i % kMaxSums;
    double v = 0.0;
    if (((mask >> q) & 1) || q == kCOUNT)
      for (int w = 0; w < kWaves; ++w) v += wsum[(w * k + c) * kMaxSums + q];  // fixed order: reproducible
    tot[i] = v;
    if (out_sums) out_sums[i] = v;
  }
  __syncthreads();
  if (abl & 2) return;
  if (pre) {
    if (tid < items) apply_sums_pre(tot + (tid / (spec.n + 1)) * kMaxSums, tid / (spec.n + 1), tid % (spec.n + 1), spec, ap);
    return;
  }
  for (int i = tid; i < items; i += kSmallThreads) {
    const int c = i / (spec.n + 1), j = i % (spec.n + 1);
    apply_sums(tot + c * kMaxSums, c, j, spec);
  }
}

// Small batches on MANY blocks, still one launch and no fence: every block reduces its slice to per-column sums
// and stores them with agent-scope (sc1) stores; after every storing wave's vmcnt(0) wait and a block barrier, one
// lane adds 1 to the stream's ticket with an agent-scope atomic.  The block whose add returns G - 1 is last: it loads
// all G partial rows with agent-scope (sc1) loads, sums them in block order (reproducible), applies the destinations /
// the Pearson fold, and re-arms the ticket.  (The hand-off of MI355X_MICROARCH.md's table, first row: sc1 payload,
// one counter, the last adder loads after its add returned, its block's other waves after a barrier.)  The single-
// block kernel above left the chip idle but one CU: 13 us for config #5's 8192 pairs.
constexpr int kHandoffThreads = 256;
constexpr int kHandoffRows = 512;     // values per block (G = ceil(n / 512), at most 128 blocks)
constexpr int kHandoffMaxRows = 256;  // G * k: the last block stages every partial row in LDS (<= 39 KB)

template <typename scalar_t>
__global__ void __launch_bounds__(kHandoffThreads) moments_handoff_kernel(
    const scalar_t* __restrict__ preds, const scalar_t* __restrict__ target, long long total, int k, int mask,
    double eps, double pw, const float* __restrict__ shift_p, const float* __restrict__ shift_t, DestSpec spec,
    double* __restrict__ out_sums, double* __restrict__ partial, unsigned int* __restrict__ ticket, bool fenced) {
  // phase 1: [wave][column][sum]; the last block then reuses it for [G][column][sum] staged rows + [column][sum] totals
  extern __shared__ double lds[];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  constexpr int kWaves = kHandoffThreads / kWave;
  const int kk = k * kMaxSums;
  double acc[kMaxSums];
#pragma unroll
  for (int q = 0; q < kMaxSums; ++q) acc[q] = 0.0;
  const int col = tid % k;  // (block size and block offsets are multiples of k: a thread keeps its column)
  const float sp = shift_p ? shift_p[col] : 0.f;
  const float st = shift_t ? shift_t[col] : 0.f;
  const int items = k * (spec.n + 1);
  const bool pre = items <= kHandoffThreads;  // uniform (every block prefetches: it does not know yet who is last)
  ApplyPre ap{};
  if (pre && tid < items) ap = apply_prefetch(tid / (spec.n + 1), tid % (spec.n + 1), spec);
  const long long stride = static_cast<long long>(gridDim.x) * kHandoffThreads;
  for (long long i = static_cast<long long>(blockIdx.x) * kHandoffThreads + tid; i < total; i += stride)
    accumulate_pair(acc, preds[i], target[i], sp, st, mask, eps, pw);
  wave_colsum_f64_masked(acc, k, mask | (1 << kCOUNT));  // the requested sums only (config #5: 8 of 19)
#pragma unroll
  for (int q = 0; q < kMaxSums; ++q)
    if ((((mask >> q) & 1) || q == kCOUNT) && lane < k) lds[(wid * k + lane) * kMaxSums + q] = acc[q];
  __syncthreads();
  double* row = partial + static_cast<long long>(blockIdx.x) * kk;
  for (int i = tid; i < kk; i += kHandoffThreads) {
    const int c = i / kMaxSums, q = i % kMaxSums;
    double v = 0.0;
    if (((mask >> q) & 1) || q == kCOUNT)
      for (int w = 0; w < kWaves; ++w) v += lds[(w * k + c) * kMaxSums + q];
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(row + i),
                       static_cast<unsigned long long>(__double_as_longlong(v)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // Memory-model note.  The hand-off is the "sc1 payload" form of MI355X_MICROARCH.md (Valid forms): EVERY
  // store of the partial rows is an agent-scope (sc1, write-through) atomic store drained by `s_waitcnt vmcnt(0)`
  // before the block's barrier and ticket add, and EVERY load of them in the last block is an agent-scope (sc1)
  // atomic load -- no L1 / non-coherent L2 copy is ever read, so no release / acquire fence (buffer_wbl2 / buffer_inv
  // sc1, ~1.7 us each on gfx950) is needed on this ISA.  It is NOT ordered by the C++/HIP memory model alone (relaxed
  // stores vs a relaxed ticket): `fenced` (TM_AMD_MOMENTS_FENCED=1) adds the model's agent-scope release before the
  // ticket and acquire after it, for measurement and for any other target; tests/test_moments_handoff_gpu.py
  // checks every sum under uneven load on gfx950 with the fence-free default.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores are done
  __syncthreads();
  if (tid == 0) {
    if (fenced) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    } else {
      last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
  }
  __syncthreads();
  if (!last) return;
  if (fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // the last block: all G partial rows with coalesced, independent sc1 loads into LDS (a per-column chain of G
  // dependent loads cost ~0.3 us per block), then per (column, sum) a block-order sum (reproducible)
  const int nload = static_cast<int>(gridDim.x) * kk;
  for (int base = tid; base < nload; base += 4 * kHandoffThreads) {
    unsigned long long v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int f = base + u * kHandoffThreads;
      v[u] = f < nload ? __hip_atomic_load(reinterpret_cast<unsigned long long*>(partial + f), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                       : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int f = base + u * kHandoffThreads;
      if (f < nload) lds[f] = __longlong_as_double(static_cast<long long>(v[u]));
    }
  }
  __syncthreads();
  double* tot = lds + nload;
  for (int i = tid; i < kk; i += kHandoffThreads) {
    const int q = i % kMaxSums;
    double v = 0.0;
    if (((mask >> q) & 1) || q == kCOUNT)
      for (unsigned b = 0; b < gridDim.x; ++b) v += lds[b * kk + i];
    tot[i] = v;
    if (out_sums) out_sums[i] = v;
  }
  __syncthreads();
  if (pre) {
    if (tid < items) apply_sums_pre(tot + (tid / (spec.n + 1)) * kMaxSums, tid / (spec.n + 1), tid % (spec.n + 1), spec, ap);
  } else {
    for (int i = tid; i < items; i += kHandoffThreads) {
      const int c = i / (spec.n + 1), j = i % (spec.n + 1);
      apply_sums(tot + c * kMaxSums, c, j, spec);
    }
  }
  if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
}

}  // namespace

// kStreamTickets zeroed uint32 words per (device, stream), kept for the process (tm_common.h): the last-block folds
// of moments_partial_kernel / moments_handoff_kernel count finished blocks in word 0 and reset it, so consecutive
// launches on a stream reuse it (launches on one stream never overlap).
unsigned int* stream_ticket(int device, hipStream_t s) {
  static std::mutex mu;
  // never destroyed: the tensors must not be freed after the runtime has shut down at process exit
  static auto* tickets = new std::map<std::pair<int, hipStream_t>, at::Tensor>();
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_pair(device, s);
  auto it = tickets->find(key);
  if (it == tickets->end())
    it = tickets->emplace(key, at::zeros({kStreamTickets}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, device)))
             .first;
  return reinterpret_cast<unsigned int*>(it->second.data_ptr<int>());
}

// preds/target: [N, k] (or [N] with k = 1), same floating dtype. dests[j] += sum[sum_ids[j]] (per column, or over
// column 0 when dest has one element and k > 1, e.g. observation counts). Returns the [k, 19] fp64 sums when want_sums.
at::Tensor moments_update(const at::Tensor& preds, const at::Tensor& target, int64_t num_outputs, int64_t mask,
                          double eps, double power, const c10::optional<at::Tensor>& shift_p,
                          const c10::optional<at::Tensor>& shift_t, at::TensorList dests,
                          at::IntArrayRef sum_ids, bool want_sums, int64_t fold) {
  TM_CHECK_CUDA(preds);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.scalar_type() == target.scalar_type(), "moments_update: preds/target dtype mismatch");
  TORCH_CHECK(preds.numel() == target.numel(), "moments_update: preds/target numel mismatch");
  const int nfold = fold != 0 ? 6 : 0;
  TORCH_CHECK(static_cast<int64_t>(dests.size()) == nfold + static_cast<int64_t>(sum_ids.size()) &&
                  sum_ids.size() <= static_cast<size_t>(kMaxDests),
              "moments_update: bad destination list (fold states first, then one sum id per plain destination)");
  const int k = static_cast<int>(num_outputs);
  TORCH_CHECK(k >= 1 && preds.numel() % k == 0, "moments_update: numel not divisible by num_outputs");
  const long long n_rows = preds.numel() / k;
  auto dopt = preds.options().dtype(at::kDouble);
  at::Tensor sums = want_sums ? at::zeros({k, kMaxSums}, dopt) : at::Tensor();
  if (n_rows == 0) return sums;
  // thread count must be a multiple of k so each thread keeps one column
  int block = kBlock;
  long long blocks = (n_rows * k + block - 1) / block;
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
  if (k > 1) {
    // grid * block multiple of k: use block = 256 and blocks multiple of k/gcd(256,k)
    long long g = k;
    long long a = block;
    while (a) { long long r = g % a; g = a; a = r; }
    const long long step = k / g;
    blocks = ((blocks + step - 1) / step) * step;
  }
  DestSpec spec{};
  spec.n = static_cast<int>(sum_ids.size());
  spec.fold = static_cast<int>(fold);
  TORCH_CHECK(fold == kFoldNone || fold == kFoldPearson, "moments_update: bad fold mode");
  if (fold == kFoldPearson) {
    TORCH_CHECK((mask >> kCOUNT & 1) && (mask >> kSPT & 1) && (mask >> kSPP & 1) && (mask >> kSTT & 1),
                "moments_update: the Pearson fold needs the SP/ST/SPP/STT/SPT/COUNT sums");
    for (int j = 0; j < 6; ++j) {
      const at::Tensor& d = dests[j];
      TORCH_CHECK(d.is_cuda() && d.is_contiguous() && d.get_device() == preds.get_device() && d.numel() == k,
                  "moments_update: folded states must be contiguous [k] tensors on the input's device");
      TORCH_CHECK(d.scalar_type() == at::kFloat || d.scalar_type() == at::kDouble,
                  "moments_update: folded states must be f32/f64");
      spec.fptr[j] = d.data_ptr();
      spec.fdtype[j] = d.scalar_type() == at::kFloat ? 0 : 1;
    }
  }
  for (int j = 0; j < spec.n; ++j) {
    const at::Tensor& d = dests[nfold + j];
    TORCH_CHECK(d.is_cuda() && d.is_contiguous(), "moments_update: destination states must be contiguous GPU tensors");
    TORCH_CHECK(d.get_device() == preds.get_device(), "moments_update: destination on another device");
    TORCH_CHECK(d.numel() == k || d.numel() == 1, "moments_update: destination must have k or 1 elements");
    spec.ptr[j] = d.data_ptr();
    // id < 32: sum[id];  id >= 32: sum[a] - sum[b] with id = 32 + 32 a + b
    const int64_t id = sum_ids[j];
    spec.sum_id[j] = static_cast<int>(id < 32 ? id : (id - 32) / 32);
    spec.sub_id[j] = static_cast<int>(id < 32 ? -1 : (id - 32) % 32);
    TORCH_CHECK(spec.sum_id[j] >= 0 && spec.sum_id[j] < kMaxSums && spec.sub_id[j] < kMaxSums,
                "moments_update: bad sum id");
    spec.per_col[j] = d.numel() == k && k > 1 ? 1 : (k == 1 ? 1 : 0);
    switch (d.scalar_type()) {
      case at::kFloat: spec.dtype[j] = 0; break;
      case at::kDouble: spec.dtype[j] = 1; break;
      case at::kLong: spec.dtype[j] = 2; break;
      default: TORCH_CHECK(false, "moments_update: destination dtype must be f32/f64/i64");
    }
  }
  auto s = stream();
  const float* sp = nullptr;
  const float* st = nullptr;
  if (shift_p.has_value()) {
    TORCH_CHECK(shift_p->scalar_type() == at::kFloat && shift_p->numel() == k, "shift_p must be f32[k]");
    sp = shift_p->data_ptr<float>();
  }
  if (shift_t.has_value()) {
    TORCH_CHECK(shift_t->scalar_type() == at::kFloat && shift_t->numel() == k, "shift_t must be f32[k]");
    st = shift_t->data_ptr<float>();
  }
  if (k > kColParMin) {
    // the one-column-per-thread-with-grid-stride scheme below needs a grid that is a multiple of k (partials of
    // O(k^2)): many outputs take the column-parallel kernel, ~2^18 threads in total, partials <= ~30 MB
    const long long col_blocks = (k + kBlock - 1) / kBlock;
    long long chunks = (1LL << 18) / k;
    chunks = chunks < 1 ? 1 : chunks;
    const long long max_chunks = (n_rows + 15) / 16;  // >= 16 rows per thread
    chunks = chunks > max_chunks ? max_chunks : chunks;
    chunks = chunks < 1 ? 1 : (chunks > 65535 ? 65535 : chunks);
    const long long rows_per_chunk = (n_rows + chunks - 1) / chunks;
    chunks = (n_rows + rows_per_chunk - 1) / rows_per_chunk;
    at::Tensor partial = at::empty({chunks, k, kMaxSums}, dopt);
    TM_DISPATCH_FLOAT(preds.scalar_type(), "moments_update", [&] {
      hipLaunchKernelGGL((moments_colpar_kernel<scalar_t>), dim3(static_cast<unsigned>(col_blocks),
                         static_cast<unsigned>(chunks)), dim3(kBlock), 0, s,
                         reinterpret_cast<const scalar_t*>(preds.data_ptr()),
                         reinterpret_cast<const scalar_t*>(target.data_ptr()), n_rows, k, rows_per_chunk,
                         static_cast<int>(mask), eps, power, sp, st, partial.data_ptr<double>());
    });
    hipLaunchKernelGGL(moments_finalize_kernel, dim3(k), dim3(kBlock), 0, s, partial.data_ptr<double>(),
                       static_cast<int>(chunks), k, spec, want_sums ? sums.data_ptr<double>() : nullptr,
                       static_cast<int>(mask));
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return sums;
  }
  // TM_AMD_MOMENTS_HANDOFF: the smallest n * k taking the multi-block hand-off (0 = never)
  static const long long handoff_min = [] {
    const char* e = std::getenv("TM_AMD_MOMENTS_HANDOFF");
    return e ? std::atoll(e) : 8192LL;  // below: the single block (one fewer round trip)
  }();
  if (handoff_min > 0 && n_rows * k >= handoff_min && kWave % k == 0 && n_rows * k <= kSmallMax) {
    // per-batch sizes of the streaming metrics (config #5: 8192 pairs): G blocks, the last one folds (no fence)
    const long long total = n_rows * k;
    static const long long per_block = [] {  // values per block (TM_AMD_MOMENTS_ROWS: measurement knob)
      const char* e = std::getenv("TM_AMD_MOMENTS_ROWS");
      return e ? std::max(64LL, std::atoll(e)) : static_cast<long long>(kHandoffRows);
    }();
    long long g = (total + per_block - 1) / per_block;
    g = std::min<long long>(g, std::min<long long>(128, kHandoffMaxRows / k));
    const int G = static_cast<int>(std::max<long long>(1, g));
    unsigned int* ticket = stream_ticket(preds.get_device(), s);
    static const bool fenced = [] {
      const char* e = std::getenv("TM_AMD_MOMENTS_FENCED");
      return e && std::atoi(e) != 0;
    }();
    at::Tensor partial = at::empty({G, k, kMaxSums}, dopt);
    const size_t lds = static_cast<size_t>(std::max(kHandoffThreads / kWave, G + 1)) * k * kMaxSums * sizeof(double);
    TM_DISPATCH_FLOAT(preds.scalar_type(), "moments_update", [&] {
      hipLaunchKernelGGL((moments_handoff_kernel<scalar_t>), dim3(G), dim3(kHandoffThreads), lds, s,
                         reinterpret_cast<const scalar_t*>(preds.data_ptr()),
                         reinterpret_cast<const scalar_t*>(target.data_ptr()), total, k, static_cast<int>(mask), eps,
                         power, sp, st, spec, want_sums ? sums.data_ptr<double>() : nullptr, partial.data_ptr<double>(),
                         ticket, fenced);
    });
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return sums;
  }
  static const int ablate = [] {
    const char* e = std::getenv("TM_AMD_MOMENTS_ABLATE");
    return e ? (std::atoi(e) & 7) : 0;
  }();
  if (kWave % k == 0 && n_rows * k <= kSmallMax) {
    // small per-batch sizes (below the hand-off threshold above): ONE 512-thread block, one launch
    const size_t lds = static_cast<size_t>(kSmallThreads / kWave + 1) * k * kMaxSums * sizeof(double);
    TM_DISPATCH_FLOAT(preds.scalar_type(), "moments_update", [&] {
      hipLaunchKernelGGL((moments_small_kernel<scalar_t>), dim3(1), dim3(kSmallThreads), lds, s,
                         reinterpret_cast<const scalar_t*>(preds.data_ptr()),
                         reinterpret_cast<const scalar_t*>(target.data_ptr()), n_rows * k, k,
                         static_cast<int>(mask) | (ablate << 27), eps, power, sp, st, spec,
                         want_sums ? sums.data_ptr<double>() : nullptr);
    });
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return sums;
  }
  // small updates (the common per-batch case): one block does the pass AND the fold -> a single launch
  // (measured, 8192 rows, k = 1: one block 16.4 us, 32 blocks + last-block fold 12.5 us, 32 blocks + finalize
  // launch 6.0 + 5.2 us: the single block stays for <= 4096 values)
  const bool fuse = n_rows * k <= 4096 && kBlock % k == 0;
  if (fuse) blocks = 1;
  // mid-size (a few blocks of partials): the last block folds them (a per-stream ticket word, re-armed by that block)
  unsigned int* ticket = nullptr;
  if (!fuse && blocks * k <= 256) ticket = stream_ticket(preds.get_device(), s);
  at::Tensor partial = at::empty({blocks, k, kMaxSums}, dopt);
  TM_DISPATCH_FLOAT(preds.scalar_type(), "moments_update", [&] {
    hipLaunchKernelGGL((moments_partial_kernel<scalar_t>), dim3(blocks), dim3(block), 0, s,
                       reinterpret_cast<const scalar_t*>(preds.data_ptr()),
                       reinterpret_cast<const scalar_t*>(target.data_ptr()), n_rows, k, static_cast<int>(mask), eps,
                       power, sp, st, partial.data_ptr<double>(), fuse ? 1 : 0, spec,
                       want_sums ? sums.data_ptr<double>() : nullptr, ticket);
  });
  if (!fuse && ticket == nullptr) {
    hipLaunchKernelGGL(moments_finalize_kernel, dim3(k), dim3(kBlock), 0, s, partial.data_ptr<double>(),
                       static_cast<int>(blocks), k, spec, want_sums ? sums.data_ptr<double>() : nullptr,
                       static_cast<int>(mask));
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return sums;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "moments_update(Tensor preds, Tensor target, int num_outputs, int mask, float eps, float power, "
      "Tensor? shift_p, Tensor? shift_t, Tensor(a!)[] dests, int[] sum_ids, bool want_sums, int fold=0) -> Tensor");
}

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("moments_update", &tm_amd::moments_update); }
