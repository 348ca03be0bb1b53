// Classification statistics kernels: confusion matrices and tp/fp/tn/fn for binary, multiclass and multilabel tasks.
//
// Replaces the reference's per-update chain (validation torch.unique + argmax + mask + bincount + diag/sum algebra,
// F/classification/stat_scores.py:90-131,344-419,647-681; confusion_matrix.py:333-337) with:
//   update = 1 fused pass over the inputs (argmax / threshold+sigmoid / ignore mask / range validation / histogram)
//          + 1 tiny finalize launch that folds the batch counts into the metric states and re-zeros the workspace.
// No host synchronisation anywhere in the update: invalid inputs raise bits in a device flag word.
//
// Multiclass argmax rows (C >= 32, X == 1): one wave64 per row, 16-byte vector loads, wave argmax with
// torch.argmax tie-breaking (first index; NaN wins).  Everything else: one thread per (sample, spatial) item.
// Small histograms are privatised in LDS (one int32 sub-histogram per block) and flushed with 64-bit atomics.
#include "../common/tm_common.h"

#include <mutex>
#include <unordered_map>

#include <cstdlib>

namespace tm_amd {
namespace {

constexpr int kBlock = 256;
constexpr int kLdsBins = 12288;  // 48 KiB of int32 bins
constexpr int kStageBytes = 16384;
constexpr long long kFinalizeOneBlock = 8192;  // label groups a single finalize block folds (then no re-arm launch)  // few-bin kernel: LDS copy of a block's 256 argmax rows

// ----------------------------------------------------------------------------------------------------------------
// multiclass: per-item predicted label
// ----------------------------------------------------------------------------------------------------------------
enum McMode : int { kMcConfmat = 0, kMcStats = 1, kMcConfmatDual = 2, kMcStatsDirect = 3 };
// dual: the batch matrix and the global one; stats-direct: straight into the tp / fp / tn / fn states (see
// mc_stats_direct)

template <typename target_t>
__device__ __forceinline__ bool mc_target(const target_t* __restrict__ target, long long item, int C, long long ignore,
                                          bool has_ignore, int* flag, int& t_out) {
  const long long t = static_cast<long long>(target[item]);
  if (has_ignore && t == ignore) return false;
  if (t < 0 || t >= C) {
    raise_flag(flag, kErrTargetOutOfRange);
    return false;
  }
  t_out = static_cast<int>(t);
  return true;
}

// accumulate one (target, predicted-set) observation; the K predicted labels are at pidx[0], pidx[pstride], ...
__device__ __forceinline__ void mc_accumulate(int mode, int t, const int* preds_k, int K, int C, int64_t* out,
                                              int* lds, bool use_lds, long long group) {
  if (mode == kMcConfmat) {
    const long long bin = static_cast<long long>(t) * C + preds_k[0];
    if (use_lds)
      atomicAdd(&lds[bin], 1);
    else
      atomic_add_i64(out + bin, 1);
    return;
  }
  // stats workspace layout per group: [tp(C) | fp(C) | fn(C) | (unused)]; every valid row adds exactly one to tp[t] or
  // fn[t], so the finalize derives the row count from them -- no per-row atomic on one shared count address (with
  // 8192 rows into one int64 that alone serialised the update at ~100 us)
  const long long base = group * (3LL * C + 1);
  bool hit = false;
  for (int k = 0; k < K; ++k) {
    const int p = preds_k[k];
    if (p == t) {
      hit = true;
    } else {
      if (use_lds) atomicAdd(&lds[C + p], 1);
      else atomic_add_i64(out + base + C + p, 1);
    }
  }
  const long long slot = hit ? t : 2LL * C + t;
  if (use_lds) atomicAdd(&lds[slot], 1);
  else atomic_add_i64(out + base + slot, 1);
}

__device__ __forceinline__ void lds_flush(int* lds, int nbins, int64_t* out) {
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    const int v = lds[b];
    if (v) atomic_add_i64(out + b, v);
  }
}

// wave-per-row argmax (X == 1). preds: [N, C] row-major. 16-B vector loads when rows are 16-B aligned.
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) mc_argmax_rows_kernel(const scalar_t* __restrict__ preds,
                                                                const target_t* __restrict__ target, long long N, int C,
                                                                long long ignore, bool has_ignore, int mode,
                                                                int64_t* __restrict__ out, int* __restrict__ flag,
                                                                bool vec, bool samplewise) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const int nbins = mode == kMcConfmat ? C * C : 3 * C + 1;
  const bool use_lds = !samplewise && nbins <= kLdsBins && (gridDim.x * (blockDim.x / kWave)) * 4LL <= N;
  if (use_lds) {
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) lds[b] = 0;
    __syncthreads();
  }
  const int lane = threadIdx.x & (kWave - 1);
  const long long wave = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  const long long nwaves = static_cast<long long>(gridDim.x) * blockDim.x / kWave;
  constexpr int kVec = 16 / sizeof(scalar_t);
  for (long long row = wave; row < N; row += nwaves) {
    const scalar_t* rp = preds + row * C;
    float best = -INFINITY;
    int bidx = 0x7fffffff;
    if (vec) {
      for (int c0 = lane * kVec; c0 < C; c0 += kWave * kVec) {
        const uint4 raw = *reinterpret_cast<const uint4*>(rp + c0);
        const scalar_t* e = reinterpret_cast<const scalar_t*>(&raw);
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
          const float v = to_f32(e[j]);
          if (argmax_better(v, c0 + j, best, bidx)) {
            best = v;
            bidx = c0 + j;
          }
        }
      }
    } else {
      for (int c = lane; c < C; c += kWave) {
        const float v = to_f32(rp[c]);
        if (argmax_better(v, c, best, bidx)) {
          best = v;
          bidx = c;
        }
      }
    }
    wave_argmax(best, bidx);
    if (lane == 0) {
      int t;
      if (mc_target(target, row, C, ignore, has_ignore, flag, t)) {
        mc_accumulate(mode, t, &bidx, 1, C, out, lds, use_lds, samplewise ? row : 0);
      }
    }
  }
  if (use_lds) lds_flush(lds, nbins, out);
}

// Sub-wave rows: a wave64 handles 64/LPR rows at once, LPR lanes per row. Every lane issues up to kBatch independent
// 16-byte loads before consuming any (memory-level parallelism instead of one dependent load chain per wave), the
// row's target is fetched in the same batch, and the argmax is reduced inside the LPR-lane group (log2(LPR)
// shuffles).  For C = 1000 bf16 (2000 B rows) LPR = 16 gives 8 loads in flight per lane, 4 rows per wave.
// Wave-per-row argmax with a software pipeline across rows: a persistent grid (a few blocks per CU) walks rows
// with a wave-uniform stride, and the 16-byte chunks of the *next* row are issued before the current row is reduced,
// so every wave keeps two rows of loads in flight instead of paying one full memory latency per row.
// kPer = 16-byte chunks per lane per row (ceil(C * sizeof(T) / 16 / 64)).
template <typename scalar_t, typename target_t, int kPer>
__global__ void __launch_bounds__(kBlock) mc_argmax_pipe_kernel(const scalar_t* __restrict__ preds,
                                                                const target_t* __restrict__ target, long long N,
                                                                int C, long long ignore, bool has_ignore, int mode,
                                                                int64_t* __restrict__ out, int* __restrict__ flag) {
  constexpr int kVec = 16 / sizeof(scalar_t);
  const int lane = threadIdx.x & (kWave - 1);
  const long long nwaves = static_cast<long long>(gridDim.x) * (blockDim.x / kWave);
  const long long wave = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  const int nchunks = C / kVec;
  u32x4 cur[kPer], nxt[kPer];
  long long tcur = 0, tnxt = 0;
  auto issue = [&](long long row, u32x4* buf, long long& t) {
    const u32x4* rp = reinterpret_cast<const u32x4*>(preds + row * C);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * kWave;
      if (ci < nchunks) buf[j] = __builtin_nontemporal_load(rp + ci);
    }
    if (lane == 0) t = static_cast<long long>(target[row]);
  };
  long long row = wave;
  if (row < N) issue(row, cur, tcur);
  for (; row < N; row += nwaves) {  // wave-uniform
    const long long next = row + nwaves;
    if (next < N) issue(next, nxt, tnxt);
    float best = -INFINITY;
    int bidx = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * kWave;
      if (ci < nchunks) {
        const scalar_t* e = reinterpret_cast<const scalar_t*>(&cur[j]);
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
          const float v = to_f32(e[k]);
          const int idx = ci * kVec + k;
          if (argmax_better(v, idx, best, bidx)) {
            best = v;
            bidx = idx;
          }
        }
      }
    }
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
      const float ov = __shfl_xor(best, off, kWave);
      const int oi = __shfl_xor(bidx, off, kWave);
      if (argmax_better(ov, oi, best, bidx)) {
        best = ov;
        bidx = oi;
      }
    }
    if (lane == 0) {
      const long long t = tcur;
      bool ok = true;
      if (has_ignore && t == ignore) ok = false;
      else if (t < 0 || t >= C) {
        raise_flag(flag, kErrTargetOutOfRange);
        ok = false;
      }
      if (ok) mc_accumulate(mode, static_cast<int>(t), &bidx, 1, C, out, nullptr, false, 0);
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) cur[j] = nxt[j];
    tcur = tnxt;
  }
}

// 16-bit float rows (bf16 / fp16): argmax on packed 16-bit ordinals.  A sign-magnitude half h maps to the
// order-preserving ordinal  h ^ ((h >>a 15) | 0x8000)  -- two halves per 32-bit word with v_pk_ashrrev_i16 + or + xor,
// folded into a lane max / min with v_pk_max_u16 / v_pk_min_u16.  A reverse scan then finds the lane's first column
// holding its max and ONE wave max over (ordinal << 16 | 0xffff - column) yields torch.argmax's first-max column.
// Rows where that shortcut is not exact fall back, wave-uniformly, to the float compare on the same registers:
// any NaN (positive NaN ordinals sit above +inf, negative ones below -inf) and a max of +-0 (-0 == +0 ties by index).
// Measured on MI355X (8192 x 1000 bf16, 8 blocks/CU): 5.2 us vs 8.1 us for the float-compare wave argmax, against a
// 3.3 us back-to-back empty-launch floor -- the float compare made the kernel VALU-bound (tools/mb/confmat_mb.hip).
template <typename scalar_t>
struct Ord16;
template <>
struct Ord16<c10::BFloat16> {
  static constexpr uint32_t kPosInf = 0xff80u, kNegInf = 0x007fu;
};
template <>
struct Ord16<c10::Half> {
  static constexpr uint32_t kPosInf = 0xfc00u, kNegInf = 0x03ffu;
};

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  return static_cast<uint32_t>(__reduce_max_sync(~0ull, static_cast<int>(v ^ 0x80000000u))) ^ 0x80000000u;
}

constexpr int kOrdBlock = 512;  // 8 waves: half the workgroups of 256-thread blocks for the same waves (measured on
                                // the 406 MB ring, tools/mb/confmat_ring_mb.hip: 5.06 us vs 5.38 us per 8192 x 1000)

template <typename scalar_t, typename target_t, int kPer, int kMode>
__global__ void __launch_bounds__(kOrdBlock) mc_argmax_ord16_kernel(const scalar_t* __restrict__ preds,
                                                                 const target_t* __restrict__ target, long long N,
                                                                 int C, long long ignore, bool has_ignore,
                                                                 int64_t* __restrict__ out, int* __restrict__ flag,
                                                                 int64_t* __restrict__ out2 = nullptr,
                                                                 int64_t* __restrict__ tn_st = nullptr,
                                                                 int64_t* __restrict__ fn_st = nullptr,
                                                                 long long tn_all = 0) {
  static_assert(sizeof(scalar_t) == 2, "16-bit floats only");
  if constexpr (kMode == kMcStatsDirect) {
    // every class gains a true negative per row of the batch; the rows' own classes give theirs back below (spread
    // over the grid's first threads: one add each, no block starts its rows behind C / 512 rounds of them)
    for (long long c = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; c < C;
         c += static_cast<long long>(gridDim.x) * blockDim.x)
      atomic_add_i64(tn_st + c, tn_all);
  }
  const int lane = threadIdx.x & (kWave - 1);
  const long long nwaves = static_cast<long long>(gridDim.x) * (blockDim.x / kWave);
  const long long wave = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  const int nchunks = C / 8;
  u32x4 cur[kPer], nxt[kPer];
  long long tcur = 0, tnxt = 0;
  auto issue = [&](long long row, u32x4* buf, long long& t) {
    const u32x4* rp = reinterpret_cast<const u32x4*>(preds + row * C);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * kWave;
      if (ci < nchunks) buf[j] = __builtin_nontemporal_load(rp + ci);
    }
    if (lane == 0) t = static_cast<long long>(target[row]);
  };
  long long row = wave;
  if (row < N) issue(row, cur, tcur);
  for (; row < N; row += nwaves) {  // wave-uniform
    const long long next = row + nwaves;
    if (next < N) issue(next, nxt, tnxt);
    u16x2 mx = {0, 0}, mn = {0xffff, 0xffff};
    uint32_t ordw[kPer][4];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * kWave;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t w = cur[j][k];
        const s16x2 sw = __builtin_bit_cast(s16x2, w);
        const uint32_t sgn = __builtin_bit_cast(uint32_t, static_cast<s16x2>(sw >> (s16x2){15, 15}));
        const uint32_t o = w ^ (sgn | 0x80008000u);
        ordw[j][k] = o;
        if (ci < nchunks) {
          const u16x2 ov = __builtin_bit_cast(u16x2, o);
          mx = __builtin_elementwise_max(mx, ov);
          mn = __builtin_elementwise_min(mn, ov);
        }
      }
    }
    const uint32_t lmax = mx.x > mx.y ? mx.x : mx.y;
    const uint32_t lmin = mn.x < mn.y ? mn.x : mn.y;
    uint32_t first = 0xffffu;  // lane's first column holding lmax (reverse scan: the last hit is the first column)
#pragma unroll
    for (int j = kPer - 1; j >= 0; --j) {
      const int ci = lane + j * kWave;
      if (ci < nchunks) {
#pragma unroll
        for (int k = 3; k >= 0; --k) {
          const uint32_t o = ordw[j][k];
          if ((o >> 16) == lmax) first = ci * 8 + 2 * k + 1;
          if ((o & 0xffffu) == lmax) first = ci * 8 + 2 * k;
        }
      }
    }
    const uint32_t key = wave_max_u32((lmax << 16) | (0xffffu - first));
    const uint32_t kmax = key >> 16;
    const bool exact = kmax <= Ord16<scalar_t>::kPosInf && kmax != 0x8000u && kmax != 0x7fffu &&
                       !__any(lmin < Ord16<scalar_t>::kNegInf);
    int bidx = 0xffff - static_cast<int>(key & 0xffffu);
    if (!exact) {  // wave-uniform, rare
      float best = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int ci = lane + j * kWave;
        if (ci < nchunks) {
          const scalar_t* e = reinterpret_cast<const scalar_t*>(&cur[j]);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float v = to_f32(e[k]);
            if (argmax_better(v, ci * 8 + k, best, bi)) {
              best = v;
              bi = ci * 8 + k;
            }
          }
        }
      }
      wave_argmax(best, bi);
      bidx = bi;
    }
    if (lane == 0) {
      const long long t = tcur;
      bool ok = true;
      if (has_ignore && t == ignore) ok = false;
      else if (t < 0 || t >= C) {
        raise_flag(flag, kErrTargetOutOfRange);
        ok = false;
      }
      if (ok) {
        if constexpr (kMode == kMcConfmat) {
          atomic_add_i64(out + static_cast<long long>(t) * C + bidx, 1);
        } else if constexpr (kMode == kMcConfmatDual) {  // forward(): the batch value and the global state at once
          atomic_add_i64(out + static_cast<long long>(t) * C + bidx, 1);
          atomic_add_i64(out2 + static_cast<long long>(t) * C + bidx, 1);
        } else if constexpr (kMode == kMcStatsDirect) {  // out = tp, out2 = fp
          atomic_add_i64(tn_st + t, -1);
          if (bidx == t) {
            atomic_add_i64(out + t, 1);
          } else {
            atomic_add_i64(out2 + bidx, 1);
            atomic_add_i64(fn_st + t, 1);
            atomic_add_i64(tn_st + bidx, -1);
          }
        } else {  // stats workspace [tp | fp | fn | -]: a hit or a miss of the target class (+ the predicted class)
          if (bidx == t) {
            atomic_add_i64(out + t, 1);
          } else {
            atomic_add_i64(out + C + bidx, 1);
            atomic_add_i64(out + 2LL * C + t, 1);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) cur[j] = nxt[j];
    tcur = tnxt;
  }
}

template <typename scalar_t, typename target_t, int LPR>
__global__ void __launch_bounds__(kBlock) mc_argmax_subwave_kernel(const scalar_t* __restrict__ preds,
                                                                   const target_t* __restrict__ target, long long N,
                                                                   int C, long long ignore, bool has_ignore, int mode,
                                                                   int64_t* __restrict__ out, int* __restrict__ flag,
                                                                   bool samplewise) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  constexpr int kVec = 16 / sizeof(scalar_t);
  constexpr int kRowsPerWave = kWave / LPR;
  constexpr int kBatch = 8;
  const int nbins = mode == kMcConfmat ? C * C : 3 * C + 1;
  const long long nwaves = static_cast<long long>(gridDim.x) * (blockDim.x / kWave);
  const bool use_lds = !samplewise && nbins <= kLdsBins && nwaves * kRowsPerWave * 4LL <= N;
  if (use_lds) {
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) lds[b] = 0;
    __syncthreads();
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane / LPR;
  const int sl = lane - sub * LPR;
  const long long wave = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  const int nchunks = C / kVec;
  for (long long base = wave * kRowsPerWave; base < N; base += nwaves * kRowsPerWave) {  // wave-uniform loop
    const long long row = base + sub;
    const bool live = row < N;
    long long t = 0;
    if (live && sl == 0) t = static_cast<long long>(target[row]);
    const u32x4* rp = reinterpret_cast<const u32x4*>(preds + (live ? row : 0) * C);
    float best = -INFINITY;
    int bidx = 0x7fffffff;
    for (int c0 = sl; c0 < nchunks; c0 += LPR * kBatch) {
      u32x4 buf[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int ci = c0 + j * LPR;
        if (live && ci < nchunks) buf[j] = rp[ci];
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int ci = c0 + j * LPR;
        if (live && ci < nchunks) {
          const scalar_t* e = reinterpret_cast<const scalar_t*>(&buf[j]);
#pragma unroll
          for (int k = 0; k < kVec; ++k) {
            const float v = to_f32(e[k]);
            const int idx = ci * kVec + k;
            if (argmax_better(v, idx, best, bidx)) {
              best = v;
              bidx = idx;
            }
          }
        }
      }
    }
#pragma unroll
    for (int off = LPR / 2; off > 0; off >>= 1) {
      const float ov = __shfl_xor(best, off, kWave);
      const int oi = __shfl_xor(bidx, off, kWave);
      if (argmax_better(ov, oi, best, bidx)) {
        best = ov;
        bidx = oi;
      }
    }
    if (live && sl == 0) {
      bool ok = true;
      if (has_ignore && t == ignore) ok = false;
      else if (t < 0 || t >= C) {
        raise_flag(flag, kErrTargetOutOfRange);
        ok = false;
      }
      if (ok) mc_accumulate(mode, static_cast<int>(t), &bidx, 1, C, out, lds, use_lds, samplewise ? row : 0);
    }
  }
  if (use_lds) lds_flush(lds, nbins, out);
}

// thread-per-item: preds is either float scores [N, C, X] (argmax over C, stride X) or int labels [N, K, X].
template <typename scalar_t, typename target_t, bool kArgmax>
__global__ void __launch_bounds__(kBlock) mc_items_kernel(const scalar_t* __restrict__ preds,
                                                          const target_t* __restrict__ target, long long N,
                                                          long long X, int C, int K, long long ignore, bool has_ignore,
                                                          int mode, int64_t* __restrict__ out, int* __restrict__ flag,
                                                          bool samplewise) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const int nbins = mode == kMcConfmat ? C * C : 3 * C + 1;
  const long long items = N * X;
  const bool use_lds = !samplewise && nbins <= kLdsBins && static_cast<long long>(gridDim.x) * blockDim.x * 4 <= items;
  if (use_lds) {
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) lds[b] = 0;
    __syncthreads();
  }
  int pk[16];
  for (long long it = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; it < items;
       it += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long n = it / X, x = it - n * X;
    int t;
    if (!mc_target(target, it, C, ignore, has_ignore, flag, t)) continue;
    bool ok = true;
    if constexpr (kArgmax) {
      const scalar_t* p = preds + n * C * X + x;
      float best = to_f32(p[0]);
      int bidx = 0;
      for (int c = 1; c < C; ++c) {
        const float v = to_f32(p[static_cast<long long>(c) * X]);
        if (argmax_better(v, c, best, bidx)) {
          best = v;
          bidx = c;
        }
      }
      pk[0] = bidx;
    } else {
      const scalar_t* p = preds + n * K * X + x;
      if (K == 1) {
        const long long v = static_cast<long long>(p[0]);
        ok = v >= 0 && v < C;
        pk[0] = static_cast<int>(v);
      } else for (int k = 0; k < K; ++k) {
        const long long v = static_cast<long long>(p[static_cast<long long>(k) * X]);
        if (v < 0 || v >= C) {
          ok = false;
          break;
        }
        pk[k] = static_cast<int>(v);
      }
      if (!ok) {
        raise_flag(flag, kErrPredsOutOfRange);
        continue;
      }
    }
    mc_accumulate(mode, t, pk, kArgmax ? 1 : K, C, out, lds, use_lds, samplewise ? n : 0);
  }
  if (use_lds) lds_flush(lds, nbins, out);
}

// Few-bin multiclass path (nbins <= 256, e.g. C <= 85 stats / C <= 16 confusion matrix): every bin is a popcount of
// a wave ballot, accumulated in the registers of the lane owning the bin (lane = bin % 64, slot = bin / 64).  With few
// bins the LDS/global atomic histogram serialises on a handful of hot addresses (8192 x 10 classes: 75 us); here a
// wave spends one ballot per bin per 64 items and the block flushes <= 256 int64 atomics.
template <typename scalar_t, typename target_t, bool kArgmax>
__global__ void __launch_bounds__(kBlock) mc_fewbins_kernel(const scalar_t* __restrict__ preds,
                                                            const target_t* __restrict__ target, long long N,
                                                            long long X, int C, long long ignore, bool has_ignore,
                                                            int mode, int64_t* __restrict__ out,
                                                            int* __restrict__ flag, bool stage) {
  __shared__ int lds[256];
  // stage (argmax, X == 1, 256 * C * sizeof(scalar_t) <= kStageBytes): the block's 256 rows are one contiguous
  // piece of preds, copied into LDS with 16-byte loads; each lane then reads its row from LDS (instead of C
  // 2-4 byte loads per lane with a C-element stride across the wave)
  __shared__ __attribute__((aligned(16))) unsigned char stage_raw[kStageBytes];
  const scalar_t* srow = reinterpret_cast<const scalar_t*>(stage_raw);
  const int nbins = mode == kMcConfmat ? C * C : 3 * C + 1;
  const int lane = threadIdx.x & (kWave - 1);
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) lds[b] = 0;
  __syncthreads();
  int acc[4] = {0, 0, 0, 0};
  const long long items = N * X;
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  // loop bounds are block-uniform so every ballot sees the whole wave (and the staging barriers the whole block)
  for (long long bbase = static_cast<long long>(blockIdx.x) * blockDim.x; bbase < items; bbase += stride) {
    if (kArgmax && stage) {
      __syncthreads();  // the previous rows are read
      const long long rows = items - bbase < blockDim.x ? items - bbase : blockDim.x;
      const long long nbytes = rows * C * static_cast<long long>(sizeof(scalar_t));
      const unsigned char* src = reinterpret_cast<const unsigned char*>(preds + bbase * C);
      for (long long o = threadIdx.x * 16LL; o + 16 <= nbytes; o += blockDim.x * 16LL)
        *reinterpret_cast<u32x4*>(stage_raw + o) = *reinterpret_cast<const u32x4*>(src + o);
      for (long long o = (nbytes / 16) * 16 + threadIdx.x; o < nbytes; o += blockDim.x) stage_raw[o] = src[o];
      __syncthreads();
    }
    const long long it = bbase + threadIdx.x;
    int t = -1, p = -1;
    if (it < items && mc_target(target, it, C, ignore, has_ignore, flag, t)) {
      const long long n = it / X, x = it - n * X;
      if constexpr (kArgmax) {
        const bool staged = stage;
        const scalar_t* pr = staged ? srow + static_cast<long long>(threadIdx.x) * C : preds + n * C * X + x;
        const long long cs = staged ? 1 : X;
        float best = to_f32(pr[0]);
        int bidx = 0;
        for (int c = 1; c < C; ++c) {
          const float v = to_f32(pr[static_cast<long long>(c) * cs]);
          if (argmax_better(v, c, best, bidx)) {
            best = v;
            bidx = c;
          }
        }
        p = bidx;
      } else {
        const long long v = static_cast<long long>(preds[it]);
        if (v < 0 || v >= C) {
          raise_flag(flag, kErrPredsOutOfRange);
          t = -1;
        } else {
          p = static_cast<int>(v);
        }
      }
    }
    const bool valid = t >= 0;
    if (mode == kMcConfmat) {
      const int key = valid ? t * C + p : -1;
#pragma unroll
      for (int slot = 0; slot < 4; ++slot) {
        const int b0 = slot * kWave;
        if (b0 >= nbins) break;
        const int nb = min(kWave, nbins - b0);
        for (int l = 0; l < nb; ++l) {
          const int cnt = __popcll(__ballot(key == b0 + l));
          if (lane == l) acc[slot] += cnt;
        }
      }
    } else {
      for (int c = 0; c < C; ++c) {
        const int tp = __popcll(__ballot(valid && p == c && t == c));
        const int fp = __popcll(__ballot(valid && p == c && t != c));
        const int fn = __popcll(__ballot(valid && t == c && p != c));
        const int bt = c, bf = C + c, bn = 2 * C + c;
        if ((bt & (kWave - 1)) == lane) acc[bt >> 6] += tp;
        if ((bf & (kWave - 1)) == lane) acc[bf >> 6] += fp;
        if ((bn & (kWave - 1)) == lane) acc[bn >> 6] += fn;
      }
    }
  }
#pragma unroll
  for (int slot = 0; slot < 4; ++slot) {
    const int b = slot * kWave + lane;
    if (b < nbins && acc[slot]) atomicAdd(&lds[b], acc[slot]);
  }
  lds_flush(lds, nbins, out);
}

// Few-class multiclass argmax rows, tiled (X == 1, C <= kTileMaxC, C * sizeof <= 128 B, 16-B aligned preds): the
// streaming version of mc_fewbins_kernel's LDS staging.  A persistent block walks tiles of 256 * R rows (<= 32 KiB of
// logits, one contiguous piece of preds): it issues ALL 16-byte loads of its NEXT tile (and that tile's targets) into
// registers before it evaluates the current one from LDS, so every block keeps a whole tile of loads in flight while
// it computes.  Each valid row is ONE LDS atomic into the block's C x C (target, prediction) histogram; the block
// stores the histogram to its slot of a partials buffer and fewbins_fold_kernel sums the slots into the matrix
// (confusion-matrix mode) or the tp / fp / fn derived from it (stats mode: diagonal, column sum - diagonal, row sum -
// diagonal).  TM_AMD_FEWBINS_FOLD=0 restores the per-block global-atomic flush.  (The ballot-per-bin counting this replaces cost O(bins) wave instructions per
// row: 1 M x 10 bf16 rows ran at 0.56 TB/s, a 65536-row batch took 28 us.)
constexpr int kTileChunks = 8;  // 16-byte loads per thread per tile (256 threads x 8 x 16 B = 32 KiB)
constexpr int kTileRows = 8;    // rows per thread per tile (max R)
constexpr int kTileMaxC = 64;   // the C x C LDS histogram: <= 16 KiB
// 16-bit rows of <= 32 B: ordinal argmax (row_argmax_ord16).  Measured (1 M rows, bf16): C = 10 10.4 -> 10.0 us,
// C = 16 13.7 -> 12.5 us; the 32-dword variant (C = 32 / 64) ran slower (40.8 -> 46.8 us, 85 -> 101 us)
constexpr int kOrdRowsMaxNW = 8;

// argmax of one row held in LDS at byte offset `off` (16-bit or 32-bit scores): the row's dwords are read into
// registers first (NW + 1 independent LDS reads, one wait), realigned for rows that start mid-dword (odd C with
// 16-bit scores), then compared from registers with compile-time indices -- instead of a chain of dependent
// element reads, each paying the LDS latency.  Same tie / NaN rule as argmax_better (first maximum; NaN wins).
template <typename scalar_t, int NW>
__device__ __forceinline__ int row_argmax_regs(const unsigned char* __restrict__ lds, int off, int C) {
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(lds + (off & ~3));
  uint32_t w[NW + 1];
#pragma unroll
  for (int i = 0; i <= NW; ++i) w[i] = wp[i];
  const uint32_t sh = static_cast<uint32_t>(off & 3) * 8;  // 0 or 16
  uint32_t a[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) a[i] = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
  constexpr int kPerWord = 4 / sizeof(scalar_t);
  float best = 0.0f;
  int bidx = 0;
#pragma unroll
  for (int j = 0; j < NW * kPerWord; ++j) {
    if (j < C) {
      const uint32_t word = a[j / kPerWord];
      float v;
      if constexpr (sizeof(scalar_t) == 4) {
        v = __builtin_bit_cast(float, word);
      } else {
        const uint16_t h = static_cast<uint16_t>((j % kPerWord) ? (word >> 16) : (word & 0xffffu));
        v = to_f32(__builtin_bit_cast(scalar_t, h));
      }
      if (j == 0) {
        best = v;
      } else {
        const bool take = (v != v) ? !(best != best) : (v > best);  // argmax_better against an earlier column
        if (take) {
          best = v;
          bidx = j;
        }
      }
    }
  }
  return bidx;
}

// The same argmax for 16-bit scores on order-preserving ordinals (the Ord16 mapping of mc_argmax_ord16_kernel): per
// pair of columns one packed ordinal (v_pk_ashrrev_i16 + or + xor), then per column one 32-bit key
// (ordinal << 16 | 0xffff - column) into a max -- the first maximum wins ties -- about 4 VALU per column instead of
// the ~15 of the NaN-aware float compare (the tile kernel's row work was VALU-bound: 1 M x 10 bf16 spent 6 us of its
// 11 us on it).  Rows where ordinals are not exact -- a NaN anywhere (positive NaN ordinals sit above +inf, negative
// ones below -inf) or a maximum of +-0 (-0 == +0 ties by column) -- take the float compare instead.
template <typename scalar_t, int NW>
__device__ __forceinline__ int row_argmax_ord16(const unsigned char* __restrict__ lds, int off, int C) {
  const uint32_t* wp = reinterpret_cast<const uint32_t*>(lds + (off & ~3));
  uint32_t w[NW + 1];
#pragma unroll
  for (int i = 0; i <= NW; ++i) w[i] = wp[i];
  const uint32_t sh = static_cast<uint32_t>(off & 3) * 8;  // 0 or 16
  uint32_t best = 0u, mn = 0xffffffffu;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    if (2 * i < C) {  // uniform
      const uint32_t a = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
      const s16x2 sg = __builtin_bit_cast(s16x2, a) >> static_cast<short>(15);
      uint32_t o = a ^ (__builtin_bit_cast(uint32_t, sg) | 0x80008000u);
      best = max(best, (o << 16) | (0xffffu - 2 * i));
      if (2 * i + 1 < C) best = max(best, (o & 0xffff0000u) | (0xffffu - (2 * i + 1)));
      else o |= 0xffff0000u;  // past the row's end: out of the min
      mn = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, mn), __builtin_bit_cast(u16x2, o)));
    }
  }
  const uint32_t mo = best >> 16;
  const uint32_t lo = min(mn & 0xffffu, mn >> 16);
  if (mo > Ord16<scalar_t>::kPosInf || lo < Ord16<scalar_t>::kNegInf || mo == 0x7fffu || mo == 0x8000u)
    return row_argmax_regs<scalar_t, NW>(lds, off, C);
  return static_cast<int>(0xffffu - (best & 0xffffu));
}

// Add one C x C (target, prediction) histogram held in LDS to its destination: the confusion matrix (kMcConfmat), the
// stats workspace [tp | fp | fn | -] (kMcStats), or the four int64 states (kMcStatsDirect: out = tp; tn gets the
// histogram's rows minus tp + fp + fn).  Every output is linear in the histogram, so per-block or per-group
// histograms add up to the batch's.  `red`: >= C long longs of LDS scratch (not aliasing `hist`).  Block-uniform.
template <typename count_t>
__device__ __forceinline__ void flush_hist(const count_t* hist, int C, int mode, int64_t* __restrict__ out,
                                           int64_t* __restrict__ fp_s, int64_t* __restrict__ tn_s,
                                           int64_t* __restrict__ fn_s, long long* red) {
  if (mode == kMcConfmat) {
    for (int b = threadIdx.x; b < C * C; b += kBlock) {
      const long long v = hist[b];
      if (v) atomic_add_i64(out + b, v);
    }
    return;
  }
  const int c = threadIdx.x;  // C <= kTileMaxC < kBlock: one thread per class
  long long tp = 0, row = 0, col = 0;
  if (c < C) {
    tp = hist[c * C + c];
    for (int j = 0; j < C; ++j) {
      row += hist[c * C + j];  // target c
      col += hist[j * C + c];  // predicted c
    }
  }
  if (mode == kMcStats) {
    if (c < C) {
      if (tp) atomic_add_i64(out + c, tp);
      if (col - tp) atomic_add_i64(out + C + c, col - tp);
      if (row - tp) atomic_add_i64(out + 2LL * C + c, row - tp);
    }
    return;
  }
  if (c < C) red[c] = row;
  __syncthreads();
  if (c < C) {
    long long rows = 0;
    for (int j = 0; j < C; ++j) rows += red[j];
    if (tp) atomic_add_i64(out + c, tp);
    if (col - tp) atomic_add_i64(fp_s + c, col - tp);
    if (row - tp) atomic_add_i64(fn_s + c, row - tp);
    if (rows - row - col + tp) atomic_add_i64(tn_s + c, rows - row - col + tp);
  }
}

// Group hand-off of the tile kernel (tickets != nullptr): block b belongs to group b % ngroups (with blocks dispatched
// round-robin over the XCDs, a group of 8 is one XCD's blocks); it stores its histogram to its partials row, and the
// LAST block of each group to finish sums the group's rows and flushes them with flush_hist -- ngroups x (C^2 or 4C)
// atomics instead of one per block, and no fold / finalize launch.  Only for C^2 <= 256 bins (the folder's loads stay
// one round: 8 x 256 / C^2 rows per group); measured (1 M x 10 bf16): 9.9 us tile + 4.7 us fold kernel + finalize ->
// 14.1 us in one launch (groups of 32 blocks, two load rounds: 17.9 us; per-block int64 flush: 26.8 us).  Memory model: the "sc1 payload" hand-off of
// moments_handoff_kernel (agent-scope stores drained by vmcnt(0) before the barrier and the agent-scope ticket add;
// agent-scope loads in the last block); the last block re-arms its ticket word.
constexpr int kGroupLoads = 8;       // member rows per folding thread: a group's rows are ONE round of loads
constexpr int kGroupMaxBlocks = 16;  // blocks per ticket word

template <typename scalar_t, typename target_t, int NW>
__global__ void __launch_bounds__(kBlock) mc_fewbins_tile_kernel(const scalar_t* __restrict__ preds,
                                                                 const target_t* __restrict__ target, long long N,
                                                                 int C, int R, long long ignore, bool has_ignore,
                                                                 int mode, int64_t* __restrict__ out,
                                                                 int* __restrict__ part, int* __restrict__ flag,
                                                                 unsigned int* __restrict__ tickets, int ngroups,
                                                                 int64_t* __restrict__ fp_s, int64_t* __restrict__ tn_s,
                                                                 int64_t* __restrict__ fn_s) {
  // dynamic LDS: the C x C histogram (padded to 16 B), then the logits tile (+ 256 B: row_argmax_regs reads up to
  // NW + 1 dwords from the last row's start) -- a 10-class block takes 33 KiB, so 4 blocks fit a CU
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int last;
  const int ncm = C * C;
  int* hist = reinterpret_cast<int*>(smem);
  unsigned char* tile_raw = smem + ((ncm * 4 + 15) & ~15);
  for (int b = threadIdx.x; b < ncm; b += kBlock) hist[b] = 0;
  const long long TR = static_cast<long long>(kBlock) * R;  // rows per tile
  const long long ntiles = (N + TR - 1) / TR;
  const long long row_bytes = static_cast<long long>(C) * sizeof(scalar_t);
  u32x4 buf[kTileChunks];
  long long tbuf[kTileRows];
  long long nbytes_cur = 0;
  auto issue = [&](long long tile, long long& nbytes) {
    const long long r0 = tile * TR;
    const long long rows = N - r0 < TR ? N - r0 : TR;
    nbytes = rows * row_bytes;
    const unsigned char* src = reinterpret_cast<const unsigned char*>(preds + r0 * C);
#pragma unroll
    for (int j = 0; j < kTileChunks; ++j) {
      const long long o = (static_cast<long long>(j) * kBlock + threadIdx.x) * 16;
      if (o + 16 <= nbytes) buf[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + o));
    }
#pragma unroll
    for (int k = 0; k < kTileRows; ++k) {
      const long long row = r0 + static_cast<long long>(k) * kBlock + threadIdx.x;
      if (k < R && row < N) tbuf[k] = static_cast<long long>(__builtin_nontemporal_load(target + row));
    }
  };
  long long tile = blockIdx.x;
  if (tile < ntiles) issue(tile, nbytes_cur);
  for (; tile < ntiles; tile += gridDim.x) {  // block-uniform
    const long long nbytes = nbytes_cur;
    long long tcur[kTileRows];
#pragma unroll
    for (int k = 0; k < kTileRows; ++k) tcur[k] = tbuf[k];
    __syncthreads();  // the previous tile's rows are read (and, first time round, the histogram is zeroed)
#pragma unroll
    for (int j = 0; j < kTileChunks; ++j) {
      const long long o = (static_cast<long long>(j) * kBlock + threadIdx.x) * 16;
      if (o + 16 <= nbytes) *reinterpret_cast<u32x4*>(tile_raw + o) = buf[j];
    }
    if (nbytes % 16) {  // the last tile's ragged end
      const unsigned char* src = reinterpret_cast<const unsigned char*>(preds + tile * TR * C);
      for (long long o = (nbytes / 16) * 16 + threadIdx.x; o < nbytes; o += kBlock) tile_raw[o] = src[o];
    }
    __syncthreads();
    const long long next = tile + gridDim.x;
    if (next < ntiles) issue(next, nbytes_cur);  // in flight while this tile is evaluated
    const scalar_t* lrow = reinterpret_cast<const scalar_t*>(tile_raw);
#pragma unroll
    for (int k = 0; k < kTileRows; ++k) {
      if (k >= R) break;  // uniform
      const long long rt = static_cast<long long>(k) * kBlock + threadIdx.x;  // row within the tile
      const long long row = tile * TR + rt;
      if (row >= N) continue;
      const long long tv = tcur[k];
      if (has_ignore && tv == ignore) continue;
      if (tv < 0 || tv >= C) {
        raise_flag(flag, kErrTargetOutOfRange);
        continue;
      }
      int bidx = 0;
      if constexpr (NW > 0 && (sizeof(scalar_t) == 2 || sizeof(scalar_t) == 4)) {
        if constexpr (sizeof(scalar_t) == 2 && NW <= kOrdRowsMaxNW)
          bidx = row_argmax_ord16<scalar_t, NW>(tile_raw, static_cast<int>(rt * C * sizeof(scalar_t)), C);
        else
          bidx = row_argmax_regs<scalar_t, NW>(tile_raw, static_cast<int>(rt * C * sizeof(scalar_t)), C);
      } else {  // 8-byte scores: element reads from LDS
        const scalar_t* pr = lrow + rt * C;
        float best = to_f32(pr[0]);
        for (int c = 1; c < C; ++c) {
          const float v = to_f32(pr[c]);
          if (argmax_better(v, c, best, bidx)) {
            best = v;
            bidx = c;
          }
        }
      }
      atomicAdd(&hist[static_cast<int>(tv) * C + bidx], 1);
    }
  }
  __syncthreads();
  if (tickets != nullptr) {
    const int g = static_cast<int>(blockIdx.x % ngroups);
    const int gsize = static_cast<int>((gridDim.x - g + ngroups - 1) / ngroups);
    int* dst = part + static_cast<long long>(blockIdx.x) * ncm;
    for (int b = threadIdx.x; b < ncm; b += kBlock)
      __hip_atomic_store(dst + b, hist[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores are done
    __syncthreads();
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(tickets + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             static_cast<unsigned>(gsize - 1);
    __syncthreads();
    if (!last) return;
    // the group's rows g, g + ngroups, ...: per bin, tpb threads each sum every tpb-th member row (independent loads,
    // 8 in flight), then the tpb partial sums are combined in LDS (the tile area is free now)
    long long* psum = reinterpret_cast<long long*>(tile_raw);                     // [tpb][ncm] when ncm <= kBlock
    long long* tot = ncm <= kBlock ? psum + kBlock : psum;                        // [ncm]
    long long* red = reinterpret_cast<long long*>(hist);                          // >= C long longs (C >= 2)
    const int tpb = ncm <= kBlock ? kBlock / ncm : 1;
    for (int b0 = 0; b0 < ncm; b0 += kBlock / tpb) {
      const int b = b0 + (threadIdx.x % (kBlock / tpb)), j = threadIdx.x / (kBlock / tpb);
      long long s = 0;
      if (b < ncm && j < tpb) {
        for (int m = j; m < gsize; m += 8 * tpb) {
          int v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int mm = m + u * tpb;
            v[u] = mm < gsize ? __hip_atomic_load(part + static_cast<long long>(g + mm * ngroups) * ncm + b,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : 0;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) s += v[u];
        }
      }
      if (tpb == 1) {
        if (b < ncm) tot[b] = s;
      } else if (b < ncm && j < tpb) {
        psum[j * ncm + b] = s;
      }
    }
    if (tpb > 1) {
      __syncthreads();
      for (int b = threadIdx.x; b < ncm; b += kBlock) {
        long long s = 0;
        for (int j = 0; j < tpb; ++j) s += psum[j * ncm + b];
        tot[b] = s;
      }
    }
    __syncthreads();
    flush_hist(tot, C, mode, out, fp_s, tn_s, fn_s, red);
    if (threadIdx.x == 0) __hip_atomic_store(tickets + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
  } else if (part != nullptr) {  // this block's histogram, plain stores: fewbins_fold_kernel sums the blocks
    int* dst = part + static_cast<long long>(blockIdx.x) * ncm;
    for (int b = threadIdx.x; b < ncm; b += kBlock) dst[b] = hist[b];
  } else {  // per-block flush (a few blocks)
    flush_hist(hist, C, mode, out, fp_s, tn_s, fn_s, reinterpret_cast<long long*>(tile_raw));
  }
}

// Sum of the tile kernel's per-block C x C histograms [nblk, C * C] (int32).  Grid: x = groups of 64 bins (lanes walk
// consecutive bins), y = splits of the blocks; each of the block's 16 waves sums at most kFoldRows rows, all its loads
// in flight at once.  Confusion-matrix mode adds each bin into the matrix (plain add when there is one split, else one
// atomic per split); stats mode gathers the block's tp (diagonal), fp (prediction column) and fn (target row) per
// class in LDS and adds each non-zero one to the workspace with one atomic.  Measured on MI355X (1 M x 10 bf16, 512
// tile blocks): the per-block global-atomic flush this replaces cost 6.4 us (confusion matrix, C^2 addresses) and
// 12 us (stats, 3C addresses: every address takes one serialised atomic per block); the fold runs in ~4.6 us.
constexpr int kFoldThreads = 1024;
constexpr int kFoldRows = 8;
constexpr int kFoldMinBlocks = 64;  // grids up to this many blocks keep the per-block atomic flush
__global__ void __launch_bounds__(kFoldThreads) fewbins_fold_kernel(const int* __restrict__ part, int nblk, int C,
                                                                     int mode, int64_t* __restrict__ out) {
  constexpr int kW = kFoldThreads / kWave;
  __shared__ long long red[kW][kWave];  // 64-bit sums: up to 128 blocks' int32 counts
  __shared__ unsigned long long cls[3][kTileMaxC];
  const int ncm = C * C;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int bin = blockIdx.x * kWave + lane;
  const int r0 = blockIdx.y * kW * kFoldRows + w;
  int v[kFoldRows];
#pragma unroll
  for (int i = 0; i < kFoldRows; ++i) {
    const int r = r0 + i * kW;
    v[i] = (bin < ncm && r < nblk) ? part[static_cast<long long>(r) * ncm + bin] : 0;
  }
  long long acc = 0;
#pragma unroll
  for (int i = 0; i < kFoldRows; ++i) acc += v[i];
  red[w][lane] = acc;
  if (mode != kMcConfmat)
    for (int i = threadIdx.x; i < 3 * kTileMaxC; i += kFoldThreads) cls[i / kTileMaxC][i % kTileMaxC] = 0;
  __syncthreads();
  if (w == 0 && bin < ncm) {
    long long tot = 0;
#pragma unroll
    for (int i = 0; i < kW; ++i) tot += red[i][lane];
    if (tot) {
      if (mode == kMcConfmat) {
        if (gridDim.y == 1) out[bin] += tot;
        else atomic_add_i64(out + bin, tot);
      } else {
        const int t = bin / C, p = bin - t * C;
        if (t == p) {
          atomicAdd(&cls[0][t], static_cast<unsigned long long>(tot));
        } else {
          atomicAdd(&cls[1][p], static_cast<unsigned long long>(tot));
          atomicAdd(&cls[2][t], static_cast<unsigned long long>(tot));
        }
      }
    }
  }
  if (mode != kMcConfmat) {
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * C; i += kFoldThreads) {
      const long long c = static_cast<long long>(cls[i / C][i % C]);
      if (c) atomic_add_i64(out + i, c);  // [tp | fp | fn] are consecutive C-blocks of the workspace
    }
  }
}

// fold a multiclass stats workspace [G, 3C+1] into the states; optionally micro-reduce over classes.
// accumulate=true: states += batch ; false: states = batch (samplewise outputs). Re-zeros the workspace.
template <int kT>
__global__ void __launch_bounds__(kT) mc_finalize_kernel(int64_t* __restrict__ ws, int C, bool micro,
                                                             bool accumulate, int64_t* __restrict__ tp,
                                                             int64_t* __restrict__ fp, int64_t* __restrict__ tn,
                                                             int64_t* __restrict__ fn) {
  const long long g = blockIdx.x;
  int64_t* w = ws + g * (3LL * C + 1);
  __shared__ long long red[3][kT / kWave];
  // rows counted in this group = sum over classes of tp + fn (each valid row is a hit or a miss of its target class)
  long long rows = 0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) rows += w[c] + w[2 * C + c];
  rows = wave_sum_ll(rows);
  if ((threadIdx.x & (kWave - 1)) == 0) red[0][threadIdx.x / kWave] = rows;
  __syncthreads();
  long long cnt = 0;
  for (int i = 0; i < static_cast<int>(blockDim.x / kWave); ++i) cnt += red[0][i];
  __syncthreads();  // red is reused by the micro reduction below
  long long st = 0, sf = 0, sn = 0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const long long a = w[c], b = w[C + c], d = w[2 * C + c];
    if (micro) {
      st += a;
      sf += b;
      sn += d;
    } else {
      const long long o = g * C + c;
      const long long e = cnt - a - b - d;
      if (accumulate) {
        tp[o] += a; fp[o] += b; fn[o] += d; tn[o] += e;
      } else {
        tp[o] = a; fp[o] = b; fn[o] = d; tn[o] = e;
      }
    }
    w[c] = 0;
    w[C + c] = 0;
    w[2 * C + c] = 0;
  }
  if (micro) {
    st = wave_sum_ll(st);
    sf = wave_sum_ll(sf);
    sn = wave_sum_ll(sn);
    const int wid = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    if (lane == 0) {
      red[0][wid] = st;
      red[1][wid] = sf;
      red[2][wid] = sn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      long long a = 0, b = 0, d = 0;
      for (int i = 0; i < static_cast<int>(blockDim.x / kWave); ++i) {
        a += red[0][i];
        b += red[1][i];
        d += red[2][i];
      }
      const long long e = static_cast<long long>(C) * cnt - a - b - d;
      if (accumulate) {
        tp[g] += a; fp[g] += b; fn[g] += d; tn[g] += e;
      } else {
        tp[g] = a; fp[g] = b; fn[g] = d; tn[g] = e;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) w[3 * C] = 0;
}

int pick_grid(long long work_items, int per_block) {
  return grid_cap((work_items + per_block - 1) / per_block, 256 * 8);
}

// ----------------------------------------------------------------------------------------------------------------
// binary / multilabel
// ----------------------------------------------------------------------------------------------------------------
// workspace per (group, label): [tpA, fpA, fnA, tpB, fpB, fnB, count]  (A = preds as probabilities,
// B = preds as logits -> sigmoid).  A per-call "not a probability" word decides between A and B at finalize, which
// reproduces the reference's `if not torch.all((preds >= 0) * (preds <= 1)): preds = preds.sigmoid()` without a
// host round trip.
constexpr int kBinSlots = 7;

// Reading B decides `round_to<scalar_t>(sigmoid(v)) > thr` -- a non-decreasing function of v, so it equals
// `v >= cut` for the smallest float `cut` where it holds (NaN when it never does; v = NaN is false either way).
// Every thread finds the cut once by a 32-step search over the ordered float bit patterns, with the very same
// expression; the per-element exp / reciprocal / rounding disappear from the hot loops.
__device__ __forceinline__ bool sigmoid_gt(float x, float thr_t, int kind) {
  const float s = 1.f / (1.f + __expf(-x));
  const float r = kind == 1 ? round_to<c10::BFloat16>(s) : kind == 2 ? round_to<c10::Half>(s) : s;
  return r > thr_t;
}

__device__ __forceinline__ uint32_t ordered_key(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float ordered_float(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <typename scalar_t>
__device__ __forceinline__ int round_kind() {
  return std::is_same<scalar_t, c10::BFloat16>::value ? 1 : std::is_same<scalar_t, c10::Half>::value ? 2 : 0;
}

template <typename scalar_t>
__device__ float sigmoid_cut(float thr_t) {
  const int kind = round_kind<scalar_t>();
  if (!sigmoid_gt(INFINITY, thr_t, kind)) return __uint_as_float(0x7fc00000u);  // never: NaN compares false
  if (sigmoid_gt(-INFINITY, thr_t, kind)) return -INFINITY;
  uint32_t lo = ordered_key(-INFINITY), hi = ordered_key(INFINITY);  // f(lo) false, f(hi) true
  while (hi - lo > 1) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    if (sigmoid_gt(ordered_float(mid), thr_t, kind)) hi = mid;
    else lo = mid;
  }
  return ordered_float(hi);
}

template <typename scalar_t>
__device__ __forceinline__ void bin_pred(scalar_t raw, float thr_t, float cut, int* flag, bool& pa, bool& pb,
                                         bool& valid) {
  valid = true;
  if constexpr (IsFloating<scalar_t>::value) {
    const float v = to_f32(raw);
    pa = v > thr_t;
    pb = v >= cut;
  } else {
    const long long v = static_cast<long long>(raw);
    if (v != 0 && v != 1) {
      raise_flag(flag, kErrPredsNotBinary);
      valid = false;
    }
    pa = pb = (v == 1);
  }
}

// Branch-free element step of the binary counters: six raw counts (t & pa, pa, t & pb, pb, t, valid) -- the 7 slots
// (tp / fp / fn under both probability readings + count) follow from them in bin_to_slots.  The per-element
// `continue`s of the earlier form (ignored, non-binary target / pred) made every element its own exec-masked basic
// block: ~86 instructions per element in bin_vec_kernel, VALU / SALU-bound at 2.7 TB/s.  Flag bits are collected in
// registers and raised once per wave.
struct BinAcc {
  int a = 0, p = 0, b = 0, q = 0, t = 0, n = 0;
  int not_prob = 0, bad_t = 0, bad_p = 0;
};

// kIgn: an ignore_index is set (else the compare is compiled out); kProb: check "probabilities" per element here (the
// vector kernel instead tracks a packed ordinal range, see OrdRange)
template <bool kIgn = true, bool kProb = true, typename scalar_t, typename target_t>
__device__ __forceinline__ void bin_step(BinAcc& c, scalar_t raw, target_t traw, float thr_t, float cut,
                                         long long ignore, bool has_ignore, bool prob_check_all) {
  const long long tv = static_cast<long long>(traw);
  const bool ignored = kIgn && has_ignore && tv == ignore;
  bool tbin;
  if constexpr (sizeof(target_t) <= 4)
    tbin = static_cast<uint32_t>(static_cast<int32_t>(traw)) <= 1u;  // 32-bit compare for narrow targets
  else
    tbin = static_cast<unsigned long long>(tv) <= 1ull;
  c.bad_t |= !ignored && !tbin;
  bool pa, pb, pvalid;
  if constexpr (IsFloating<scalar_t>::value) {
    const float v = to_f32(raw);
    pa = v > thr_t;
    pb = v >= cut;
    pvalid = true;
    if constexpr (kProb) c.not_prob |= !(v >= 0.f && v <= 1.f) && (prob_check_all || !ignored);
  } else {
    const long long pv = static_cast<long long>(raw);
    pvalid = static_cast<unsigned long long>(pv) <= 1ull;
    c.bad_p |= !ignored && tbin && !pvalid;
    pa = pb = pv == 1;
  }
  const int valid = !ignored && tbin && pvalid;
  int t;
  if constexpr (sizeof(target_t) <= 4)
    t = valid & (static_cast<int32_t>(traw) == 1);
  else
    t = valid & (tv == 1);
  const int ia = valid & pa, ib = valid & pb;
  c.a += t & ia;
  c.p += ia;
  c.b += t & ib;
  c.q += ib;
  c.t += t;
  c.n += valid;
}

__device__ __forceinline__ void bin_to_slots(const BinAcc& c, int (&s)[kBinSlots]) {
  s[0] = c.a;
  s[1] = c.p - c.a;
  s[2] = c.t - c.a;
  s[3] = c.b;
  s[4] = c.q - c.b;
  s[5] = c.t - c.b;
  s[6] = c.n;
}

// the flags an accumulation saw, raised once per wave (call with every lane of the wave)
__device__ __forceinline__ void bin_raise(const BinAcc& c, int* flag, int* not_prob) {
  const bool lead = (threadIdx.x & (kWave - 1)) == 0;
  if (__any(c.bad_t) && lead) raise_flag(flag, kErrTargetNotBinary);
  if (__any(c.bad_p) && lead) raise_flag(flag, kErrPredsNotBinary);
  if (not_prob != nullptr && __any(c.not_prob) && lead) atomicOr(not_prob, 1);
}

__device__ __forceinline__ void bin_slots(bool t, bool pa, bool pb, int& sa, int& sb) {
  // tp=0 fp=1 fn=2 (tn implicit); -1 = tn
  sa = t ? (pa ? 0 : 2) : (pa ? 1 : -1);
  sb = t ? (pb ? 3 : 5) : (pb ? 4 : -1);
}

// flat kernel: elements of preds [N, L, X] visited in memory order; group = samplewise ? n*L + l : l
// partials != nullptr (LDS histogram, many labels): each block stores its [L * 7] int32 histogram to its own row of
// `partials` and partials_fold_kernel folds the rows into ws -- instead of up to L * 7 global atomics per block.
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) bin_flat_kernel(const scalar_t* __restrict__ preds,
                                                          const target_t* __restrict__ target, long long total,
                                                          long long L, long long X, float thr_t, long long ignore,
                                                          bool has_ignore, bool samplewise, int64_t* __restrict__ ws,
                                                          int* __restrict__ flag, int* __restrict__ not_prob,
                                                          bool prob_check_all, int* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const long long nbins = L * kBinSlots;
  const bool use_lds = !samplewise && nbins <= kLdsBins && static_cast<long long>(gridDim.x) * blockDim.x * 4 <= total;
  if (use_lds) {
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) lds[b] = 0;
    __syncthreads();
  }
  int local_not_prob = 0;
  const float cut = IsFloating<scalar_t>::value ? sigmoid_cut<scalar_t>(thr_t) : 0.f;
  // (i / X, i % X, (i / X) % L) are advanced incrementally: no 64-bit division per element
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  const long long i_start = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long s_q = stride / X, s_r = stride % X, s_l = s_q % L;
  long long nl = i_start / X, rx = i_start % X, l = nl % L;
  for (long long i = i_start; i < total; i += stride) {
    if (i != i_start) {
      rx += s_r;
      long long carry = 0;
      if (rx >= X) {
        rx -= X;
        carry = 1;
      }
      nl += s_q + carry;
      l += s_l + carry;
      if (l >= L) l -= L;
    }
    const long long tv = static_cast<long long>(target[i]);
    bool pa, pb, valid;
    // stat scores decide logits-vs-probabilities over ALL preds (ignored positions included); the binary
    // confusion matrix decides after dropping ignored positions (reference F/classification/confusion_matrix.py)
    const bool ignored = has_ignore && tv == ignore;
    if constexpr (IsFloating<scalar_t>::value) {
      const float v = to_f32(preds[i]);
      if (!(v >= 0.f && v <= 1.f) && (prob_check_all || !ignored)) local_not_prob = 1;
    }
    if (ignored) continue;
    if (tv != 0 && tv != 1) {
      raise_flag(flag, kErrTargetNotBinary);
      continue;
    }
    bin_pred<scalar_t>(preds[i], thr_t, cut, flag, pa, pb, valid);
    if (!valid) continue;
    int sa, sb;
    bin_slots(tv == 1, pa, pb, sa, sb);
    const long long g = samplewise ? nl : l;
    if (use_lds) {
      int* h = lds + l * kBinSlots;
      if (sa >= 0) atomicAdd(h + sa, 1);
      if (sb >= 0) atomicAdd(h + sb, 1);
      atomicAdd(h + 6, 1);
    } else {
      int64_t* h = ws + g * kBinSlots;
      if (sa >= 0) atomic_add_i64(h + sa, 1);
      if (sb >= 0) atomic_add_i64(h + sb, 1);
      atomic_add_i64(h + 6, 1);
    }
  }
  if (IsFloating<scalar_t>::value) {
    if (__any(local_not_prob) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(not_prob, 1);
  }
  if (partials != nullptr && !use_lds) {  // (the launcher only passes partials when LDS is used: keep the row valid)
    int* row = partials + static_cast<long long>(blockIdx.x) * nbins;
    for (long long b = threadIdx.x; b < nbins; b += blockDim.x) row[b] = 0;
  }
  if (use_lds) {
    __syncthreads();
    if (partials != nullptr) {
      int* row = partials + static_cast<long long>(blockIdx.x) * nbins;
      for (long long b = threadIdx.x; b < nbins; b += blockDim.x) row[b] = lds[b];
    } else {
      for (long long b = threadIdx.x; b < nbins; b += blockDim.x) {
        const int v = lds[b];
        if (v) atomic_add_i64(ws + b, v);
      }
    }
  }
}

// ws[b] += sum over the blocks' partial histograms [nrows, nbins] (int32).  Grid: x = groups of 64 bins (lanes walk
// consecutive bins), y = splits of the rows; each of the block's 16 waves sums at most kFoldRows rows with all its
// loads in flight, the block reduces in LDS and adds once per bin (a plain add when there is one split).  Partials +
// this fold replace per-block global atomics onto a few shared addresses, which serialise at ~11 ns each (binary
// inputs: 2048 blocks x 7 counters).
__global__ void __launch_bounds__(kFoldThreads) partials_fold_kernel(const int* __restrict__ part, int nrows,
                                                                      int nbins, int64_t* __restrict__ ws) {
  constexpr int kW = kFoldThreads / kWave;
  __shared__ long long red[kW][kWave];  // 64-bit sums (no int32 wrap)
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int bin = blockIdx.x * kWave + lane;
  const int r0 = blockIdx.y * kW * kFoldRows + w;
  int v[kFoldRows];
#pragma unroll
  for (int i = 0; i < kFoldRows; ++i) {
    const int r = r0 + i * kW;
    v[i] = (bin < nbins && r < nrows) ? part[static_cast<long long>(r) * nbins + bin] : 0;
  }
  long long acc = 0;
#pragma unroll
  for (int i = 0; i < kFoldRows; ++i) acc += v[i];
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && bin < nbins) {
    long long tot = 0;
#pragma unroll
    for (int i = 0; i < kW; ++i) tot += red[i][lane];
    if (tot) {
      if (gridDim.y == 1) ws[bin] += tot;
      else atomic_add_i64(ws + bin, tot);
    }
  }
}

void launch_partials_fold(const int* part, int nrows, int nbins, int64_t* ws, hipStream_t s) {
  constexpr int per = kFoldThreads / kWave * kFoldRows;
  hipLaunchKernelGGL(partials_fold_kernel, dim3((nbins + kWave - 1) / kWave, (nrows + per - 1) / per),
                     dim3(kFoldThreads), 0, s, part, nrows, nbins, ws);
}

// Multilabel rows [N, L] (X == 1, L % VEC == 0, VEC = 16 / sizeof(preds)): a thread reads one 16-byte vector of VEC
// consecutive labels (and their targets) per step, and the grid stride S (in vectors) is a multiple of L / VEC, so a
// thread's VEC labels never change -- its 7 x VEC counters stay in registers for the whole walk (kU vectors in flight
// per thread).  No per-element atomics at all (bin_flat_kernel did 3 LDS atomics per element: MultilabelF1Score(1000)
// on 16384 x 1000 bf16 ran at 1.3 TB/s); the block folds its counters into an LDS histogram once and stores it as its
// row of `partials`, which partials_fold_kernel folds into the workspace.
constexpr int kVecBlock = 512;

// "Are all scores in [0, 1]?" over whole 16-byte vectors: the order-preserving ordinal of each value (sign-magnitude
// float bits u -> u ^ ((u >>a msb) | msb), NaNs land beyond +-inf) folded into a running min / max (packed 16-bit
// min / max for bf16 / fp16: 2 values per instruction).  In range iff min >= ord(-0) and max <= ord(1).  Replaces
// four compares / selects per element when every position counts (no ignore_index, or prob_check_all).
template <typename scalar_t>
struct OrdRange;
template <>
struct OrdRange<float> {
  uint32_t lo = 0xffffffffu, hi = 0u;
  __device__ __forceinline__ void add(const u32x4& v) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w = v[k];
      const uint32_t o = w ^ (static_cast<uint32_t>(static_cast<int32_t>(w) >> 31) | 0x80000000u);
      lo = o < lo ? o : lo;
      hi = o > hi ? o : hi;
    }
  }
  __device__ __forceinline__ bool ok() const { return lo >= 0x7fffffffu && hi <= 0xbf800000u; }
};
template <typename scalar_t>
struct OrdRange16 {
  u16x2 lo = {0xffff, 0xffff}, hi = {0, 0};
  __device__ __forceinline__ void add(const u32x4& v) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w = v[k];
      const s16x2 sw = __builtin_bit_cast(s16x2, w);
      const uint32_t sgn = __builtin_bit_cast(uint32_t, static_cast<s16x2>(sw >> (s16x2){15, 15}));
      const u16x2 o = __builtin_bit_cast(u16x2, w ^ (sgn | 0x80008000u));
      lo = __builtin_elementwise_min(lo, o);
      hi = __builtin_elementwise_max(hi, o);
    }
  }
  __device__ __forceinline__ bool ok() const {
    constexpr uint32_t one = std::is_same<scalar_t, c10::BFloat16>::value ? 0xbf80u : 0xbc00u;  // ord(1.0)
    const uint32_t l = lo.x < lo.y ? lo.x : lo.y, h = hi.x > hi.y ? hi.x : hi.y;
    return l >= 0x7fffu && h <= one;
  }
};
template <>
struct OrdRange<c10::BFloat16> : OrdRange16<c10::BFloat16> {};
template <>
struct OrdRange<c10::Half> : OrdRange16<c10::Half> {};

template <typename scalar_t, typename target_t, int VEC, int kU = 4>
__global__ void __launch_bounds__(kVecBlock) bin_vec_kernel(const scalar_t* __restrict__ preds,
                                                            const target_t* __restrict__ target, long long nvec,
                                                            int L, float thr_t, long long ignore, bool has_ignore,
                                                            int* __restrict__ flag, int* __restrict__ not_prob,
                                                            bool prob_check_all, int* __restrict__ partials,
                                                            int64_t* __restrict__ ws) {
  static_assert(VEC * sizeof(scalar_t) == 16, "one 16-byte vector of preds per step");
  constexpr int kTChunks = (VEC * sizeof(target_t) + 15) / 16;  // 16-byte chunks of the matching targets
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const int nbins = L * kBinSlots;
  for (int b = threadIdx.x; b < nbins; b += kVecBlock) lds[b] = 0;
  __syncthreads();
  const long long S = static_cast<long long>(gridDim.x) * kVecBlock;
  const long long v0 = static_cast<long long>(blockIdx.x) * kVecBlock + threadIdx.x;
  const int l0 = static_cast<int>((v0 * VEC) % L);
  BinAcc c[VEC];
  const float cut = sigmoid_cut<scalar_t>(thr_t);
  const u32x4* pv = reinterpret_cast<const u32x4*>(preds);
  const u32x4* tvp = reinterpret_cast<const u32x4*>(target);
  OrdRange<scalar_t> range;
  auto walk = [&](auto ign) {  // ign: std::integral_constant<bool, has_ignore> (wave-uniform, two instantiations)
    constexpr bool kIgn = decltype(ign)::value;
    for (long long base = v0; base < nvec; base += kU * S) {
      u32x4 praw[kU];
      u32x4 traw[kU][kTChunks];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const long long v = base + u * S;
        if (v < nvec) {
          praw[u] = __builtin_nontemporal_load(pv + v);
#pragma unroll
          for (int j = 0; j < kTChunks; ++j) traw[u][j] = __builtin_nontemporal_load(tvp + v * kTChunks + j);
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (base + u * S >= nvec) break;
        const scalar_t* pe = reinterpret_cast<const scalar_t*>(&praw[u]);
        const target_t* te = reinterpret_cast<const target_t*>(&traw[u][0]);
        if constexpr (!kIgn) range.add(praw[u]);  // every position counts for the probability check
#pragma unroll
        for (int e = 0; e < VEC; ++e)
          bin_step<kIgn, kIgn>(c[e], pe[e], te[e], thr_t, cut, ignore, has_ignore, prob_check_all);
      }
    }
  };
  if (has_ignore) {
    walk(std::true_type{});
  } else {
    walk(std::false_type{});
    c[0].not_prob |= !range.ok();
  }
  BinAcc any;
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    any.bad_t |= c[e].bad_t;
    any.not_prob |= c[e].not_prob;
  }
  bin_raise(any, flag, not_prob);
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    int sl[kBinSlots];
    bin_to_slots(c[e], sl);
#pragma unroll
    for (int k = 0; k < kBinSlots; ++k)
      if (sl[k]) atomicAdd(&lds[(l0 + e) * kBinSlots + k], sl[k]);
  }
  __syncthreads();
  if (partials == nullptr) {  // TM_AMD_BIN_VEC_ATOMIC: each block adds its histogram straight into ws (no fold launch)
    for (int b = threadIdx.x; b < nbins; b += kVecBlock) {
      const int v = lds[b];
      if (v) atomic_add_i64(ws + b, v);
    }
    return;
  }
  int* row = partials + static_cast<long long>(blockIdx.x) * nbins;
  for (int b = threadIdx.x; b < nbins; b += kVecBlock) row[b] = lds[b];
}

// segment kernel for long contiguous segments (X large): block = one chunk of one (n, l) segment, register
// accumulation + block reduction, 7 atomics per block.
// Binary / small multilabel (L * X <= 64, not samplewise): the grid stride is a multiple of L * X, so every thread
// always sees the SAME label -- its 7 counters (tp/fp/fn for both probability readings + count) stay in registers
// for its whole grid-stride walk (4 independent loads in flight per iteration).  At the end one LDS add per counter
// (after a wave reduction when the block has a single label), then the block stores its row of partials.
// The flat kernel instead did 2-3 LDS atomics per element onto the same 7 addresses (64-way serialised for binary
// inputs): 16.8 M fp32 binary elements 115 us -> HBM-bound.
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) bin_reg_kernel(const scalar_t* __restrict__ preds,
                                                         const target_t* __restrict__ target, long long total,
                                                         long long L, long long X, float thr_t, long long ignore,
                                                         bool has_ignore, int64_t* __restrict__ ws,
                                                         int* __restrict__ partials, int* __restrict__ flag,
                                                         int* __restrict__ not_prob, bool prob_check_all) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const int nbins = static_cast<int>(L) * kBinSlots;
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) lds[b] = 0;
  __syncthreads();
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  const long long i0 = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int label = static_cast<int>((i0 / X) % L);
  BinAcc acc;
  const float cut = IsFloating<scalar_t>::value ? sigmoid_cut<scalar_t>(thr_t) : 0.f;
  constexpr int kU = 4;
  for (long long base = i0; base < total; base += kU * stride) {
    target_t tv[kU];
    scalar_t pv[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const long long i = base + u * stride;
      if (i < total) {
        tv[u] = target[i];
        pv[u] = preds[i];
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (base + u * stride < total) bin_step(acc, pv[u], tv[u], thr_t, cut, ignore, has_ignore, prob_check_all);
  }
  bin_raise(acc, flag, IsFloating<scalar_t>::value ? not_prob : nullptr);
  int c[kBinSlots];
  bin_to_slots(acc, c);
  if (L * X == 1) {  // one label in the whole grid: reduce across the wave first
#pragma unroll
    for (int k = 0; k < kBinSlots; ++k) {
      const int v = wave_sum(c[k]);
      if ((threadIdx.x & (kWave - 1)) == 0 && v) atomicAdd(&lds[k], v);
    }
  } else {
#pragma unroll
    for (int k = 0; k < kBinSlots; ++k)
      if (c[k]) atomicAdd(&lds[label * kBinSlots + k], c[k]);
  }
  __syncthreads();
  if (partials != nullptr) {
    int* row = partials + static_cast<long long>(blockIdx.x) * nbins;  // folded by partials_fold_kernel
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) row[b] = lds[b];
  } else {  // a small grid: one global add per (label, counter) and block
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
      const int v = lds[b];
      if (v) atomic_add_i64(ws + b, v);
    }
  }
}

template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) bin_seg_kernel(const scalar_t* __restrict__ preds,
                                                         const target_t* __restrict__ target, long long nseg,
                                                         long long L, long long X, long long chunk, float thr_t,
                                                         long long ignore, bool has_ignore, bool samplewise,
                                                         int64_t* __restrict__ ws, int* __restrict__ flag,
                                                         int* __restrict__ not_prob, bool prob_check_all) {
  const long long chunks_per_seg = (X + chunk - 1) / chunk;
  const long long seg = blockIdx.x / chunks_per_seg;
  const long long cidx = blockIdx.x - seg * chunks_per_seg;
  if (seg >= nseg) return;
  const long long beg = cidx * chunk, end = min(X, beg + chunk);
  const scalar_t* p = preds + seg * X;
  const target_t* t = target + seg * X;
  long long acc[kBinSlots] = {0, 0, 0, 0, 0, 0, 0};
  int local_not_prob = 0;
  const float cut = IsFloating<scalar_t>::value ? sigmoid_cut<scalar_t>(thr_t) : 0.f;
  for (long long x = beg + threadIdx.x; x < end; x += blockDim.x) {
    const long long tv = static_cast<long long>(t[x]);
    const bool ignored = has_ignore && tv == ignore;
    if constexpr (IsFloating<scalar_t>::value) {
      const float v = to_f32(p[x]);
      if (!(v >= 0.f && v <= 1.f) && (prob_check_all || !ignored)) local_not_prob = 1;
    }
    if (ignored) continue;
    if (tv != 0 && tv != 1) {
      raise_flag(flag, kErrTargetNotBinary);
      continue;
    }
    bool pa, pb, valid;
    bin_pred<scalar_t>(p[x], thr_t, cut, flag, pa, pb, valid);
    if (!valid) continue;
    int sa, sb;
    bin_slots(tv == 1, pa, pb, sa, sb);
#pragma unroll
    for (int s = 0; s < 6; ++s) acc[s] += (s == sa) + (s == sb);
    acc[6] += 1;
  }
  if (IsFloating<scalar_t>::value) {
    if (__any(local_not_prob) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(not_prob, 1);
  }
  __shared__ long long red[kBinSlots][kBlock / kWave];
  const int wid = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int s = 0; s < kBinSlots; ++s) {
    const long long v = wave_sum_ll(acc[s]);
    if (lane == 0) red[s][wid] = v;
  }
  __syncthreads();
  if (threadIdx.x < kBinSlots) {
    long long v = 0;
    for (int w = 0; w < static_cast<int>(blockDim.x / kWave); ++w) v += red[threadIdx.x][w];
    const long long g = samplewise ? seg : seg % L;
    if (v) atomic_add_i64(ws + g * kBinSlots + threadIdx.x, v);
  }
}

// states (per group g): accumulate or write tp/fp/tn/fn; picks interpretation A/B from not_prob; zeros ws + flag.
// zero_np (single-block launch): the block also re-arms not_prob after every thread has read it -- no separate
// one-thread launch
__global__ void __launch_bounds__(kBlock) bin_finalize_kernel(int64_t* __restrict__ ws, long long G,
                                                              int* __restrict__ not_prob, bool accumulate,
                                                              int64_t* __restrict__ tp, int64_t* __restrict__ fp,
                                                              int64_t* __restrict__ tn, int64_t* __restrict__ fn,
                                                              bool zero_np, int slot, bool two_slots) {
  const bool use_b = not_prob[slot] != 0;
  if (two_slots && blockIdx.x == 0 && threadIdx.x == 0) not_prob[slot ^ 1] = 0;  // the next update's word
  for (long long g = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; g < G;
       g += static_cast<long long>(gridDim.x) * blockDim.x) {
    int64_t* w = ws + g * kBinSlots;
    const long long a = use_b ? w[3] : w[0];
    const long long b = use_b ? w[4] : w[1];
    const long long d = use_b ? w[5] : w[2];
    const long long e = w[6] - a - b - d;
    if (accumulate) {
      tp[g] += a; fp[g] += b; fn[g] += d; tn[g] += e;
    } else {
      tp[g] = a; fp[g] = b; fn[g] = d; tn[g] = e;
    }
#pragma unroll
    for (int s = 0; s < kBinSlots; ++s) w[s] = 0;
  }
  if (zero_np) {
    __syncthreads();
    if (threadIdx.x == 0) *not_prob = 0;
  }
}

// binary / multilabel confusion matrices [G, 2, 2] (rows = target, cols = pred) accumulated in place
__global__ void __launch_bounds__(kBlock) bin_confmat_finalize_kernel(int64_t* __restrict__ ws, long long G,
                                                                      int* __restrict__ not_prob,
                                                                      int64_t* __restrict__ confmat, bool zero_np,
                                                                      int slot, bool two_slots) {
  const bool use_b = not_prob[slot] != 0;
  if (two_slots && blockIdx.x == 0 && threadIdx.x == 0) not_prob[slot ^ 1] = 0;
  for (long long g = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; g < G;
       g += static_cast<long long>(gridDim.x) * blockDim.x) {
    int64_t* w = ws + g * kBinSlots;
    const long long tp = use_b ? w[3] : w[0];
    const long long fp = use_b ? w[4] : w[1];
    const long long fn = use_b ? w[5] : w[2];
    const long long tn = w[6] - tp - fp - fn;
    int64_t* c = confmat + g * 4;
    c[0] += tn;
    c[1] += fp;
    c[2] += fn;
    c[3] += tp;
#pragma unroll
    for (int s = 0; s < kBinSlots; ++s) w[s] = 0;
  }
  if (zero_np) {
    __syncthreads();
    if (threadIdx.x == 0) *not_prob = 0;
  }
}

// Fold + finalize in ONE launch for an update whose per-block label histograms are still in `partials`
// ([nrows, L * 7] int32, written by bin_vec / bin_reg / bin_flat): block = LB labels x (1024 / LB) row lanes; every
// thread sums its rows' 7 counters for its label (4 rows in flight), waves reduce lanes of the same label by shuffles,
// the block reduces the 16 waves in LDS, and one thread per label picks reading A / B from not_prob[slot] and writes
// the states (or the [L, 2, 2] confusion matrices).  Any counts already folded into ws (an earlier update not yet
// finalized) are added and ws is re-zeroed.  Replaces partials_fold_kernel + bin_*_finalize_kernel (two launches).
template <int LB>
__global__ void __launch_bounds__(kFoldThreads) bin_partials_finalize_kernel(
    const int* __restrict__ part, int nrows, int L, int64_t* __restrict__ ws, int* __restrict__ not_prob, int slot,
    bool two_slots, bool accumulate, int64_t* __restrict__ tp, int64_t* __restrict__ fp, int64_t* __restrict__ tn,
    int64_t* __restrict__ fn, int64_t* __restrict__ confmat) {
  constexpr int kRowLanes = kFoldThreads / LB;
  constexpr int kW = kFoldThreads / kWave;
  __shared__ long long red[kW][LB][kBinSlots];
  const int lb = threadIdx.x % LB, rl = threadIdx.x / LB;
  const int g = blockIdx.x * LB + lb;
  const long long nbins = static_cast<long long>(L) * kBinSlots;
  long long acc[kBinSlots] = {0, 0, 0, 0, 0, 0, 0};
  if (g < L) {
    const int* base = part + static_cast<long long>(g) * kBinSlots;
    int r = rl;
    for (; r + 3 * kRowLanes < nrows; r += 4 * kRowLanes) {
      int v[4][kBinSlots];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < kBinSlots; ++k) v[u][k] = base[static_cast<long long>(r + u * kRowLanes) * nbins + k];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < kBinSlots; ++k) acc[k] += v[u][k];
    }
    for (; r < nrows; r += kRowLanes)
#pragma unroll
      for (int k = 0; k < kBinSlots; ++k) acc[k] += base[static_cast<long long>(r) * nbins + k];
  }
  wave_colsum64(acc, LB);  // lanes of one label: DPP / permlane (VALU), not 7 x 6 x 2 ds_bpermutes
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (lane < LB)
#pragma unroll
    for (int k = 0; k < kBinSlots; ++k) red[w][lane][k] = acc[k];
  __syncthreads();
  if (threadIdx.x < LB && g < L) {
    long long c[kBinSlots];
    int64_t* wg = ws + static_cast<long long>(g) * kBinSlots;
#pragma unroll
    for (int k = 0; k < kBinSlots; ++k) {
      long long t = wg[k];
      for (int i = 0; i < kW; ++i) t += red[i][threadIdx.x][k];
      c[k] = t;
      wg[k] = 0;
    }
    const bool use_b = not_prob[slot] != 0;
    const long long a = use_b ? c[3] : c[0], b = use_b ? c[4] : c[1], d = use_b ? c[5] : c[2];
    const long long e = c[6] - a - b - d;
    if (confmat != nullptr) {
      int64_t* m = confmat + static_cast<long long>(g) * 4;
      m[0] += e;
      m[1] += b;
      m[2] += d;
      m[3] += a;
    } else if (accumulate) {
      tp[g] += a; fp[g] += b; fn[g] += d; tn[g] += e;
    } else {
      tp[g] = a; fp[g] = b; fn[g] = d; tn[g] = e;
    }
  }
  if (two_slots && blockIdx.x == 0 && threadIdx.x == 0) not_prob[slot ^ 1] = 0;
}

// reset of the per-call logit flag is ordered after the finalize (same stream) -- only for one-word flags
__global__ void zero_int_kernel(int* p) { *p = 0; }

int fewbins_tile_per_cu() {  // blocks per CU of the tiled kernel; 0 = off
  static const int v = [] {
    const char* e = std::getenv("TM_AMD_FEWBINS_TILE");
    return e ? std::atoi(e) : 3;  // measured (1 M x 10 bf16, fold path): 3 / CU 10.4 us, 2 / CU 12.0
  }();
  return v;
}

// rows per thread per tile: as many as fit 32 KiB of logits (at most kTileRows; TM_AMD_FEWBINS_R caps it)
long long fewbins_tile_rows(int C, size_t elem) {
  static const int r_cap = [] {
    const char* e = std::getenv("TM_AMD_FEWBINS_R");
    return e ? std::max(1, std::min(kTileRows, std::atoi(e))) : kTileRows;
  }();
  // (fewer rows per tile -- more blocks for a small batch -- measured slower: every block adds a histogram)
  return std::min<long long>(r_cap, (kTileChunks * 16LL) / (static_cast<long long>(C) * static_cast<long long>(elem)));
}

// short rows (<= 128 B, <= 64 classes, X == 1, 16-byte aligned logits): the tiled kernel with its C x C LDS histogram
bool fewbins_tile_fits(const void* preds, int C, size_t elem) {
  return fewbins_tile_per_cu() > 0 && C >= 2 && C <= kTileMaxC && fewbins_tile_rows(C, elem) >= 1 &&
         reinterpret_cast<uintptr_t>(preds) % 16 == 0;
}

// The tiled few-class kernel and how its blocks' histograms reach the destination (mode: kMcConfmat -> out = the
// matrix; kMcStats -> out = the stats workspace; kMcStatsDirect -> out = tp, fp_s / tn_s / fn_s = the other states):
//   * <= kFoldMinBlocks blocks: per-block atomics;
//   * C^2 <= 256: the group hand-off inside the one launch;
//   * else: partials + fewbins_fold_kernel (TM_AMD_FEWBINS_FUSED=0 forces this for the confusion matrix and the
//     workspace: the round-5 form, for A/B; kMcStatsDirect keeps the hand-off -- the fold has no state destinations).
template <typename scalar_t, typename target_t>
void fewbins_tile_launch(const scalar_t* pp, const target_t* tp, long long N, int C, long long ignore_index,
                         bool has_ignore, int mode, int64_t* outp, int64_t* fp_s, int64_t* tn_s, int64_t* fn_s,
                         int* flagp, const at::Tensor& preds, hipStream_t s) {
  const long long R = fewbins_tile_rows(C, sizeof(scalar_t));
  const long long ntiles = (N + kBlock * R - 1) / (kBlock * R);
  const int tgrid = static_cast<int>(
      std::min<long long>(ntiles, static_cast<long long>(cu_count(preds.get_device())) * fewbins_tile_per_cu()));
  static const bool fused_on = [] {
    const char* e = std::getenv("TM_AMD_FEWBINS_FUSED");
    return !e || std::atoi(e) != 0;
  }();
  static const int group_env = [] {  // measurement knob: blocks per hand-off group (0: per-block atomic flush)
    const char* e = std::getenv("TM_AMD_FEWBINS_GROUP");
    return e ? std::max(0, std::atoi(e)) : -1;
  }();
  const int ncm = C * C;
  // a few blocks (small batches) flush with atomics: neither a fold launch nor a hand-off tail pays for them
  const bool few = tgrid <= kFoldMinBlocks || group_env == 0;
  const bool handoff = !few && ncm <= kBlock && (fused_on || mode == kMcStatsDirect);
  const bool fold = !few && !handoff;
  // one round of loads in the folder (kGroupLoads rows per bin-thread, 256 / C^2 threads per bin), and at most
  // kGroupMaxBlocks ticket adds per word: the adds to one address serialise (C = 2 in ONE group of 512 blocks: 16.7 us
  // against the fold launch's 13.7)
  const int gsize = group_env > 0 ? group_env : std::min(kGroupMaxBlocks, kGroupLoads * (kBlock / std::max(ncm, 1)));
  const int ngroups = handoff ? std::min(kStreamTickets - 1, (tgrid + gsize - 1) / gsize) : 0;
  unsigned int* tickets = handoff ? stream_ticket(preds.get_device(), s) + 1 : nullptr;
  at::Tensor part;
  if (handoff || fold) part = at::empty({static_cast<long long>(tgrid) * ncm}, preds.options().dtype(at::kInt));
  int* partp = (handoff || fold) ? part.data_ptr<int>() : nullptr;
  const size_t smem = static_cast<size_t>((ncm * 4 + 15) & ~15) + kTileChunks * kBlock * 16 + 256;
  // dwords per row for the register argmax: 8 (rows <= 32 B) or 32 (<= 128 B); 8-byte scores read LDS
  const long long rbytes = static_cast<long long>(C) * sizeof(scalar_t);
  auto launch_tile = [&](auto nw_tag) {
    constexpr int NW = decltype(nw_tag)::value;
    hipLaunchKernelGGL((mc_fewbins_tile_kernel<scalar_t, target_t, NW>), dim3(tgrid), dim3(kBlock), smem, s, pp, tp,
                       N, C, static_cast<int>(R), ignore_index, has_ignore, mode, outp, partp, flagp, tickets, ngroups,
                       fp_s, tn_s, fn_s);
    if (fold)
      hipLaunchKernelGGL(fewbins_fold_kernel,
                         dim3((ncm + kWave - 1) / kWave,
                              (tgrid + kFoldThreads / kWave * kFoldRows - 1) / (kFoldThreads / kWave * kFoldRows)),
                         dim3(kFoldThreads), 0, s, partp, tgrid, C, mode, outp);
  };
  if constexpr (sizeof(scalar_t) == 2 || sizeof(scalar_t) == 4) {
    if (rbytes <= 32) launch_tile(std::integral_constant<int, 8>{});
    else launch_tile(std::integral_constant<int, 32>{});
  } else {
    launch_tile(std::integral_constant<int, 0>{});
  }
}

}  // namespace

// The "scores are not probabilities" word of the binary / multilabel path, double-buffered by update parity when the
// caller gives two words (the _StatWorkspace does): bin_update ORs into word `slot`, the finalize reads it and clears
// word `slot ^ 1` for the next update -- a multi-block finalize needs no extra one-thread launch to re-arm the word.
// The parity is kept here per word address; a one-word buffer keeps the old single-slot protocol.
namespace {
std::mutex g_np_mu;
std::unordered_map<const void*, int> g_np_slot;
}  // namespace

int notprob_begin(const at::Tensor& np) {
  if (np.numel() < 2) return 0;
  std::lock_guard<std::mutex> lock(g_np_mu);
  int& s = g_np_slot[np.data_ptr()];
  s ^= 1;
  return s;
}

int notprob_current(const at::Tensor& np) {
  if (np.numel() < 2) return 0;
  std::lock_guard<std::mutex> lock(g_np_mu);
  auto it = g_np_slot.find(np.data_ptr());
  return it == g_np_slot.end() ? 0 : it->second;
}

// The reader's view of the word pair: (slot, double-buffered).  While the stream is being captured into a hipGraph the
// host parity would be frozen into the graph, so captured work uses the one-word protocol on word 0 instead: bin_update
// zeroes both words first and the finalize re-arms word 0 after reading it, on every replay.  Eager updates around the
// graph keep their parity: the graph leaves both words zero.
NpView notprob_view(const at::Tensor& np, hipStream_t s) {
  if (np.numel() < 2 || stream_capturing(s)) return NpView{0, false};
  return NpView{notprob_current(np), true};
}

// Per-block label histograms of a binary / multilabel update whose fold is deferred to the finalize (keyed by the
// workspace address): the finalize then folds AND finalizes in one launch (bin_partials_finalize_kernel).  A second
// update on the same workspace before any finalize first folds the pending rows into ws (partials_fold_kernel).
namespace {
struct PendingFold {
  at::Tensor partials;
  at::Tensor ws;  // held: the workspace's memory cannot be freed and handed to another owner while rows are pending
  int nrows;
  int nbins;
};
std::mutex g_pf_mu;
std::unordered_map<const void*, PendingFold> g_pending;

void flush_pending(const at::Tensor& ws, hipStream_t s) {
  PendingFold pf;
  {
    std::lock_guard<std::mutex> lock(g_pf_mu);
    auto it = g_pending.find(ws.data_ptr());
    if (it == g_pending.end()) return;
    pf = std::move(it->second);
    g_pending.erase(it);
  }
  launch_partials_fold(pf.partials.data_ptr<int>(), pf.nrows, pf.nbins, ws.data_ptr<int64_t>(), s);
}

void defer_fold(const at::Tensor& ws, at::Tensor partials, int nrows, int nbins, hipStream_t s) {
  static const bool off = std::getenv("TM_AMD_FUSED_BIN_FINALIZE") &&
                          std::atoi(std::getenv("TM_AMD_FUSED_BIN_FINALIZE")) == 0;
  if (off) {
    launch_partials_fold(partials.data_ptr<int>(), nrows, nbins, ws.data_ptr<int64_t>(), s);
    return;
  }
  std::lock_guard<std::mutex> lock(g_pf_mu);
  g_pending[ws.data_ptr()] = PendingFold{std::move(partials), ws, nrows, nbins};
}

}  // namespace

// consumers of the workspace other than the two finalizers (bin_stats_forward) fold pending rows into ws first
void bin_flush_pending(const at::Tensor& ws) { flush_pending(ws, stream()); }

namespace {
// true: the pending rows of `ws` were folded and finalized into the states (or confmat) in one launch
bool finalize_pending(at::Tensor ws, at::Tensor not_prob, bool accumulate, int64_t* tp, int64_t* fp, int64_t* tn,
                      int64_t* fn, int64_t* confmat, hipStream_t s) {
  PendingFold pf;
  {
    std::lock_guard<std::mutex> lock(g_pf_mu);
    auto it = g_pending.find(ws.data_ptr());
    if (it == g_pending.end()) return false;
    pf = std::move(it->second);
    g_pending.erase(it);
  }
  const int L = pf.nbins / kBinSlots;
  const NpView nv = notprob_view(not_prob, s);
  const bool two = nv.two;
  const int slot = nv.slot;
  auto go = [&](auto lbc) {
    constexpr int LB = decltype(lbc)::value;
    hipLaunchKernelGGL((bin_partials_finalize_kernel<LB>), dim3((L + LB - 1) / LB), dim3(kFoldThreads), 0, s,
                       pf.partials.data_ptr<int>(), pf.nrows, L, ws.data_ptr<int64_t>(), not_prob.data_ptr<int>(),
                       slot, two, accumulate, tp, fp, tn, fn, confmat);
  };
  // labels per block: about 4 partial rows per thread (one batch of loads in flight), at most the label count
  int lb = 1;
  while (lb < 64 && lb * 2 * std::max(pf.nrows, 1) <= 4 * kFoldThreads) lb *= 2;
  while (lb > 1 && lb / 2 >= L) lb /= 2;
  // fewer labels per block until the grid has >= 32 blocks (TM_AMD_BIN_FOLD_MIN_BLOCKS overrides): 100 labels fold
  // on 25 blocks instead of 7 -- MultilabelAccuracy(100) 18.3-18.7 us vs 19.3-19.7 (64 / 128 blocks: no better)
  static const int min_blocks = [] {
    const char* e = std::getenv("TM_AMD_BIN_FOLD_MIN_BLOCKS");
    return e ? std::max(0, std::atoi(e)) : 32;
  }();
  while (lb > 1 && (L + lb - 1) / lb < min_blocks) lb /= 2;
  if (lb <= 1) go(std::integral_constant<int, 1>{});
  else if (lb <= 4) go(std::integral_constant<int, 4>{});
  else if (lb <= 16) go(std::integral_constant<int, 16>{});
  else go(std::integral_constant<int, 64>{});
  if (!two) hipLaunchKernelGGL(zero_int_kernel, dim3(1), dim3(1), 0, s, not_prob.data_ptr<int>());
  return true;
}
}  // namespace

// ================================================================================================================
// host launchers
// ================================================================================================================

// Multiclass update.
//   preds: float [N, C, X] (argmax) or int [N, K, X] labels
//   target: int [N, X]
//   mode 0: out = confmat [C, C] int64 (accumulated in place)
//   mode 1: out = workspace [G, 3C+1] int64 (G = N if samplewise else 1); finalize with mc_stats_finalize
void mc_update(const at::Tensor& preds, const at::Tensor& target, at::Tensor out, at::Tensor flag, int64_t num_classes,
               int64_t ignore_index, bool has_ignore, int64_t mode, bool samplewise) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, out);
  TM_SAME_DEVICE(preds, flag);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TM_CHECK_CONTIG(out);
  TORCH_CHECK(out.scalar_type() == at::kLong, "mc_update: out must be int64");
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "mc_update: flag must be int32[1]");
  const int C = static_cast<int>(num_classes);
  const bool argmax = preds.is_floating_point();
  const long long N = target.numel() == 0 ? 0 : target.size(0);
  if (N == 0) return;
  const long long X = target.numel() / N;
  TORCH_CHECK(mode == kMcConfmat || mode == kMcStats, "mc_update: bad mode");
  if (mode == kMcConfmat) {
    TORCH_CHECK(out.numel() == static_cast<long long>(C) * C, "mc_update: confmat must have C*C elements");
  } else {
    TORCH_CHECK(out.numel() == (samplewise ? N : 1) * (3LL * C + 1), "mc_update: workspace has wrong size");
  }
  long long K = 1;
  if (argmax) {
    TORCH_CHECK(preds.numel() == N * C * X, "mc_update: preds must be [N, C, ...] matching target");
  } else {
    TORCH_CHECK(preds.numel() % (N * X) == 0, "mc_update: label preds must be [N, K, ...]");
    K = preds.numel() / (N * X);
    TORCH_CHECK(K >= 1 && K <= 16, "mc_update: at most 16 predicted labels per item");
    TORCH_CHECK(mode == kMcStats || K == 1, "mc_update: confmat needs exactly one predicted label");
  }
  const int nbins = mode == kMcConfmat ? C * C : 3 * C + 1;
  const size_t lds_bytes = (!samplewise && nbins <= kLdsBins) ? nbins * sizeof(int) : 0;
  auto s = stream();
  int64_t* outp = out.data_ptr<int64_t>();
  int* flagp = flag.data_ptr<int>();
  TM_DISPATCH_TARGET(target.scalar_type(), "mc_update", [&] {
    const target_t* tp = reinterpret_cast<const target_t*>(target.data_ptr());
    TM_DISPATCH_PREDS(preds.scalar_type(), "mc_update", [&] {
      const scalar_t* pp = reinterpret_cast<const scalar_t*>(preds.data_ptr());
      if constexpr (IsFloating<scalar_t>::value) {
        const bool vec = (C * sizeof(scalar_t)) % 16 == 0 && (reinterpret_cast<uintptr_t>(pp) % 16) == 0;
        if (!samplewise && X == 1 && fewbins_tile_fits(pp, C, sizeof(scalar_t))) {
          fewbins_tile_launch(pp, tp, N, C, ignore_index, has_ignore, static_cast<int>(mode), outp, nullptr, nullptr,
                              nullptr, flagp, preds, s);
        } else if (X == 1 && C >= 32 && vec) {
          // rows of <= 16 lanes x 8 loads x 16 B go 16 lanes per row; longer rows use the whole wave per row
          const long long row_bytes = static_cast<long long>(C) * sizeof(scalar_t);
          static const int lpr_override = [] {
            const char* e = std::getenv("TM_AMD_MC_LPR");  // tuning knob: 16 / 32 / 64
            return e ? std::atoi(e) : 0;
          }();
          // measured on MI355X (8192x1000 bf16, inputs cycling through MALL): LPR 64: 12.1 us, 32: 12.4, 16: 14.3, 8: 21.0;
          // the confusion-matrix LPR-64 case goes to mc_argmax_pipe_kernel (8.7 us), TM_AMD_MC_PIPE=0 disables it
          const int lpr = lpr_override ? lpr_override : (row_bytes >= 1024 ? 64 : (row_bytes >= 512 ? 32 : 16));
          static const int pipe_override = [] {
            const char* e = std::getenv("TM_AMD_MC_PIPE");  // tuning knob: blocks per CU of the pipelined kernel
            return e ? std::atoi(e) : 8;  // measured (8192 x 1000 bf16): 1/CU 23.1 us, 2: 13.9, 4: 10.3, 8: 8.75
          }();
          const int per = static_cast<int>((row_bytes / 16 + kWave - 1) / kWave);
          // the pipelined kernels (order-key for 16-bit floats) serve both the confusion matrix and the stats workspace
          const bool pipe = pipe_override > 0 && !samplewise && per >= 1 && per <= 4 && lpr == 64;
          if (pipe) {
            const int cus = cu_count(preds.get_device());
            const long long want = (N + kBlock / kWave - 1) / (kBlock / kWave);
            const int grid = static_cast<int>(std::min<long long>(want, static_cast<long long>(cus) * pipe_override));
            static const bool ord16_off = std::getenv("TM_AMD_MC_ORD16") && std::atoi(std::getenv("TM_AMD_MC_ORD16")) == 0;
            auto launch_pipe = [&](auto per_tag) {
              constexpr int P = decltype(per_tag)::value;
              if constexpr (sizeof(scalar_t) == 2) {
                if (!ord16_off) {
                  const long long want16 = (N + kOrdBlock / kWave - 1) / (kOrdBlock / kWave);  // one row per wave
                  static const int per_cu = [] {  // blocks per CU (TM_AMD_ORD16_BLOCKS_PER_CU: measurement knob)
                    const char* e = std::getenv("TM_AMD_ORD16_BLOCKS_PER_CU");
                    return e ? std::max(1, std::atoi(e)) : 4;
                  }();
                  const int grid16 =
                      static_cast<int>(std::min<long long>(want16, static_cast<long long>(cus) * per_cu));
                  if (mode == kMcConfmat)
                    hipLaunchKernelGGL((mc_argmax_ord16_kernel<scalar_t, target_t, P, kMcConfmat>), dim3(grid16),
                                       dim3(kOrdBlock), 0, s, pp, tp, N, C, ignore_index, has_ignore, outp, flagp);
                  else
                    hipLaunchKernelGGL((mc_argmax_ord16_kernel<scalar_t, target_t, P, kMcStats>), dim3(grid16),
                                       dim3(kOrdBlock), 0, s, pp, tp, N, C, ignore_index, has_ignore, outp, flagp);
                  return;
                }
              }
              hipLaunchKernelGGL((mc_argmax_pipe_kernel<scalar_t, target_t, P>), dim3(grid), dim3(kBlock), 0, s, pp,
                                 tp, N, C, ignore_index, has_ignore, static_cast<int>(mode), outp, flagp);
            };
            if (per == 1) launch_pipe(std::integral_constant<int, 1>{});
            else if (per == 2) launch_pipe(std::integral_constant<int, 2>{});
            else if (per == 3) launch_pipe(std::integral_constant<int, 3>{});
            else launch_pipe(std::integral_constant<int, 4>{});
          } else if (lpr == 32) {
            constexpr int LPR = 32;
            const int grid = pick_grid(N, (kBlock / kWave) * (kWave / LPR));
            hipLaunchKernelGGL((mc_argmax_subwave_kernel<scalar_t, target_t, LPR>), dim3(grid), dim3(kBlock),
                               lds_bytes, s, pp, tp, N, C, ignore_index, has_ignore, static_cast<int>(mode), outp,
                               flagp, samplewise);
          } else if (lpr == 8) {
            constexpr int LPR = 8;
            const int grid = pick_grid(N, (kBlock / kWave) * (kWave / LPR));
            hipLaunchKernelGGL((mc_argmax_subwave_kernel<scalar_t, target_t, LPR>), dim3(grid), dim3(kBlock),
                               lds_bytes, s, pp, tp, N, C, ignore_index, has_ignore, static_cast<int>(mode), outp,
                               flagp, samplewise);
          } else if (lpr == 16) {
            constexpr int LPR = 16;
            const int grid = pick_grid(N, (kBlock / kWave) * (kWave / LPR));
            hipLaunchKernelGGL((mc_argmax_subwave_kernel<scalar_t, target_t, LPR>), dim3(grid), dim3(kBlock),
                               lds_bytes, s, pp, tp, N, C, ignore_index, has_ignore, static_cast<int>(mode), outp,
                               flagp, samplewise);
          } else {
            constexpr int LPR = 64;
            const int grid = pick_grid(N, kBlock / kWave);
            hipLaunchKernelGGL((mc_argmax_subwave_kernel<scalar_t, target_t, LPR>), dim3(grid), dim3(kBlock),
                               lds_bytes, s, pp, tp, N, C, ignore_index, has_ignore, static_cast<int>(mode), outp,
                               flagp, samplewise);
          }
        } else if (X == 1 && C >= 32) {
          const int waves_per_block = kBlock / kWave;
          const int grid = pick_grid(N, waves_per_block);
          hipLaunchKernelGGL((mc_argmax_rows_kernel<scalar_t, target_t>), dim3(grid), dim3(kBlock), lds_bytes, s, pp,
                             tp, N, C, ignore_index, has_ignore, static_cast<int>(mode), outp, flagp, vec, samplewise);
        } else if (!samplewise && nbins <= 256) {
          // every block flushes its <= 256 bins with global atomics onto the SAME few addresses: keep the grid to
          // ~2 blocks per CU (each thread walks several items) -- 2048 blocks serialised ~2048 atomics per bin
          const int grid = static_cast<int>(std::min<long long>(pick_grid(N * X, kBlock), 2LL * cu_count(preds.get_device())));
          static const bool stage_off = std::getenv("TM_AMD_FEWBINS_STAGE") &&
                                        std::atoi(std::getenv("TM_AMD_FEWBINS_STAGE")) == 0;  // A/B knob
          const bool stage = !stage_off && X == 1 &&
                             static_cast<long long>(kBlock) * C * sizeof(scalar_t) <= kStageBytes &&
                             reinterpret_cast<uintptr_t>(pp) % 16 == 0;
          hipLaunchKernelGGL((mc_fewbins_kernel<scalar_t, target_t, true>), dim3(grid), dim3(kBlock), 0, s, pp, tp, N,
                             X, C, ignore_index, has_ignore, static_cast<int>(mode), outp, flagp, stage);
        } else {
          const int grid = pick_grid(N * X, kBlock);
          hipLaunchKernelGGL((mc_items_kernel<scalar_t, target_t, true>), dim3(grid), dim3(kBlock), lds_bytes, s, pp,
                             tp, N, X, C, 1, ignore_index, has_ignore, static_cast<int>(mode), outp, flagp, samplewise);
        }
      } else if (!samplewise && nbins <= 256 && K == 1) {
        const int grid = static_cast<int>(std::min<long long>(pick_grid(N * X, kBlock), 2LL * cu_count(preds.get_device())));
        hipLaunchKernelGGL((mc_fewbins_kernel<scalar_t, target_t, false>), dim3(grid), dim3(kBlock), 0, s, pp, tp, N,
                           X, C, ignore_index, has_ignore, static_cast<int>(mode), outp, flagp, false);
      } else {
        const int grid = pick_grid(N * X, kBlock);
        hipLaunchKernelGGL((mc_items_kernel<scalar_t, target_t, false>), dim3(grid), dim3(kBlock), lds_bytes, s, pp,
                           tp, N, X, C, static_cast<int>(K), ignore_index, has_ignore, static_cast<int>(mode), outp,
                           flagp, samplewise);
      }
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// MulticlassStatScores-family update (top_k = 1, global, per-class states, no ignore_index) on 16-bit logits with
// rows of >= 1 KiB (the order-key kernel's shape): ONE launch straight into the int64 states, instead of the
// workspace pass + mc_finalize_kernel.  Per valid row: tp[t] or (fp[argmax], fn[t]); tn[c] += N for every class (block
// 0) and -1 for the row's target and predicted classes -- tn = rows - tp - fp - fn per class without a count.  A
// target out of range raises the flag (compute() raises) and its row is skipped.  Returns false, doing nothing,
// anywhere else (the caller takes mc_update + mc_stats_finalize).
bool mc_stats_direct(const at::Tensor& preds, const at::Tensor& target, at::Tensor tp, at::Tensor fp, at::Tensor tn,
                     at::Tensor fn, at::Tensor flag, int64_t num_classes) {
  const long long C = num_classes;
  if (!preds.is_cuda() || preds.dim() != 2 || target.dim() != 1 || preds.size(1) != C || preds.size(0) != target.size(0))
    return false;
  const bool f32 = preds.scalar_type() == at::kFloat;
  if (preds.scalar_type() != at::kBFloat16 && preds.scalar_type() != at::kHalf && !f32) return false;
  if (target.scalar_type() != at::kLong && target.scalar_type() != at::kInt) return false;
  if (!preds.is_contiguous() || !target.is_contiguous() || reinterpret_cast<uintptr_t>(preds.data_ptr()) % 16 != 0)
    return false;
  for (const at::Tensor* t : {&tp, &fp, &tn, &fn})
    if (!t->is_cuda() || t->get_device() != preds.get_device() || t->scalar_type() != at::kLong ||
        !t->is_contiguous() || t->numel() != C)
      return false;
  static const bool off = std::getenv("TM_AMD_MC_STATS_DIRECT") && std::atoi(std::getenv("TM_AMD_MC_STATS_DIRECT")) == 0;
  if (off) return false;
  // few classes (C <= 16): the tiled kernel, its group hand-off flushing straight into the states
  if (C * C <= kBlock && fewbins_tile_fits(preds.data_ptr(), static_cast<int>(C), preds.element_size())) {
    const long long N = preds.size(0);
    if (N == 0) return true;
    auto s = stream();
    TM_DISPATCH_TARGET(target.scalar_type(), "mc_stats_direct", [&] {
      const target_t* tg = reinterpret_cast<const target_t*>(target.data_ptr());
      auto go = [&](auto scalar_tag) {
        using scalar_t = decltype(scalar_tag);
        fewbins_tile_launch(reinterpret_cast<const scalar_t*>(preds.data_ptr()), tg, N, static_cast<int>(C), 0LL,
                            false, kMcStatsDirect, tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(),
                            tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(), flag.data_ptr<int>(), preds, s);
      };
      if (preds.scalar_type() == at::kBFloat16) go(c10::BFloat16{});
      else if (preds.scalar_type() == at::kHalf) go(c10::Half{});
      else go(float{});
    });
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return true;
  }
  if (f32) return false;
  const long long row_bytes = C * 2;
  if (row_bytes % 16 != 0 || row_bytes < 1024 || row_bytes > 4 * 1024) return false;
  const long long N = preds.size(0);
  if (N == 0) return true;
  auto s = stream();
  const int cus = cu_count(preds.get_device());
  const long long want16 = (N + kOrdBlock / kWave - 1) / (kOrdBlock / kWave);
  const int grid16 = static_cast<int>(std::min<long long>(want16, static_cast<long long>(cus) * 4));
  const int per = static_cast<int>((row_bytes / 16 + kWave - 1) / kWave);
  TM_DISPATCH_TARGET(target.scalar_type(), "mc_stats_direct", [&] {
    const target_t* tg = reinterpret_cast<const target_t*>(target.data_ptr());
    auto go = [&](auto scalar_tag, auto per_tag) {
      using scalar_t = decltype(scalar_tag);
      constexpr int P = decltype(per_tag)::value;
      hipLaunchKernelGGL((mc_argmax_ord16_kernel<scalar_t, target_t, P, kMcStatsDirect>), dim3(grid16),
                         dim3(kOrdBlock), 0, s, reinterpret_cast<const scalar_t*>(preds.data_ptr()), tg, N,
                         static_cast<int>(C), 0LL, false, tp.data_ptr<int64_t>(), flag.data_ptr<int>(),
                         fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(), N);
    };
    auto by_per = [&](auto scalar_tag) {
      if (per == 1) go(scalar_tag, std::integral_constant<int, 1>{});
      else if (per == 2) go(scalar_tag, std::integral_constant<int, 2>{});
      else if (per == 3) go(scalar_tag, std::integral_constant<int, 3>{});
      else go(scalar_tag, std::integral_constant<int, 4>{});
    };
    if (preds.scalar_type() == at::kBFloat16) by_per(c10::BFloat16{});
    else by_per(c10::Half{});
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return true;
}

void mc_stats_finalize(at::Tensor ws, int64_t num_classes, bool micro, bool accumulate, at::Tensor tp, at::Tensor fp,
                       at::Tensor tn, at::Tensor fn) {
  TM_CHECK_CUDA(ws);
  const int C = static_cast<int>(num_classes);
  const long long G = ws.numel() / (3LL * C + 1);
  for (auto* t : {&tp, &fp, &tn, &fn}) {
    TM_SAME_DEVICE(ws, (*t));
    TORCH_CHECK(t->scalar_type() == at::kLong && t->is_contiguous(), "mc_stats_finalize: states must be int64");
    TORCH_CHECK(t->numel() == (micro ? G : G * C), "mc_stats_finalize: state size mismatch");
  }
  // one block per group; a single large group (the usual global stats, C in the hundreds or more) gets 1024 threads so
  // both passes over the classes are one strided step per thread instead of a chain of dependent loads
  if (G <= 8 && C >= 512)
    hipLaunchKernelGGL(mc_finalize_kernel<1024>, dim3(G), dim3(1024), 0, stream(), ws.data_ptr<int64_t>(), C, micro,
                       accumulate, tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(),
                       fn.data_ptr<int64_t>());
  else
    hipLaunchKernelGGL(mc_finalize_kernel<kBlock>, dim3(G), dim3(kBlock), 0, stream(), ws.data_ptr<int64_t>(), C,
                       micro, accumulate, tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(),
                       fn.data_ptr<int64_t>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// Binary / multilabel update. preds, target: [N, L, X] (same numel). ws: [G, 7] int64 with G = N*L (samplewise)
// or L.  not_prob: int32[1] per-call flag (zeroed by finalize).
// Grid for bin_reg_kernel: its stride (grid x kBlock) must be a multiple of P = L * X (<= 64: binary inputs and
// small label sets).  0 = not applicable (the flat kernel is used).  Larger label sets were measured slower on this
// scheme (one block per CU: latency-bound; many blocks: the per-block flush dominates), so they keep the flat kernel.
long long reg_grid(long long P, long long total) {
  if (P > kWave) return 0;
  long long a = kBlock, b = P;
  while (b) {
    const long long r = a % b;
    a = b;
    b = r;
  }
  const long long q = P / a;  // grid must be a multiple of q
  const long long grid = pick_grid(total, kBlock * 16);
  return (grid + q - 1) / q * q;
}

// Grid of bin_vec_kernel, or 0 where it does not apply: [N, L] floating rows (X == 1) of > 64 labels, L a multiple of
// VEC, 16-byte aligned preds / targets, the per-block histogram in LDS; the grid (~1 block of 8 waves per CU) is a
// multiple of q = (L / VEC) / gcd(kVecBlock, L / VEC), so the stride keeps every thread on its labels.
template <typename scalar_t>
long long vec_grid(const at::Tensor& preds, const at::Tensor& target, long long L, long long X, bool samplewise,
                   long long total, int cus) {
  if constexpr (!IsFloating<scalar_t>::value || sizeof(scalar_t) > 4) {
    return 0;
  } else {
    constexpr long long VEC = 16 / sizeof(scalar_t);
    static const bool off = std::getenv("TM_AMD_BIN_VEC") && std::atoi(std::getenv("TM_AMD_BIN_VEC")) == 0;
    if (off || samplewise || X != 1 || L <= kWave || L % VEC != 0 || L * kBinSlots > kLdsBins) return 0;
    const auto tsz = target.element_size();
    if (tsz != 4 && tsz != 8) return 0;
    if (reinterpret_cast<uintptr_t>(preds.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(target.data_ptr()) % 16)
      return 0;
    long long m = L / VEC, a = kVecBlock, b = m;
    while (b) {
      const long long r = a % b;
      a = b;
      b = r;
    }
    const long long q = m / a;
    static const int mult = [] {  // blocks per CU (TM_AMD_BIN_VEC_BLOCKS_PER_CU, measurement knob; default 1)
      const char* e = std::getenv("TM_AMD_BIN_VEC_BLOCKS_PER_CU");
      return e ? std::max(1, std::atoi(e)) : 1;
    }();
    const long long want =
        std::max<long long>(1, std::min<long long>(cus * mult, (total / VEC + kVecBlock - 1) / kVecBlock));
    const long long grid = std::max<long long>(1, (want + q / 2) / q) * q;
    return grid > 4096 ? 0 : grid;
  }
}

void bin_update(const at::Tensor& preds, const at::Tensor& target, at::Tensor ws, at::Tensor flag, at::Tensor not_prob,
                int64_t num_labels, double threshold, int64_t ignore_index, bool has_ignore, bool samplewise,
                bool prob_check_all) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, ws);
  TM_SAME_DEVICE(preds, flag);
  TM_SAME_DEVICE(preds, not_prob);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.numel() == target.numel(), "bin_update: preds/target numel mismatch");
  const long long total = preds.numel();
  if (total == 0) return;
  const long long N = preds.size(0);
  const long long L = num_labels;
  TORCH_CHECK(total % (N * L) == 0, "bin_update: shape must be [N, L, ...]");
  const long long X = total / (N * L);
  const long long G = samplewise ? N * L : L;
  TORCH_CHECK(ws.numel() == G * kBinSlots && ws.scalar_type() == at::kLong, "bin_update: bad workspace");
  auto s = stream();
  flush_pending(ws, s);  // an earlier update of this workspace not finalized yet: fold its rows into ws first
  const bool captured = not_prob.numel() >= 2 && stream_capturing(s);
  if (captured) launch_zero_words(not_prob.data_ptr<int>(), 2, s);  // one-word protocol inside a graph
  // this update's "not probabilities" word
  int* const npw = not_prob.data_ptr<int>() + (captured ? 0 : notprob_begin(not_prob));
  TM_DISPATCH_TARGET(target.scalar_type(), "bin_update", [&] {
    const target_t* tp = reinterpret_cast<const target_t*>(target.data_ptr());
    TM_DISPATCH_PREDS(preds.scalar_type(), "bin_update", [&] {
      const scalar_t* pp = reinterpret_cast<const scalar_t*>(preds.data_ptr());
      float thr_t = static_cast<float>(threshold);
      if constexpr (std::is_same<scalar_t, c10::BFloat16>::value) thr_t = static_cast<float>(c10::BFloat16(thr_t));
      if constexpr (std::is_same<scalar_t, c10::Half>::value) thr_t = static_cast<float>(c10::Half(thr_t));
      if (X >= 1024) {
        const long long chunk = 16384;
        const long long nseg = N * L;
        const long long blocks = nseg * ((X + chunk - 1) / chunk);
        TORCH_CHECK(blocks < (1LL << 31), "bin_update: too many segments");
        hipLaunchKernelGGL((bin_seg_kernel<scalar_t, target_t>), dim3(blocks), dim3(kBlock), 0, s, pp, tp, nseg, L, X,
                           chunk, thr_t, ignore_index, has_ignore, samplewise, ws.data_ptr<int64_t>(),
                           flag.data_ptr<int>(), npw, prob_check_all);
      } else if (vec_grid<scalar_t>(preds, target, L, X, samplewise, total, cu_count(preds.get_device())) > 0) {
        constexpr int VEC = 16 / sizeof(scalar_t);
        const int grid = static_cast<int>(vec_grid<scalar_t>(preds, target, L, X, samplewise, total,
                                                             cu_count(preds.get_device())));
        const long long nbins = L * kBinSlots;
        // measurement knob, off by default: block histograms by int64 atomics into ws (no fold launch) measured
        // 19.1 vs 19.2 us for MultilabelAccuracy(100) and 39.1 vs 33.2 us for MultilabelF1Score(1000)
        static const bool atomic_flush = [] {
          const char* e = std::getenv("TM_AMD_BIN_VEC_ATOMIC");
          return e && std::atoi(e) != 0;
        }();
        at::Tensor partials;
        if (!atomic_flush) partials = at::empty({static_cast<long long>(grid) * nbins}, ws.options().dtype(at::kInt));
        if constexpr (VEC * sizeof(scalar_t) == 16 && IsFloating<scalar_t>::value && sizeof(scalar_t) <= 4) {
          // vectors in flight per thread (TM_AMD_BIN_VEC_U: 4 or 8, measurement knob; 8 measured 19.5-19.6 vs
          // 19.3-19.5 us at MultilabelAccuracy(100), 33.9-34.0 vs 33.3 us at MultilabelF1Score(1000): 4 stays)
          static const int unroll = [] {
            const char* e = std::getenv("TM_AMD_BIN_VEC_U");
            return e && std::atoi(e) == 8 ? 8 : 4;
          }();
          auto vec_kernel = unroll == 8 ? bin_vec_kernel<scalar_t, target_t, VEC, 8>
                                        : bin_vec_kernel<scalar_t, target_t, VEC, 4>;
          hipLaunchKernelGGL(vec_kernel, dim3(grid), dim3(kVecBlock),
                             nbins * sizeof(int), s, pp, tp, total / VEC, static_cast<int>(L), thr_t, ignore_index,
                             has_ignore, flag.data_ptr<int>(), npw, prob_check_all,
                             atomic_flush ? nullptr : partials.data_ptr<int>(), ws.data_ptr<int64_t>());
        }
        if (!atomic_flush) defer_fold(ws, partials, grid, static_cast<int>(nbins), s);
      } else if (!samplewise && reg_grid(L * X, total) > 0 && L * kBinSlots <= kLdsBins) {
        // grid stride a multiple of L * X: a fixed label per thread (register counters)
        const long long grid = reg_grid(L * X, total);
        const long long nbins = L * kBinSlots;
        const size_t lds = nbins * sizeof(int);
        const bool fold = grid > kFoldMinBlocks;
        at::Tensor partials;
        if (fold) partials = at::empty({grid * nbins}, ws.options().dtype(at::kInt));
        hipLaunchKernelGGL((bin_reg_kernel<scalar_t, target_t>), dim3(static_cast<unsigned>(grid)), dim3(kBlock), lds,
                           s, pp, tp, total, L, X, thr_t, ignore_index, has_ignore, ws.data_ptr<int64_t>(),
                           fold ? partials.data_ptr<int>() : nullptr, flag.data_ptr<int>(), npw,
                           prob_check_all);
        if (fold) defer_fold(ws, partials, static_cast<int>(grid), static_cast<int>(nbins), s);
      } else {
        const long long nbins = L * kBinSlots;
        const bool lds_hist = !samplewise && nbins <= kLdsBins;
        const size_t lds_bytes = lds_hist ? nbins * sizeof(int) : 0;
        const int grid = pick_grid(total, kBlock * 4);
        // many labels: per-block histograms go through a partials buffer instead of L * 7 atomics per block
        // (the kernel itself only uses LDS when every thread sees >= 4 elements)
        const bool use_partials = lds_hist && nbins > 64 && static_cast<long long>(grid) * kBlock * 4 <= total;
        at::Tensor partials;
        if (use_partials) partials = at::empty({static_cast<long long>(grid) * nbins}, ws.options().dtype(at::kInt));
        hipLaunchKernelGGL((bin_flat_kernel<scalar_t, target_t>), dim3(grid), dim3(kBlock), lds_bytes, s, pp, tp,
                           total, L, X, thr_t, ignore_index, has_ignore, samplewise, ws.data_ptr<int64_t>(),
                           flag.data_ptr<int>(), npw, prob_check_all,
                           use_partials ? partials.data_ptr<int>() : nullptr);
        if (use_partials) defer_fold(ws, partials, grid, static_cast<int>(nbins), s);
      }
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

void bin_stats_finalize(at::Tensor ws, at::Tensor not_prob, bool accumulate, at::Tensor tp, at::Tensor fp,
                        at::Tensor tn, at::Tensor fn) {
  TM_CHECK_CUDA(ws);
  TM_SAME_DEVICE(ws, not_prob);
  const long long G = ws.numel() / kBinSlots;
  for (auto* t : {&tp, &fp, &tn, &fn})
    TORCH_CHECK(t->device() == ws.device() && t->scalar_type() == at::kLong && t->is_contiguous() && t->numel() == G,
                "bin_stats_finalize: states must be contiguous int64 with G elements");
  auto s = stream();
  if (finalize_pending(ws, not_prob, accumulate, tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(),
                       tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(), nullptr, s)) {
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return;
  }
  const NpView nv = notprob_view(not_prob, s);
  const bool two = nv.two;                  // double-buffered word: no re-arm launch
  const bool one = G <= kFinalizeOneBlock;  // one block folds and re-arms not_prob itself
  hipLaunchKernelGGL(bin_finalize_kernel, dim3(one ? 1 : grid_cap((G + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     ws.data_ptr<int64_t>(), G, not_prob.data_ptr<int>(), accumulate, tp.data_ptr<int64_t>(),
                     fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(), one && !two, nv.slot, two);
  if (!one && !two) hipLaunchKernelGGL(zero_int_kernel, dim3(1), dim3(1), 0, s, not_prob.data_ptr<int>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

void bin_confmat_finalize(at::Tensor ws, at::Tensor not_prob, at::Tensor confmat) {
  TM_CHECK_CUDA(ws);
  TM_SAME_DEVICE(ws, not_prob);
  TM_SAME_DEVICE(ws, confmat);
  const long long G = ws.numel() / kBinSlots;
  TORCH_CHECK(confmat.scalar_type() == at::kLong && confmat.is_contiguous() && confmat.numel() == 4 * G,
              "bin_confmat_finalize: confmat must be contiguous int64 [G, 2, 2]");
  auto s = stream();
  if (finalize_pending(ws, not_prob, false, nullptr, nullptr, nullptr, nullptr, confmat.data_ptr<int64_t>(), s)) {
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return;
  }
  const bool one = G <= kFinalizeOneBlock;
  const NpView nv = notprob_view(not_prob, s);
  const bool two = nv.two;
  hipLaunchKernelGGL(bin_confmat_finalize_kernel, dim3(one ? 1 : grid_cap((G + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     s, ws.data_ptr<int64_t>(), G, not_prob.data_ptr<int>(), confmat.data_ptr<int64_t>(),
                     one && !two, nv.slot, two);
  if (!one && !two) hipLaunchKernelGGL(zero_int_kernel, dim3(1), dim3(1), 0, s, not_prob.data_ptr<int>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// forward() of the confusion matrix on 16-bit logits: ONE pass of the order-key argmax kernel adds every row into the
// zeroed batch matrix AND the global state (no separate update + add of two C x C matrices).  Returns false, doing
// nothing, where the order-key kernel is not the one mc_update would pick (the caller takes update + add).
bool mc_confmat_dual(const at::Tensor& preds, const at::Tensor& target, at::Tensor batch, at::Tensor global,
                     at::Tensor flag, int64_t num_classes, int64_t ignore_index, bool has_ignore) {
  const long long C = num_classes;
  if (!preds.is_cuda() || preds.dim() != 2 || target.dim() != 1 || preds.size(1) != C || preds.size(0) != target.size(0))
    return false;
  if (preds.scalar_type() != at::kBFloat16 && preds.scalar_type() != at::kHalf) return false;
  if (target.scalar_type() != at::kLong && target.scalar_type() != at::kInt) return false;
  if (!preds.is_contiguous() || !target.is_contiguous() || reinterpret_cast<uintptr_t>(preds.data_ptr()) % 16 != 0)
    return false;
  const long long row_bytes = C * 2;
  if (row_bytes % 16 != 0 || row_bytes < 1024) return false;  // the LPR-64 rows of the order-key kernel
  const int per = static_cast<int>((row_bytes / 16 + kWave - 1) / kWave);
  if (per < 1 || per > 4 || std::getenv("TM_AMD_MC_ORD16") || std::getenv("TM_AMD_MC_PIPE") || std::getenv("TM_AMD_MC_LPR"))
    return false;
  for (const at::Tensor* m : {&batch, &global})
    TORCH_CHECK(m->is_cuda() && m->get_device() == preds.get_device() && m->scalar_type() == at::kLong &&
                    m->is_contiguous() && m->numel() == C * C,
                "mc_confmat_dual: matrices must be contiguous int64 [C, C] on the logits' device");
  TORCH_CHECK(flag.is_cuda() && flag.scalar_type() == at::kInt && flag.get_device() == preds.get_device(),
              "mc_confmat_dual: bad flag");
  TM_SAME_DEVICE(preds, target);
  const long long N = preds.size(0);
  if (N == 0) return true;
  const int cus = cu_count(preds.get_device());
  const long long want16 = (N + kOrdBlock / kWave - 1) / (kOrdBlock / kWave);
  const int grid16 = static_cast<int>(std::min<long long>(want16, static_cast<long long>(cus) * 4));
  auto s = stream();
  TM_DISPATCH_TARGET(target.scalar_type(), "mc_confmat_dual", [&] {
    const target_t* tp = reinterpret_cast<const target_t*>(target.data_ptr());
    auto go = [&](auto* pp, auto per_tag) {
      using scalar_t = std::remove_const_t<std::remove_pointer_t<decltype(pp)>>;
      constexpr int P = decltype(per_tag)::value;
      hipLaunchKernelGGL((mc_argmax_ord16_kernel<scalar_t, target_t, P, kMcConfmatDual>), dim3(grid16),
                         dim3(kOrdBlock), 0, s, pp, tp, N, static_cast<int>(C), ignore_index, has_ignore,
                         batch.data_ptr<int64_t>(), flag.data_ptr<int>(), global.data_ptr<int64_t>());
    };
    auto by_per = [&](auto* pp) {
      if (per == 1) go(pp, std::integral_constant<int, 1>{});
      else if (per == 2) go(pp, std::integral_constant<int, 2>{});
      else if (per == 3) go(pp, std::integral_constant<int, 3>{});
      else go(pp, std::integral_constant<int, 4>{});
    };
    if (preds.scalar_type() == at::kBFloat16) by_per(reinterpret_cast<const c10::BFloat16*>(preds.data_ptr()));
    else by_per(reinterpret_cast<const c10::Half*>(preds.data_ptr()));
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return true;
}

__global__ void launch_probe_kernel(int* __restrict__ flag) {
  if (threadIdx.x == 1000) flag[0] = 0;  // never taken: an empty dispatch with one real argument
}

// Host-cost probe: one empty kernel launch on the current stream (benchmarks/host_overhead.py).
void launch_probe(at::Tensor flag) {
  TM_CHECK_CUDA(flag);
  hipLaunchKernelGGL(launch_probe_kernel, dim3(1), dim3(64), 0, stream(), flag.data_ptr<int>());
}

__global__ void sigmoid_cut_probe_kernel(const float* __restrict__ x, long long n, float thr_t, int kind,
                                         int* __restrict__ out) {
  const float cut = kind == 1 ? sigmoid_cut<c10::BFloat16>(thr_t)
                    : kind == 2 ? sigmoid_cut<c10::Half>(thr_t) : sigmoid_cut<float>(thr_t);
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    out[i] = (sigmoid_gt(x[i], thr_t, kind) ? 1 : 0) | (x[i] >= cut ? 2 : 0);
}

// Test probe of the reading-B cut: per value, bit 0 = the direct `round(sigmoid(x)) > thr`, bit 1 = `x >= cut`.
// kind 0 fp32, 1 bf16, 2 fp16 rounding of the sigmoid (the threshold is rounded as bin_update rounds it).
at::Tensor sigmoid_cut_probe(const at::Tensor& x, double threshold, int64_t kind) {
  TM_CHECK_CUDA(x);
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous(), "sigmoid_cut_probe: contiguous fp32 values");
  float thr_t = static_cast<float>(threshold);
  if (kind == 1) thr_t = static_cast<float>(c10::BFloat16(thr_t));
  if (kind == 2) thr_t = static_cast<float>(c10::Half(thr_t));
  at::Tensor out = at::empty({x.numel()}, x.options().dtype(at::kInt));
  if (x.numel())
    hipLaunchKernelGGL(sigmoid_cut_probe_kernel, dim3(grid_cap((x.numel() + 255) / 256, 1024)), dim3(256), 0,
                       stream(), x.data_ptr<float>(), static_cast<long long>(x.numel()), thr_t,
                       static_cast<int>(kind), out.data_ptr<int>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("sigmoid_cut_probe(Tensor x, float threshold, int kind) -> Tensor");
  m.def("bin_flush_pending(Tensor(a!) ws) -> ()");
  m.def(
      "mc_update(Tensor preds, Tensor target, Tensor(a!) out, Tensor(b!) flag, int num_classes, int ignore_index, "
      "bool has_ignore, int mode, bool samplewise) -> ()");
  m.def(
      "mc_stats_finalize(Tensor(a!) ws, int num_classes, bool micro, bool accumulate, Tensor(b!) tp, Tensor(c!) fp, "
      "Tensor(d!) tn, Tensor(e!) fn) -> ()");
  m.def(
      "bin_update(Tensor preds, Tensor target, Tensor(a!) ws, Tensor(b!) flag, Tensor(c!) not_prob, int num_labels, "
      "float threshold, int ignore_index, bool has_ignore, bool samplewise, bool prob_check_all) -> ()");
  m.def("bin_confmat_finalize(Tensor(a!) ws, Tensor(b!) not_prob, Tensor(c!) confmat) -> ()");
  m.def(
      "bin_stats_finalize(Tensor(a!) ws, Tensor(b!) not_prob, bool accumulate, Tensor(c!) tp, Tensor(d!) fp, "
      "Tensor(e!) tn, Tensor(f!) fn) -> ()");
}

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("mc_update", &tm_amd::mc_update);
  m.impl("mc_stats_finalize", &tm_amd::mc_stats_finalize);
  m.impl("bin_update", &tm_amd::bin_update);
  m.impl("bin_stats_finalize", &tm_amd::bin_stats_finalize);
  m.impl("bin_confmat_finalize", &tm_amd::bin_confmat_finalize);
  m.impl("sigmoid_cut_probe", &tm_amd::sigmoid_cut_probe);
  m.impl("bin_flush_pending", &tm_amd::bin_flush_pending);
}
