// One fused update for a MetricCollection's few-class multiclass members on the same (logits, target) batch.
//
// Reference: S/collections.py:200-226 updates every compute group's leader separately, and each leader re-reads the
// batch: the stat-score family (F/classification/stat_scores.py:405-419: argmax + bincount), the confusion-matrix
// family (F/classification/confusion_matrix.py:333-337), the binned PR-curve family (F/classification/
// precision_recall_curve.py:482-527: softmax-if-needed + per-threshold confmats) and the calibration error
// (F/classification/calibration_error.py:29-59: softmax-if-needed, top-1 confidence / correctness).  On the
// [8192, 10] bf16 batches of config #5 that was ~10 launches per step, every one latency-bound.
//
// Here the batch is read ONCE by `family_rows_g_kernel` (G lanes per row, a lane per class; C <= 64; the first
// version, `family_rows_kernel`, ran one row per thread -- 25 us for 8192 x 10 with a curve member, serial per-class
// threshold searches at one wave per SIMD): it computes the row's argmax,
// its softmax (rounded to the input dtype, as torch.softmax stores it), the "score outside [0, 1]" bit, and feeds a
// per-block LDS image of everything the members need:
//   * the C x C (target, argmax) histogram          -> confusion matrices, and tp / fp / tn / fn of the stat scores;
//   * per-class threshold-bucket histograms, for the raw scores AND for the softmax (the batch-wide softmax decision
//     is only known when every block is done) -> the [T, C, 2, 2] binned-curve state;
//   * top-1 (confidence, correct) candidates of both variants per row -> the calibration error's list states.
// Each block adds its (non-zero) image words into one batch image in global memory (integer atomics: exact) and ORs
// its outside bit into the batch's decision word; `family_fold_kernel` (one launch, blocks by role) reads the batch
// image once, adds it into every member's state, selects the calibration outputs and bins the kept variant into the
// metric's (count, Σconf, Σacc) cache (float atomics, arrival order), publishes the target-range bit into every
// member's validation word, and re-zeroes the image for the next update (the decision word is double-buffered by
// update parity).  Two launches per step for the whole classification group, whatever the number of members.
#include "common/tm_common.h"

#include <utility>

namespace tm_amd {
namespace {

constexpr int kFamThreads = 256;      // fold kernel
constexpr int kFamRowThreads = 1024;  // rows kernel: 16 waves per block -- config #5's 8192 rows are ONE block step on
                                      // 128 blocks (256-thread blocks ran 4 dependent steps per wave: 20.4 us vs ...)
constexpr int kFamMaxC = 64;
constexpr int kFamMaxCons = 4;   // confusion-matrix / stat-score consumers per launch
constexpr int kFamMaxErr = 12;   // validation words (4 + 4 consumers, a curve and a calibration member)
constexpr int kFoldCols = kFamThreads / kWave;  // curve columns per fold block (one wave each)
constexpr int kFoldMaxBins = 512;               // calibration bins binned in a fold block's LDS (more: global atomics)

struct FamilySpec {
  int C;
  int n_cm;
  int64_t* cm[kFamMaxCons];                // [C, C] += batch
  int n_st;
  int64_t* st[kFamMaxCons][4];             // tp, fp, tn, fn: [C] (or [1] when micro) +=
  int st_micro[kFamMaxCons];
  int T;                                   // thresholds of the curve member (0: none)
  const double* thr;                       // [T] ascending
  const int64_t* perm;                     // caller index of each sorted threshold
  int64_t* curve;                          // [T, C, 2, 2]
  int nb;                                  // calibration bin bounds (0: no calibration member)
  const float* bounds;                     // [nb] ascending
  float* conf;                             // [N] outputs (list-state elements)
  float* acc;
  float* bins;                             // [nb, 3] cache or nullptr
  int n_err;
  int* err[kFamMaxErr];
  // scratch (zero on entry, re-zeroed by the fold)
  int* img;                                // batch image: [C*C cm][2][T+1][C][2] curve]
  int* outside;                            // [2] decision words, by update parity
  int slot;
  float4* cand;                            // [N]
  int* err_scratch;
  int part_words, off_cv, off_cb;
  int need_cm;
  int abl;  // profiling ablation (TM_AMD_FAMILY_ABLATE, default 0: results are WRONG when set): 1 no threshold
            // searches, 8 no class-ordered softmax sums, 16 no curve histogram at all, 32 binary threshold search even
            // on an even grid
};

__device__ __forceinline__ int bucket_of(const double* __restrict__ thr, int t, double p) {
  int lo = 0, hi = t;  // number of thresholds <= p (NaN -> 0)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (thr[mid] <= p) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Thresholds near an even grid (torch.linspace: the usual binned-curve argument): guess the count from the grid, then
// step to the exact count -- one or two LDS reads instead of a log2(T)-deep chain of dependent ones.  Exact for any
// sorted thresholds (the steps correct any guess); the grid only makes it short.
__device__ __forceinline__ int bucket_guess(const double* __restrict__ thr, int t, double p, double t0, double inv) {
  if (!(p == p)) return 0;  // NaN: no threshold is <= p
  const double g = (p - t0) * inv + 1.0;
  int b = g <= 0.0 ? 0 : (g >= static_cast<double>(t) ? t : static_cast<int>(g));
  while (b < t && thr[b] <= p) ++b;
  while (b > 0 && thr[b - 1] > p) --b;
  return b;
}

// ---- VALU (DPP) group exchanges for G <= 16 lanes per row: a row group never straddles a 16-lane DPP row.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(dpp_i32<CTRL>(__float_as_int(x)));
}

// a butterfly partner at distance 1, 2, 4, 8 once the smaller distances are reduced: quad_perm [1,0,3,2] / [2,3,0,1],
// then row_half_mirror / row_mirror (they pair the already-uniform halves)
template <int STEP>
constexpr int kGroupXor = STEP == 1 ? 0xB1 : STEP == 2 ? 0x4E : STEP == 4 ? 0x141 : 0x140;

template <int G, int STEP = 1>
__device__ __forceinline__ void group_max_argmax(float& mf, float& mx, int& mi) {
  if constexpr (STEP < G) {
    mf = fmaxf(mf, dpp_f32<kGroupXor<STEP>>(mf));
    const float ov = dpp_f32<kGroupXor<STEP>>(mx);
    const int oi = dpp_i32<kGroupXor<STEP>>(mi);
    if (argmax_better(ov, oi, mx, mi)) mx = ov, mi = oi;
    group_max_argmax<G, STEP * 2>(mf, mx, mi);
  }
}

template <int G, int STEP = 1>
__device__ __forceinline__ void group_argmax(float& v, int& i) {
  if constexpr (STEP < G) {
    const float ov = dpp_f32<kGroupXor<STEP>>(v);
    const int oi = dpp_i32<kGroupXor<STEP>>(i);
    if (argmax_better(ov, oi, v, i)) v = ov, i = oi;
    group_argmax<G, STEP * 2>(v, i);
  }
}

// lane K of this lane's G-group, broadcast (row_newbcast: lane n of each 16-lane row; quad_perm inside quads)
template <int G, int K>
__device__ __forceinline__ float group_bcast(float x) {
  if constexpr (G == 16) {
    return dpp_f32<0x150 + K>(x);
  } else if constexpr (G == 8) {
    const float a = dpp_f32<0x150 + K>(x), b = dpp_f32<0x158 + K>(x);
    return (threadIdx.x & 8) ? b : a;
  } else if constexpr (G == 4) {
    return dpp_f32<K | (K << 2) | (K << 4) | (K << 6)>(x);
  } else {
    static_assert(G == 2, "G <= 16");
    return dpp_f32<K | (K << 2) | ((2 + K) << 4) | ((2 + K) << 6)>(x);
  }
}

// sum of the group's lanes 0 .. C-1 in class order (the reference's softmax denominator order): bit-identical to the
// serial loop over __shfl broadcasts
template <int G, int... Ks>
__device__ __forceinline__ float class_order_sum(float e, int C, std::integer_sequence<int, Ks...>) {
  float s = 0.f;
  ((Ks < C ? (s += group_bcast<G, Ks>(e), 0) : 0), ...);
  return s;
}

// The same image, G lanes per row (G = the power of two >= C, <= 64): lane c of a row's group owns class c, so the
// per-class curve work (two threshold searches, two LDS atomics) runs in parallel across the row's lanes instead of
// serially in one thread; the row's max / argmax come from shuffles, and its softmax denominators are summed by
// shuffling the lanes' exponentials in class order into every lane (the order the one-thread-per-row kernel and the
// members' own kernels use, so the rounded softmax values are the same).
template <typename scalar_t, typename target_t, int G>
__global__ void __launch_bounds__(kFamRowThreads) family_rows_g_kernel(const scalar_t* __restrict__ preds,
                                                                    const target_t* __restrict__ target, long long N,
                                                                    FamilySpec sp) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  int* h = smem;
  double* thr_s = reinterpret_cast<double*>(smem + ((sp.part_words + 1) & ~1));
  __shared__ int blk_outside;
  constexpr int R = kFamRowThreads / G;  // rows per block step
  const int C = sp.C, T = sp.T, nb = sp.nb;
  for (int i = threadIdx.x; i < sp.part_words; i += kFamRowThreads) h[i] = 0;
  for (int i = threadIdx.x; i < T; i += kFamRowThreads) thr_s[i] = sp.thr[i];
  if (threadIdx.x == 0) blk_outside = 0;
  __syncthreads();
  // thresholds on an even grid (within 1e-9 of a step): the short search
  const double t0 = T > 0 ? thr_s[0] : 0.0, tl = T > 0 ? thr_s[T - 1] : 0.0;
  const double inv = T > 1 && tl > t0 ? static_cast<double>(T - 1) / (tl - t0) : 0.0;
  bool off_grid = false;
  for (int i = threadIdx.x; i < T; i += kFamRowThreads)
    off_grid |= !(fabs((thr_s[i] - t0) * inv - static_cast<double>(i)) <= 1e-9);
  const bool on_grid = !__syncthreads_or(off_grid);  // (every thread takes part)
  const bool grid = !(sp.abl & 32) && T > 1 && inv > 0.0 && on_grid;
  const int c = threadIdx.x % G;
  const int gbase = (threadIdx.x & (kWave - 1)) - c;  // the group's first lane in the wave
  const bool has_c = c < C;
  bool outside = false, bad = false;
  // 4 block steps per pass, their loads issued together (one wave per SIMD: a load per step would expose the
  // memory latency 4 times)
  const long long step = static_cast<long long>(gridDim.x) * R;
  for (long long rb = static_cast<long long>(blockIdx.x) * R; rb < N; rb += 4 * step) {
    float vv[4];
    long long tt[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long row = rb + u * step + threadIdx.x / G;
      vv[u] = (row < N && has_c) ? to_f32(preds[row * C + c]) : -INFINITY;
      tt[u] = row < N ? static_cast<long long>(target[row]) : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    const long long row0 = rb + u * step;  // uniform across the block: shuffles see whole groups
    if (row0 >= N) break;
    const long long row = row0 + threadIdx.x / G;
    const bool live = row < N;
    const bool mine = live && has_c;
    const float v = vv[u];
    outside |= mine && !(v >= 0.f && v <= 1.f);
    float mf = mine ? v : -INFINITY;  // NaN-ignoring max (fmaxf drops NaN)
    float mx = v;
    int mi = mine ? c : 0x7fffffff;
    if constexpr (G <= 16) {
      group_max_argmax<G>(mf, mx, mi);  // DPP (VALU): a ds_bpermute butterfly was ~100 cycles per dependent step
    } else {
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1) {
        mf = fmaxf(mf, __shfl_xor(mf, off, kWave));
        const float ov = __shfl_xor(mx, off, kWave);
        const int oi = __shfl_xor(mi, off, kWave);
        if (argmax_better(ov, oi, mx, mi)) mx = ov, mi = oi;
      }
    }
    // softmax denominators in class order (every lane gets the same sums)
    auto order_sum = [&](float e) {
      if constexpr (G <= 16) {
        return class_order_sum<G>(e, C, std::make_integer_sequence<int, G>{});
      } else {
        float t = 0.f;
        for (int k = 0; k < C; ++k) t += __shfl(e, gbase + k, kWave);
        return t;
      }
    };
    const float e_cal = mine ? expf(v - mx) : 0.f;
    float s_cal = 0.f;
    if (sp.abl & 8) s_cal = 1.f;
    else s_cal = order_sum(e_cal);
    float s_cur = s_cal;
    const bool nan_row = !(mf == mx);  // a NaN in the row: the two shifts differ (uniform within the group)
    float e_cur = e_cal;
    if (__any(nan_row)) {
      e_cur = mine ? expf(v - mf) : 0.f;
      const float t2 = order_sum(e_cur);
      if (nan_row) s_cur = t2;
      else e_cur = e_cal;
    }
    const long long tv = tt[u];
    const bool valid = tv >= 0 && tv < C;
    bad |= live && c == 0 && !valid;
    const int t = static_cast<int>(valid ? tv : 0);
    if (live && valid && c == 0 && sp.need_cm) atomicAdd(&h[t * C + mi], 1);
    if (mine && valid && T > 0 && !(sp.abl & 16)) {
      const double praw = static_cast<double>(v);
      const double psoft = static_cast<double>(round_to<scalar_t>(e_cur / s_cur));
      const int pos = c == t;
      int braw, bsoft;
      if (sp.abl & 1) {
        braw = 0;
        bsoft = static_cast<int>(psoft);
      } else if (grid) {
        braw = bucket_guess(thr_s, T, praw, t0, inv);
        bsoft = bucket_guess(thr_s, T, psoft, t0, inv);
      } else {
        braw = bucket_of(thr_s, T, praw);
        bsoft = bucket_of(thr_s, T, psoft);
      }
      atomicAdd(&h[sp.off_cv + ((0 * (T + 1) + braw) * C + c) * 2 + pos], 1);
      atomicAdd(&h[sp.off_cv + ((1 * (T + 1) + bsoft) * C + c) * 2 + pos], 1);
    }
    if (nb > 0) {
      float sv = mine ? round_to<scalar_t>(e_cal / s_cal) : -INFINITY;
      int si = mine ? c : 0x7fffffff;
      if constexpr (G <= 16) {
        group_argmax<G>(sv, si);
      } else {
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) {
          const float ov = __shfl_xor(sv, off, kWave);
          const int oi = __shfl_xor(si, off, kWave);
          if (argmax_better(ov, oi, sv, si)) sv = ov, si = oi;
        }
      }
      // both top-1 candidates of the row; the fold keeps the variant the batch-wide decision picks and bins it
      if (live && c == 0) sp.cand[row] = make_float4(mx, mi == tv ? 1.f : 0.f, sv, si == tv ? 1.f : 0.f);
    }
  }
    }
  if (__any(outside) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(&blk_outside, 1);
  if (__any(bad) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(sp.err_scratch, kErrTargetOutOfRange);
  __syncthreads();
  for (int i = threadIdx.x; i < sp.part_words; i += kFamRowThreads)
    if (h[i]) atomicAdd(&sp.img[i], h[i]);
  if (threadIdx.x == 0 && blk_outside) atomicOr(&sp.outside[sp.slot], 1);
}

__device__ __forceinline__ long long wave_incl_scan_ll(long long v) {
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const long long u = __shfl_up(v, o, kWave);
    if (lane >= o) v += u;
  }
  return v;
}

// Fold roles by block: [0] confusion matrix + stat scores (+ validation words), then ceil(C / 4) curve blocks (a
// wave per class column), then the calibration select blocks (rows), then one calibration-bins block.  Every image
// word is read, and re-zeroed, by exactly one block.
__global__ void __launch_bounds__(kFamThreads) family_fold_kernel(FamilySpec sp, long long N, int r_cv, int r_sel,
                                                                  int n_sel) {
  __shared__ long long cmb[kFamMaxC * kFamMaxC];
  __shared__ long long red[4][kFamThreads / kWave];
  const int C = sp.C, T = sp.T, nb = sp.nb;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const int var = sp.outside[sp.slot] ? 1 : 0;  // the batch-wide `softmax unless every score is in [0, 1]`
  const int bid = blockIdx.x;
  if (bid == 0) {
    if (tid == 0) {
      const int e = *sp.err_scratch;
      if (e) {
        for (int k = 0; k < sp.n_err; ++k) atomicOr(sp.err[k], e);
        *sp.err_scratch = 0;
      }
      sp.outside[sp.slot ^ 1] = 0;  // the next update's decision word
    }
    if (!sp.need_cm) return;
    for (int i = tid; i < C * C; i += kFamThreads) {
      const long long v = sp.img[i];
      sp.img[i] = 0;
      cmb[i] = v;
      for (int k = 0; k < sp.n_cm; ++k)  // no-return atomics: a plain += chained a load round trip per consumer
        if (v) atomic_add_i64(sp.cm[k] + i, v);
    }
    __syncthreads();
    if (sp.n_st == 0) return;
    long long tp = 0, fp = 0, fn = 0, all = 0;
    if (tid < C) {
      long long rows = 0, cols = 0;
      for (int j = 0; j < C; ++j) {
        rows += cmb[tid * C + j];  // target == tid
        cols += cmb[j * C + tid];  // argmax == tid
      }
      tp = cmb[tid * C + tid];
      fp = cols - tp;
      fn = rows - tp;
      all = rows;
    }
    long long v4[4] = {tp, fp, fn, all};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long sum = wave_sum_ll(v4[q]);
      if (lane == 0) red[q][wave] = sum;
    }
    __syncthreads();
    long long tot[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      for (int w = 0; w < kFamThreads / kWave; ++w) tot[q] += red[q][w];
    const long long n_valid = tot[3];
    for (int k = 0; k < sp.n_st; ++k) {
      if (sp.st_micro[k]) {
        if (tid == 0) {  // (no-return atomics: four += per consumer were 4 x n_st dependent load round trips)
          atomic_add_i64(sp.st[k][0], tot[0]);
          atomic_add_i64(sp.st[k][1], tot[1]);
          atomic_add_i64(sp.st[k][2], static_cast<long long>(C) * n_valid - tot[0] - tot[1] - tot[2]);
          atomic_add_i64(sp.st[k][3], tot[2]);
        }
      } else if (tid < C) {
        atomic_add_i64(sp.st[k][0] + tid, tp);
        atomic_add_i64(sp.st[k][1] + tid, fp);
        atomic_add_i64(sp.st[k][2] + tid, n_valid - tp - fp - fn);
        atomic_add_i64(sp.st[k][3] + tid, fn);
      }
    }
    return;
  }
  if (bid >= r_cv && bid < r_sel) {
    const int col = (bid - r_cv) * kFoldCols + wave;
    if (col >= C || T == 0) return;
    // the chosen variant's bucket counts of this column; then curve_finalize_kernel's suffix scan: predicted positive
    // at sorted threshold i <=> bucket > i.  Both variants' words of the column are re-zeroed.
    int* base = sp.img + sp.off_cv + var * (T + 1) * C * 2;
    int* other = sp.img + sp.off_cv + (var ^ 1) * (T + 1) * C * 2;
    long long tot_neg = 0, tot_pos = 0;
    for (int b = lane; b <= T; b += kWave) {
      tot_neg += base[(b * C + col) * 2];
      tot_pos += base[(b * C + col) * 2 + 1];
    }
    tot_neg = wave_sum_ll(tot_neg);
    tot_pos = wave_sum_ll(tot_pos);
    long long carry_neg = 0, carry_pos = 0;
    for (int start = 0; start <= T; start += kWave) {
      const int b = T - (start + lane);
      long long neg = 0, pos = 0;
      if (b >= 0) {
        int* h = base + (b * C + col) * 2;
        neg = h[0];
        pos = h[1];
        h[0] = 0;
        h[1] = 0;
        int* g = other + (b * C + col) * 2;
        g[0] = 0;
        g[1] = 0;
      }
      const long long sneg = wave_incl_scan_ll(neg) + carry_neg;
      const long long spos = wave_incl_scan_ll(pos) + carry_pos;
      if (b >= 1) {
        const long long i = sp.perm[b - 1];
        int64_t* out = sp.curve + (i * C + col) * 4;
        out[0] += tot_neg - sneg;  // tn
        out[1] += sneg;            // fp
        out[2] += tot_pos - spos;  // fn
        out[3] += spos;            // tp
      }
      carry_neg = __shfl(sneg, kWave - 1, kWave);
      carry_pos = __shfl(spos, kWave - 1, kWave);
    }
    return;
  }
  if (bid >= r_sel && bid < r_sel + n_sel) {
    // the calibration member's outputs: the variant the batch-wide decision picked, and its (count, sum conf,
    // sum acc) bins into the metric's cache -- per block in LDS, then one float atomic per non-zero word (binning
    // only the kept variant here halved the rows kernel's calibration work; it bins no discarded candidate)
    __shared__ float bsh[kFoldMaxBins * 3];
    __shared__ float bnd[kFoldMaxBins];
    const bool do_bins = sp.bins != nullptr && nb > 0;
    const bool lds_bins = nb <= kFoldMaxBins;
    if (do_bins && lds_bins) {
      for (int i = tid; i < nb * 3; i += kFamThreads) bsh[i] = 0.f;
      for (int i = tid; i < nb; i += kFamThreads) bnd[i] = sp.bounds[i];
      __syncthreads();
    }
    const float* bb = lds_bins ? bnd : sp.bounds;
    float* bins = lds_bins ? bsh : sp.bins;
    const float b_lo = do_bins ? bb[0] : 0.f;
    const float b_inv = do_bins && nb > 1 && bb[nb - 1] > b_lo ? static_cast<float>(nb - 1) / (bb[nb - 1] - b_lo)
                                                               : 0.f;
    for (long long i = static_cast<long long>(bid - r_sel) * kFamThreads + tid; i < N;
         i += static_cast<long long>(n_sel) * kFamThreads) {
      const float4 c = sp.cand[i];
      const float cv = var ? c.z : c.x, av = var ? c.w : c.y;
      sp.conf[i] = cv;
      sp.acc[i] = av;
      if (do_bins) {
        // b = #{bounds <= conf} - 1: a guess from the bounds' even grid (linspace), then exact steps (any sorted
        // bounds); NaN: past every bound (torch.bucketize), the reference's last bin
        int b;
        if (cv != cv) {
          b = nb - 1;
        } else {
          const float g = (cv - b_lo) * b_inv;
          b = g < 0.f ? -1 : (g >= static_cast<float>(nb - 1) ? nb - 1 : static_cast<int>(g));
          while (b + 1 < nb && bb[b + 1] <= cv) ++b;
          while (b >= 0 && bb[b] > cv) --b;
        }
        if (b >= 0) {
          atomicAdd(bins + b * 3, 1.f);
          atomicAdd(bins + b * 3 + 1, cv);
          atomicAdd(bins + b * 3 + 2, av);
        }
      }
    }
    if (do_bins && lds_bins) {
      __syncthreads();
      for (int i = tid; i < nb * 3; i += kFamThreads)
        if (bsh[i] != 0.f) atomicAdd(sp.bins + i, bsh[i]);
    }
  }
}

}  // namespace

// preds [N, C] (bf16 / fp16 / fp32, C <= 64), target [N] (int32 / int64).  Consumers:
//   cm: confusion matrices int64 [C, C]; st: stat-score states, 4 per consumer (tp, fp, tn, fn) int64 [C] or [1]
//   (st_micro[k] = 1); curve: int64 [T, C, 2, 2] with thr_sorted f64 [T] / perm i64 [T] (empty curve: none);
//   conf / acc: f32 [N] outputs with bounds f32 [nb] (empty conf: no calibration member), bins f32 [nb, 3] (may be
//   empty); err: validation words (int32) that get the target-range bit.
// work: int32 scratch of at least family_work_words(...) words, ZERO before its first use (every fold re-zeroes
// what it read); slot: update parity (the decision word's double buffer); cand: f32 [4 N] scratch when a calibration
// member is present.  Two launches.
void mc_family_update(const at::Tensor& preds, const at::Tensor& target, at::TensorList cm, at::TensorList st,
                      at::IntArrayRef st_micro, const at::Tensor& curve, const at::Tensor& thr_sorted,
                      const at::Tensor& perm, const at::Tensor& conf, const at::Tensor& acc, const at::Tensor& bounds,
                      const at::Tensor& bins, at::TensorList err, at::Tensor work, int64_t slot,
                      at::Tensor cand) {
  TM_CHECK_CUDA(preds);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.dim() == 2 && target.dim() == 1 && target.size(0) == preds.size(0),
              "mc_family_update: preds [N, C], target [N]");
  const long long N = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  TORCH_CHECK(C >= 1 && C <= kFamMaxC, "mc_family_update: 1 <= C <= ", kFamMaxC);
  TORCH_CHECK(cm.size() <= static_cast<size_t>(kFamMaxCons) && st.size() % 4 == 0 &&
                  st.size() / 4 <= static_cast<size_t>(kFamMaxCons) && st_micro.size() == st.size() / 4 &&
                  err.size() <= static_cast<size_t>(kFamMaxErr),
              "mc_family_update: too many consumers");
  FamilySpec sp{};
  sp.C = C;
  sp.n_cm = static_cast<int>(cm.size());
  for (int k = 0; k < sp.n_cm; ++k) {
    TORCH_CHECK(cm[k].scalar_type() == at::kLong && cm[k].is_contiguous() && cm[k].numel() == C * C &&
                    cm[k].get_device() == preds.get_device(), "mc_family_update: confmat int64 [C, C]");
    sp.cm[k] = cm[k].data_ptr<int64_t>();
  }
  sp.n_st = static_cast<int>(st.size() / 4);
  for (int k = 0; k < sp.n_st; ++k) {
    sp.st_micro[k] = static_cast<int>(st_micro[k]);
    for (int q = 0; q < 4; ++q) {
      const at::Tensor& s = st[4 * k + q];
      TORCH_CHECK(s.scalar_type() == at::kLong && s.is_contiguous() && s.get_device() == preds.get_device() &&
                      s.numel() == (sp.st_micro[k] ? 1 : C), "mc_family_update: stat states int64 [C] / [1]");
      sp.st[k][q] = s.data_ptr<int64_t>();
    }
  }
  sp.need_cm = sp.n_cm > 0 || sp.n_st > 0;
  static const int abl = [] {
    const char* e = std::getenv("TM_AMD_FAMILY_ABLATE");
    return e ? std::atoi(e) : 0;
  }();
  sp.abl = abl;
  if (curve.numel() > 0) {
    sp.T = static_cast<int>(thr_sorted.numel());
    TORCH_CHECK(sp.T >= 1 && thr_sorted.scalar_type() == at::kDouble && perm.scalar_type() == at::kLong &&
                    perm.numel() == sp.T && curve.scalar_type() == at::kLong && curve.is_contiguous() &&
                    curve.numel() == static_cast<long long>(sp.T) * C * 4,
                "mc_family_update: curve state int64 [T, C, 2, 2] with f64 thresholds and i64 perm");
    sp.thr = thr_sorted.data_ptr<double>();
    sp.perm = perm.data_ptr<int64_t>();
    sp.curve = curve.data_ptr<int64_t>();
  }
  if (conf.numel() > 0 || N == 0) {
    sp.nb = static_cast<int>(bounds.numel());
    TORCH_CHECK(sp.nb >= 1 && bounds.scalar_type() == at::kFloat && conf.scalar_type() == at::kFloat &&
                    acc.scalar_type() == at::kFloat && conf.numel() == N && acc.numel() == N,
                "mc_family_update: calibration outputs f32 [N] with f32 bounds");
    sp.bounds = bounds.data_ptr<float>();
    sp.conf = conf.data_ptr<float>();
    sp.acc = acc.data_ptr<float>();
    if (bins.numel() > 0) {
      TORCH_CHECK(bins.scalar_type() == at::kFloat && bins.is_contiguous() && bins.numel() == sp.nb * 3,
                  "mc_family_update: bins f32 [nb, 3]");
      sp.bins = bins.data_ptr<float>();
    }
  }
  sp.n_err = static_cast<int>(err.size());
  for (int k = 0; k < sp.n_err; ++k) {
    TORCH_CHECK(err[k].scalar_type() == at::kInt && err[k].numel() >= 1, "mc_family_update: int32 error words");
    sp.err[k] = err[k].data_ptr<int>();
  }
  if (N == 0) return;
  sp.off_cv = sp.need_cm ? C * C : 0;
  sp.off_cb = sp.off_cv + (sp.T > 0 ? 2 * (sp.T + 1) * C * 2 : 0);
  sp.part_words = sp.off_cb;  // (the calibration bins are binned by the fold, from the kept variant)
  const size_t lds = static_cast<size_t>((sp.part_words + 1) & ~1) * 4 + static_cast<size_t>(sp.T) * 8;
  TORCH_CHECK(lds <= 64 * 1024, "mc_family_update: partial image exceeds 64 KiB of LDS");
  // G lanes per row; blocks capped so a hot image word takes at most that many global atomics (TM_AMD_FAMILY_BLOCKS)
  static const int max_blocks = [] {
    const char* e = std::getenv("TM_AMD_FAMILY_BLOCKS");
    return e ? std::max(1, std::atoi(e)) : 128;
  }();
  const int G = C <= 4 ? 4 : C <= 8 ? 8 : C <= 16 ? 16 : C <= 32 ? 32 : 64;
  const int rows_per_blk = kFamRowThreads / G;
  const int nblk = static_cast<int>(std::min<long long>((N + rows_per_blk - 1) / rows_per_blk, max_blocks));
  TORCH_CHECK(work.scalar_type() == at::kInt && work.is_contiguous() && work.numel() >= sp.part_words + 3,
              "mc_family_update: work scratch too small");
  TORCH_CHECK(slot == 0 || slot == 1, "mc_family_update: slot 0 / 1");
  sp.img = work.data_ptr<int>();
  sp.outside = sp.img + sp.part_words;
  sp.slot = static_cast<int>(slot);
  sp.err_scratch = sp.outside + 2;
  if (sp.nb > 0) {
    TORCH_CHECK(cand.scalar_type() == at::kFloat && cand.numel() >= 4 * N, "mc_family_update: cand f32 [4 N]");
    sp.cand = reinterpret_cast<float4*>(cand.data_ptr<float>());
  }
  auto s = stream();
  // inside a hipGraph capture the host parity would be frozen into the graph: word 0 is zeroed before the rows pass
  // and re-armed after the fold on every replay (both words end zero, so eager updates around the graph keep theirs)
  const bool captured = stream_capturing(s);
  if (captured) {
    sp.slot = 0;
    launch_zero_words(sp.outside, 2, s);
  }
  TM_DISPATCH_TARGET(target.scalar_type(), "mc_family_update", [&] {
    const target_t* tp = reinterpret_cast<const target_t*>(target.data_ptr());
    auto run = [&](auto tag) {
      using scalar_t = decltype(tag);
      const scalar_t* pp = reinterpret_cast<const scalar_t*>(preds.data_ptr());
      auto go = [&](auto gc) {
        constexpr int GG = decltype(gc)::value;
        hipLaunchKernelGGL((family_rows_g_kernel<scalar_t, target_t, GG>), dim3(nblk), dim3(kFamRowThreads), lds, s,
                           pp, tp, N, sp);
      };
      if (G == 4) go(std::integral_constant<int, 4>{});
      else if (G == 8) go(std::integral_constant<int, 8>{});
      else if (G == 16) go(std::integral_constant<int, 16>{});
      else if (G == 32) go(std::integral_constant<int, 32>{});
      else go(std::integral_constant<int, 64>{});
    };
    switch (preds.scalar_type()) {
      case at::kBFloat16: run(c10::BFloat16{}); break;
      case at::kHalf: run(c10::Half{}); break;
      case at::kFloat: run(float{}); break;
      default: TORCH_CHECK(false, "mc_family_update: bf16 / fp16 / fp32 scores");
    }
  });
  const int r_cv = 1;
  const int n_cv = sp.T > 0 ? (C + kFoldCols - 1) / kFoldCols : 0;
  const int r_sel = r_cv + n_cv;
  const int n_sel = sp.nb > 0 ? static_cast<int>(std::min<long long>((N + kFamThreads - 1) / kFamThreads, 256)) : 0;
  const int grid = r_sel + n_sel;
  hipLaunchKernelGGL(family_fold_kernel, dim3(grid), dim3(kFamThreads), 0, s, sp, N, r_cv, r_sel, n_sel);
  if (captured) launch_zero_words(sp.outside, 2, s);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// int32 words the scratch `work` must hold
int64_t mc_family_work_words(int64_t C, bool need_cm, int64_t T, int64_t nb) {
  (void)nb;
  return (need_cm ? C * C : 0) + (T > 0 ? 2 * (T + 1) * C * 2 : 0) + 3;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "mc_family_update(Tensor preds, Tensor target, Tensor(a!)[] cm, Tensor(b!)[] st, int[] st_micro, "
      "Tensor(c!) curve, Tensor thr_sorted, Tensor perm, Tensor(d!) conf, Tensor(e!) acc, Tensor bounds, "
      "Tensor(f!) bins, Tensor(g!)[] err, Tensor(h!) work, int slot, Tensor(i!) cand) -> ()");
  m.def("mc_family_work_words(int C, bool need_cm, int T, int nb) -> int", &tm_amd::mc_family_work_words);
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("mc_family_update", &tm_amd::mc_family_update); }
