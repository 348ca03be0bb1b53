// Multi-threshold ("binned") confusion matrices for the PR-curve / ROC / AUROC / AP / @fixed-point family.
//
// Reference: F/classification/precision_recall_curve.py:210-250 (binary), :482-527 (multiclass), :771-795
// (multilabel).  The reference materialises `preds[:, :, None] >= thresholds` (N x C x T) and bincounts it, or loops
// over thresholds (one full pass over the data per threshold) above 50k / 1M elements, and decides sigmoid/softmax
// with a blocking `torch.all(0 <= preds <= 1)` host sync.
//
// Here every element is read once: it is bucketed by a binary search over the (sorted) thresholds held in LDS and
// counted into an LDS-privatised histogram  hist[bucket][column][is_positive]  with bucket = #{thresholds <= p};
// "p >= thr_i" is then "bucket > i", so a suffix scan of the histogram yields tp/fp for every threshold (O(N*C + T*C)
// work instead of O(N*C*T)).  The sigmoid/softmax decision stays on the device: a first pass raises a "not
// probabilities" bit in a control word (and, for multiclass, stores per-row max / sum-exp), the binning pass reads the
// bit.  Comparisons are done in fp64 between the pred rounded to its own dtype and the threshold, which is exactly
// PyTorch's type-promoted `preds >= thresholds`.
//
// Launches per update: range/rowstat pass, binning pass, finalize (suffix scan + add into the int64 state + re-zero
// of the scratch histogram and control word so the workspace is ready for the next update without a memset).
#include "common/compute_bodies.h"

namespace tm_amd {
namespace {

constexpr int kCtlNotProb = 1;
constexpr int kBinThreads = 256;
constexpr int kMaxLdsThr = 4096;        // thresholds staged in LDS (fp64) up to this many
constexpr int kLdsHistBytes = 48 * 1024; // LDS histogram budget per block

enum CurveMode : int { kBinary = 0, kMultilabel = 1, kMulticlass = 2 };

template <typename T>
__device__ __forceinline__ bool is_prob(T x) {
  const float v = to_f32(x);
  return v >= 0.f && v <= 1.f;  // NaN -> false, as torch.all((p >= 0) * (p <= 1))
}
template <>
__device__ __forceinline__ bool is_prob<double>(double x) {
  return x >= 0.0 && x <= 1.0;
}

// Pass 1 (binary / multilabel): any considered pred outside [0, 1] -> control bit.  Binary ignores masked elements
// (the reference drops them before the check); multilabel checks all of them (it applies sigmoid before masking).
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(256) curve_range_kernel(const scalar_t* __restrict__ preds,
                                                          const target_t* __restrict__ target, long long n,
                                                          long long ignore_index, bool use_ignore,
                                                          int* __restrict__ ctl) {
  bool bad = false;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    if (use_ignore && static_cast<long long>(target[i]) == ignore_index) continue;
    bad |= !is_prob(preds[i]);
  }
  if (__any(bad) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(ctl, kCtlNotProb);
}

// Pass 1 (multiclass): one wave per row (several rows per wave for small C): range check over non-ignored rows and
// per-row softmax statistics (max, sum exp(x - max)).
template <typename scalar_t, typename target_t, int LPR>
__global__ void __launch_bounds__(256) curve_rowstat_kernel(const scalar_t* __restrict__ preds,
                                                            const target_t* __restrict__ target, long long rows,
                                                            int c, long long ignore_index, bool use_ignore,
                                                            float2* __restrict__ stat, int* __restrict__ ctl) {
  const int lane = threadIdx.x & (LPR - 1);
  const long long groups = static_cast<long long>(gridDim.x) * (blockDim.x / LPR);
  bool bad = false;
  for (long long r = blockIdx.x * static_cast<long long>(blockDim.x / LPR) + threadIdx.x / LPR; r < rows;
       r += groups) {
    const scalar_t* row = preds + r * c;
    const bool considered = !(use_ignore && static_cast<long long>(target[r]) == ignore_index);
    float m = -INFINITY;
    for (int j = lane; j < c; j += LPR) {
      const scalar_t x = row[j];
      bad |= considered && !is_prob(x);
      m = fmaxf(m, to_f32(x));
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, LPR));
    float s = 0.f;
    for (int j = lane; j < c; j += LPR) s += expf(to_f32(row[j]) - m);
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, LPR);
    if (lane == 0) stat[r] = make_float2(m, s);
  }
  if (__any(bad) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(ctl, kCtlNotProb);
}

__device__ __forceinline__ int bucket_of(const double* __restrict__ thr, int t, double p) {
  // number of thresholds <= p  (thr sorted ascending); NaN -> 0
  int lo = 0, hi = t;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (thr[mid] <= p) lo = mid + 1; else hi = mid;
  }
  return lo;
}

template <typename scalar_t>
__device__ __forceinline__ double as_prob_sigmoid(scalar_t x, bool transform) {
  if (!transform) return static_cast<double>(to_f32(x));
  const float v = 1.f / (1.f + expf(-to_f32(x)));
  return static_cast<double>(round_to<scalar_t>(v));
}
template <>
__device__ __forceinline__ double as_prob_sigmoid<double>(double x, bool transform) {
  return transform ? 1.0 / (1.0 + exp(-x)) : x;
}

// Pass 2: bucket + histogram.  Block (tile, split) owns columns [c0, c0 + cw) and a contiguous range of rows.
template <typename scalar_t, typename target_t, int MODE>
__global__ void __launch_bounds__(kBinThreads) curve_bin_kernel(
    const scalar_t* __restrict__ preds, const target_t* __restrict__ target, const float2* __restrict__ stat,
    long long rows, int cols, int cw, const double* __restrict__ thr_g, int t, const int* __restrict__ ctl,
    int* __restrict__ err, long long ignore_index, bool use_ignore, bool micro, bool lds_hist,
    unsigned* __restrict__ hist_g, long long rows_per_split) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bool lds_thr = t <= kMaxLdsThr;
  double* thr_s = reinterpret_cast<double*>(smem);
  unsigned* hist_s = reinterpret_cast<unsigned*>(smem + (lds_thr ? t * sizeof(double) : 0));
  const int hcols = micro ? 1 : cw;                 // histogram columns of this block
  const int hcols_g = micro ? 1 : cols;             // histogram columns of the global histogram
  const int c0 = blockIdx.x * cw;
  const int cw_eff = min(cw, cols - c0);
  if (lds_thr)
    for (int i = threadIdx.x; i < t; i += blockDim.x) thr_s[i] = thr_g[i];
  if (lds_hist)
    for (int i = threadIdx.x; i < (t + 1) * hcols * 2; i += blockDim.x) hist_s[i] = 0u;
  __syncthreads();
  const double* thr = lds_thr ? thr_s : thr_g;
  const bool transform = (*ctl & kCtlNotProb) != 0;

  const long long r0 = static_cast<long long>(blockIdx.y) * rows_per_split;
  const long long r1 = min(rows, r0 + rows_per_split);
  // 32-bit element index inside the block's slab (the host caps an update at 2^31 elements): the per-element
  // row / column split is one 32-bit division instead of a ~40-instruction 64-bit one
  const int elems = static_cast<int>((r1 - r0) * cw_eff);
  int bad = 0;
  for (int e = threadIdx.x; e < elems; e += blockDim.x) {
    const int rr = e / cw_eff;
    const long long r = r0 + rr;
    const int cl = e - rr * cw_eff;
    const int col = c0 + cl;
    const long long idx = r * cols + col;
    double p;
    int pos;
    if (MODE == kMulticlass) {
      const long long tv = static_cast<long long>(target[r]);
      if (use_ignore && tv == ignore_index) continue;
      if (tv < 0 || tv >= cols) {
        bad |= kErrTargetOutOfRange;
        continue;
      }
      pos = tv == col;
      if (transform) {
        const float2 st = stat[r];
        const float v = expf(to_f32(preds[idx]) - st.x) / st.y;
        p = std::is_same<scalar_t, double>::value ? static_cast<double>(v) : static_cast<double>(round_to<scalar_t>(v));
      } else {
        p = std::is_same<scalar_t, double>::value ? static_cast<double>(preds[idx])
                                                  : static_cast<double>(to_f32(preds[idx]));
      }
    } else {
      const long long tv = static_cast<long long>(target[idx]);
      if (use_ignore && tv == ignore_index) continue;
      if (tv != 0 && tv != 1) {
        bad |= kErrTargetNotBinary;
        continue;
      }
      pos = static_cast<int>(tv);
      p = as_prob_sigmoid<scalar_t>(preds[idx], transform);
    }
    const int b = bucket_of(thr, t, p);
    const int hc = micro ? 0 : (lds_hist ? cl : col);
    if (lds_hist) {
      atomicAdd(&hist_s[(b * hcols + hc) * 2 + pos], 1u);
    } else {
      atomicAdd(&hist_g[(static_cast<long long>(b) * hcols_g + hc) * 2 + pos], 1u);
    }
  }
  if (bad) atomicOr(err, bad);
  if (lds_hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < (t + 1) * hcols * 2; i += blockDim.x) {
      const unsigned v = hist_s[i];
      if (v == 0u) continue;
      const int pos = i & 1;
      const int hc = (i >> 1) % hcols;
      const int b = (i >> 1) / hcols;
      const int gc = micro ? 0 : c0 + hc;
      atomicAdd(&hist_g[(static_cast<long long>(b) * hcols_g + gc) * 2 + pos], v);
    }
  }
}

__device__ __forceinline__ long long wave_incl_scan(long long v) {
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const long long u = __shfl_up(v, o, kWave);
    if (lane >= o) v += u;
  }
  return v;
}

// Pass 3: one wave per histogram column.  Suffix scan over buckets -> tp/fp at every threshold; tn/fn from the column
// totals.  Adds into state [T, hcols, 2, 2] (int64) at the caller's threshold order and zeroes the scratch.
__global__ void __launch_bounds__(256) curve_finalize_kernel(unsigned* __restrict__ hist, int t, int hcols,
                                                             const int64_t* __restrict__ perm,
                                                             int64_t* __restrict__ state, int* __restrict__ ctl) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if (blockIdx.x == 0 && threadIdx.x == 0) *ctl = 0;
  if (wave >= hcols) return;
  const int col = wave;
  long long tot_pos = 0, tot_neg = 0;
  for (int b = lane; b <= t; b += kWave) {
    tot_neg += hist[(static_cast<long long>(b) * hcols + col) * 2];
    tot_pos += hist[(static_cast<long long>(b) * hcols + col) * 2 + 1];
  }
  tot_neg = wave_sum_ll(tot_neg);
  tot_pos = wave_sum_ll(tot_pos);
  long long carry_neg = 0, carry_pos = 0;
  // lane j of chunk k handles bucket b = t - (k*64 + j), descending; suffix sum at b counts buckets >= b
  for (int base = 0; base <= t; base += kWave) {
    const int b = t - (base + lane);
    long long neg = 0, pos = 0;
    if (b >= 0) {
      unsigned* h = hist + (static_cast<long long>(b) * hcols + col) * 2;
      neg = h[0];
      pos = h[1];
      h[0] = 0u;
      h[1] = 0u;
    }
    const long long sneg = wave_incl_scan(neg) + carry_neg;
    const long long spos = wave_incl_scan(pos) + carry_pos;
    if (b >= 1) {
      // sorted threshold index i = b - 1: predicted positive <=> bucket > i <=> bucket >= b
      const long long i = perm[b - 1];
      int64_t* out = state + (i * hcols + col) * 4;
      out[0] += tot_neg - sneg;  // tn
      out[1] += sneg;            // fp
      out[2] += tot_pos - spos;  // fn
      out[3] += spos;            // tp
    }
    carry_neg = __shfl(sneg, kWave - 1, kWave);
    carry_pos = __shfl(spos, kWave - 1, kWave);
  }
}


// ---------------------------------------------------------------------------------------------------------------
// compute(): AUROC / average precision from the binned state in ONE launch.
// Reference chain (F/classification/{roc,auroc,precision_recall_curve,average_precision}.py binned branches):
// rates / precision-recall from the [T, C, 2, 2] confmat (_safe_divide: 0/0 -> 0), flip, trapz or the AP step sum,
// then a nan-aware macro / weighted reduction with two host syncs (`isnan().any()`, boolean-mask indexing).
// AUROC / AP of a binned state: one block (body in common/compute_bodies.h, shared with compute_tasks.hip)
using cbody::kScoreAp;
using cbody::kScoreAuroc;

__global__ void __launch_bounds__(256) curve_score_kernel(const int64_t* __restrict__ st, int T, int C, int kind,
                                                          int average, float* __restrict__ out,
                                                          int* __restrict__ nan_flag) {
  extern __shared__ float sm[];  // [C] scores, [C] weights
  cbody::curve_score_block(st, T, C, kind, average, out, nan_flag, sm);
}
}  // namespace

// mode: 0 binary (preds/target [N]), 1 multilabel (preds/target [N, L]), 2 multiclass (preds [N, C], target [N]).
// thr_sorted: f64 [T] ascending; perm: i64 [T] caller index of each sorted threshold; hist: i32 scratch
// [(T+1) * hcols * 2] (zero on entry, zero on exit); ctl: i32 [1] scratch (zero on entry and exit);
// state: i64 [T, hcols, 2, 2] accumulated in place, hcols = 1 for binary / micro, else L or C.
void curve_update(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& thr_sorted,
                  const at::Tensor& perm, at::Tensor hist, at::Tensor ctl, at::Tensor state, at::Tensor err,
                  int64_t mode, int64_t ignore_index, bool use_ignore, bool micro) {
  TM_CHECK_CUDA(preds);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(thr_sorted.scalar_type() == at::kDouble && thr_sorted.is_contiguous(), "curve_update: thr must be f64");
  TORCH_CHECK(perm.scalar_type() == at::kLong && perm.numel() == thr_sorted.numel(), "curve_update: perm");
  TORCH_CHECK(hist.scalar_type() == at::kInt && ctl.scalar_type() == at::kInt && err.scalar_type() == at::kInt,
              "curve_update: scratch must be int32");
  TORCH_CHECK(state.scalar_type() == at::kLong && state.is_contiguous(), "curve_update: state must be int64");
  const int t = static_cast<int>(thr_sorted.numel());
  TORCH_CHECK(t >= 1, "curve_update: need at least one threshold");
  long long rows;
  int cols;
  if (mode == kBinary) {
    rows = preds.numel();
    cols = 1;
    TORCH_CHECK(target.numel() == rows, "curve_update: shape mismatch");
  } else {
    TORCH_CHECK(preds.dim() == 2, "curve_update: preds must be 2-D");
    rows = preds.size(0);
    cols = static_cast<int>(preds.size(1));
    if (mode == kMultilabel) {
      TORCH_CHECK(target.numel() == preds.numel(), "curve_update: shape mismatch");
    } else {
      TORCH_CHECK(target.numel() == rows, "curve_update: shape mismatch");
    }
  }
  const int hcols = (mode == kBinary || micro) ? 1 : cols;
  TORCH_CHECK(hist.numel() >= static_cast<long long>(t + 1) * hcols * 2, "curve_update: hist too small");
  TORCH_CHECK(state.numel() == static_cast<long long>(t) * hcols * 4, "curve_update: state shape");
  TORCH_CHECK(rows * cols < (1LL << 31), "curve_update: at most 2^31 elements per update");
  auto s = stream();
  const long long n = rows * cols;
  at::Tensor stat;
  if (n > 0) {
    TM_DISPATCH_FLOAT(preds.scalar_type(), "curve_update", [&] {
      TM_DISPATCH_TARGET(target.scalar_type(), "curve_update", [&] {
        const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
        const target_t* tg = reinterpret_cast<const target_t*>(target.data_ptr());
        if (mode == kMulticlass) {
          stat = at::empty({rows * 2}, preds.options().dtype(at::kFloat));
          float2* st = reinterpret_cast<float2*>(stat.data_ptr<float>());
          const int blocks = grid_cap((rows + 3) / 4, 2048);
          if (cols >= 48) {
            hipLaunchKernelGGL((curve_rowstat_kernel<scalar_t, target_t, 64>), dim3(blocks), dim3(256), 0, s, p, tg,
                               rows, cols, ignore_index, use_ignore, st, ctl.data_ptr<int>());
          } else if (cols >= 12) {
            hipLaunchKernelGGL((curve_rowstat_kernel<scalar_t, target_t, 16>), dim3(grid_cap((rows + 15) / 16, 2048)),
                               dim3(256), 0, s, p, tg, rows, cols, ignore_index, use_ignore, st, ctl.data_ptr<int>());
          } else {
            hipLaunchKernelGGL((curve_rowstat_kernel<scalar_t, target_t, 4>), dim3(grid_cap((rows + 63) / 64, 2048)),
                               dim3(256), 0, s, p, tg, rows, cols, ignore_index, use_ignore, st, ctl.data_ptr<int>());
          }
        } else {
          hipLaunchKernelGGL((curve_range_kernel<scalar_t, target_t>), dim3(grid_cap((n + 255) / 256, 1024)),
                             dim3(256), 0, s, p, tg, n, ignore_index, use_ignore && mode == kBinary,
                             ctl.data_ptr<int>());
        }
        // column tile so that the LDS histogram fits; fall back to global atomics for very fine threshold grids
        int cw = (mode == kBinary) ? 1 : std::min(cols, 64);
        const long long per_col = static_cast<long long>(t + 1) * 2 * sizeof(unsigned);
        bool lds_hist = true;
        if (micro) {
          lds_hist = per_col <= kLdsHistBytes;
        } else {
          while (cw > 1 && per_col * cw > kLdsHistBytes) cw = (cw + 1) / 2;
          lds_hist = per_col * cw <= kLdsHistBytes;
          if (!lds_hist) cw = (mode == kBinary) ? 1 : std::min(cols, 64);
        }
        const int tiles = (cols + cw - 1) / cw;
        const long long elems_per_tile = rows * std::min(cw, cols);
        long long splits = std::max<long long>(1, std::min<long long>((2048 + tiles - 1) / tiles,
                                                                      (elems_per_tile + 1023) / 1024));
        splits = std::min<long long>(splits, rows);
        const long long rows_per_split = (rows + splits - 1) / splits;
        splits = (rows + rows_per_split - 1) / rows_per_split;
        size_t lds = (t <= kMaxLdsThr ? t * sizeof(double) : 0) +
                     (lds_hist ? static_cast<size_t>(per_col) * (micro ? 1 : cw) : 0);
        const float2* st = mode == kMulticlass ? reinterpret_cast<const float2*>(stat.data_ptr<float>()) : nullptr;
        const int hist_mode = static_cast<int>(mode);
        dim3 grid(tiles, static_cast<unsigned>(splits));
        if (hist_mode == kMulticlass) {
          hipLaunchKernelGGL((curve_bin_kernel<scalar_t, target_t, kMulticlass>), grid, dim3(kBinThreads), lds, s, p,
                             tg, st, rows, cols, cw, thr_sorted.data_ptr<double>(), t, ctl.data_ptr<int>(),
                             err.data_ptr<int>(), ignore_index, use_ignore, micro, lds_hist,
                             reinterpret_cast<unsigned*>(hist.data_ptr<int>()), rows_per_split);
        } else {
          hipLaunchKernelGGL((curve_bin_kernel<scalar_t, target_t, kBinary>), grid, dim3(kBinThreads), lds, s, p, tg,
                             st, rows, cols, cw, thr_sorted.data_ptr<double>(), t, ctl.data_ptr<int>(),
                             err.data_ptr<int>(), ignore_index, use_ignore, false, lds_hist,
                             reinterpret_cast<unsigned*>(hist.data_ptr<int>()), rows_per_split);
        }
      });
    });
  }
  const int waves_per_block = 256 / kWave;
  hipLaunchKernelGGL(curve_finalize_kernel, dim3((hcols + waves_per_block - 1) / waves_per_block), dim3(256), 0, s,
                     reinterpret_cast<unsigned*>(hist.data_ptr<int>()), t, hcols, perm.data_ptr<int64_t>(),
                     state.data_ptr<int64_t>(), ctl.data_ptr<int>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// state: i64 [T, C, 2, 2] (C = 1 for binary); kind 0 AUROC / 1 AP; average 1 macro / 2 weighted (0: per class only).
// out: f32 [C + 1]; nan_flag: i32 [1].
void curve_score(const at::Tensor& state, int64_t kind, int64_t average, at::Tensor out, at::Tensor nan_flag) {
  TM_CHECK_CUDA(state);
  TORCH_CHECK(state.scalar_type() == at::kLong && state.is_contiguous() && state.dim() == 4 && state.size(2) == 2 &&
                  state.size(3) == 2, "curve_score: state must be contiguous int64 [T, C, 2, 2]");
  const int T = static_cast<int>(state.size(0)), C = static_cast<int>(state.size(1));
  TORCH_CHECK(T >= 1 && C >= 1 && C <= 16384, "curve_score: bad state shape");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == C + 1, "curve_score: out");
  TORCH_CHECK(nan_flag.scalar_type() == at::kInt && nan_flag.numel() >= 1, "curve_score: nan_flag");
  TORCH_CHECK(kind == kScoreAuroc || kind == kScoreAp, "curve_score: bad kind");
  hipLaunchKernelGGL(curve_score_kernel, dim3(1), dim3(256), 2 * C * sizeof(float), stream(),
                     state.data_ptr<int64_t>(), T, C, static_cast<int>(kind), static_cast<int>(average),
                     out.data_ptr<float>(), nan_flag.data_ptr<int>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("curve_score(Tensor state, int kind, int average, Tensor(a!) out, Tensor(b!) nan_flag) -> ()");
  m.def(
      "curve_update(Tensor preds, Tensor target, Tensor thr_sorted, Tensor perm, Tensor(a!) hist, Tensor(b!) ctl, "
      "Tensor(c!) state, Tensor(d!) err, int mode, int ignore_index, bool use_ignore, bool micro) -> ()");
}

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("curve_update", &tm_amd::curve_update);
  m.impl("curve_score", &tm_amd::curve_score);
}
