// Block-level bodies of the fused compute() kernels (one 256-thread block evaluates one metric's reduction).
//
// Each body is used twice: by its own one-task kernel (stat_reduce.hip, confmat_reduce.hip, curve.hip,
// regression_compute.hip) and by compute_tasks.hip, which runs the compute() of every member of a
// MetricCollection in ONE launch (block b -> task, local block).  Same code -> bit-identical results on both paths.
#pragma once

#include "common/tm_common.h"

namespace tm_amd {
namespace cbody {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  T s = 0;
  for (int w = 0; w < kThreads / kWave; ++w) s += red[w];
  return s;
}

// ------------------------------------------------------------------------------------------- stat-score family
// Accuracy / Hamming / Precision / Recall / Specificity / F-beta of [R, C] int64 tp/fp/tn/fn (reference
// F/classification/{accuracy,precision_recall,f_beta,specificity,hamming}.py `_*_reduce`).
enum StatKind : int { kAccuracy = 0, kHamming = 1, kPrecision = 2, kRecall = 3, kSpecificity = 4, kFBeta = 5 };
enum StatAvg : int { kMicro = 0, kMacro = 1, kWeighted = 2, kNone = 3 };

__device__ __forceinline__ float sdiv(float n, float d) { return n / (d == 0.f ? 1.f : d); }

__device__ __forceinline__ float class_score(int kind, float tp, float fp, float tn, float fn, bool multilabel,
                                             float beta2) {
  switch (kind) {
    case kAccuracy: return multilabel ? sdiv(tp + tn, tp + tn + fp + fn) : sdiv(tp, tp + fn);
    case kHamming: return 1.f - (multilabel ? sdiv(tp + tn, tp + tn + fp + fn) : sdiv(tp, tp + fn));
    case kPrecision: return sdiv(tp, tp + fp);
    case kRecall: return sdiv(tp, tp + fn);
    case kSpecificity: return sdiv(tn, tn + fp);
    default: return sdiv((1.f + beta2) * tp, (1.f + beta2) * tp + beta2 * fn + fp);
  }
}

// Reduction of C per-class counts to the score of ``avg``.  ``get(k, tp, fp, tn, fn)`` loads class k's counts (a state
// row, or a forward()'s batch counts straight out of the update workspace); out: [C] (none) or out[0].
// red: >= 4 doubles of LDS.  Every caller uses this one body, so every path gives bit-identical scores.
template <typename Get>
__device__ __forceinline__ void stat_reduce_body(Get get, int C, int kind, int avg, bool multilabel, float beta2,
                                                 float* __restrict__ out, double* red) {
  if (avg == kNone) {
    for (int k = threadIdx.x; k < C; k += kThreads) {
      long long a, b, c, d;
      get(k, a, b, c, d);
      out[k] = class_score(kind, static_cast<float>(a), static_cast<float>(b), static_cast<float>(c),
                           static_cast<float>(d), multilabel, beta2);
    }
    return;
  }
  if (avg == kMicro) {
    double s[4] = {0, 0, 0, 0};
    for (int k = threadIdx.x; k < C; k += kThreads) {
      long long a, b, c, d;
      get(k, a, b, c, d);
      s[0] += static_cast<double>(a);
      s[1] += static_cast<double>(b);
      s[2] += static_cast<double>(c);
      s[3] += static_cast<double>(d);
    }
    for (int i = 0; i < 4; ++i) s[i] = block_sum(s[i], red);
    if (threadIdx.x == 0) {
      // micro accuracy / hamming of a multilabel problem use the binary formula, everything else the class formula
      const bool binary_form = multilabel && (kind == kAccuracy || kind == kHamming);
      out[0] = class_score(kind, static_cast<float>(s[0]), static_cast<float>(s[1]), static_cast<float>(s[2]),
                           static_cast<float>(s[3]), binary_form, beta2);
    }
    return;
  }
  double num = 0.0, den = 0.0;
  for (int k = threadIdx.x; k < C; k += kThreads) {
    long long a, b, c, d;
    get(k, a, b, c, d);
    const float ftp = static_cast<float>(a), ffp = static_cast<float>(b), ftn = static_cast<float>(c),
                ffn = static_cast<float>(d);
    const float sc = class_score(kind, ftp, ffp, ftn, ffn, multilabel, beta2);
    float w;
    if (avg == kWeighted)
      w = ftp + ffn;
    else
      w = (!multilabel && a + b + d == 0) ? 0.f : 1.f;
    num += static_cast<double>(w * sc);
    den += static_cast<double>(w);
  }
  num = block_sum(num, red);
  den = block_sum(den, red);
  if (threadIdx.x == 0) out[0] = static_cast<float>(num / (den == 0.0 ? 1.0 : den));
}

// one row of the [R, C] states; red: >= 4 doubles of LDS
__device__ __forceinline__ void stat_reduce_row(const int64_t* __restrict__ tp, const int64_t* __restrict__ fp,
                                                const int64_t* __restrict__ tn, const int64_t* __restrict__ fn, int C,
                                                int kind, int avg, bool multilabel, float beta2,
                                                float* __restrict__ out, long long row, double* red) {
  const long long o = row * C;
  stat_reduce_body(
      [&](int k, long long& a, long long& b, long long& c, long long& d) {
        a = tp[o + k];
        b = fp[o + k];
        c = tn[o + k];
        d = fn[o + k];
      },
      C, kind, avg, multilabel, beta2, avg == kNone ? out + o : out + row, red);
}

// ---------------------------------------------------------------------------------- confusion-matrix family
// Jaccard / Cohen kappa / MCC of a [C, C] int64 matrix (reference F/classification/{jaccard,cohen_kappa,
// matthews_corrcoef}.py `_*_reduce`, including MCC's degenerate binary cases).  sm: 3*C doubles; red: 4 doubles.
enum CmKind : int { kJaccard = 0, kKappa = 1, kMcc = 2 };
enum KappaW : int { kWNone = 0, kWLinear = 1, kWQuadratic = 2 };

__device__ __forceinline__ void confmat_reduce_block(const int64_t* __restrict__ cm, int C, int kind, int average,
                                                     int ignore, int kw, float* __restrict__ out, double* sm,
                                                     double* red) {
  double* rows = sm;
  double* cols = sm + C;
  double* diag = sm + 2 * C;
  for (int i = threadIdx.x; i < C; i += kThreads) {
    double r = 0.0, c = 0.0;
    for (int j = 0; j < C; ++j) {
      r += static_cast<double>(cm[static_cast<long long>(i) * C + j]);
      c += static_cast<double>(cm[static_cast<long long>(j) * C + i]);
    }
    rows[i] = r;
    cols[i] = c;
    diag[i] = static_cast<double>(cm[static_cast<long long>(i) * C + i]);
  }
  __syncthreads();

  if (kind == kJaccard) {
    const bool drop = ignore >= 0 && ignore < C;
    double tp_sum = 0.0, un_sum = 0.0, wsum = 0.0, wiou = 0.0;
    for (int i = threadIdx.x; i < C; i += kThreads) {
      const double tp = diag[i], un = rows[i] + cols[i] - tp;
      const double iou = tp / (un == 0.0 ? 1.0 : un);
      out[i] = static_cast<float>(iou);
      tp_sum += tp;
      un_sum += (drop && i == ignore) ? 0.0 : un;
      double w = average == kWeighted ? rows[i] : 1.0;
      if (average == kMacro && ((drop && i == ignore) || rows[i] + cols[i] == 0.0)) w = 0.0;
      wsum += w;
      wiou += w * iou;
    }
    tp_sum = block_sum(tp_sum, red);
    un_sum = block_sum(un_sum, red);
    wsum = block_sum(wsum, red);
    wiou = block_sum(wiou, red);
    if (threadIdx.x == 0) {
      out[C] = average == kMicro ? static_cast<float>(tp_sum / (un_sum == 0.0 ? 1.0 : un_sum))
                                 : static_cast<float>(wiou / wsum);  // 0/0 -> nan, as ((w * iou) / w.sum()).sum()
    }
    return;
  }

  double n = 0.0;
  for (int i = threadIdx.x; i < C; i += kThreads) n += rows[i];
  n = block_sum(n, red);

  if (kind == kKappa) {
    // 1 - sum(W * O) / sum(W * E),  E_ij = rows_i cols_j / n
    double wo = 0.0, we = 0.0;
    for (long long e = threadIdx.x; e < static_cast<long long>(C) * C; e += kThreads) {
      const int i = static_cast<int>(e / C), j = static_cast<int>(e - static_cast<long long>(i) * C);
      const double d = static_cast<double>(i - j);
      const double w = kw == kWNone ? (i == j ? 0.0 : 1.0) : (kw == kWLinear ? fabs(d) : d * d);
      wo += w * static_cast<double>(cm[e]);
      we += w * rows[i] * cols[j] / n;
    }
    wo = block_sum(wo, red);
    we = block_sum(we, red);
    if (threadIdx.x == 0) out[0] = static_cast<float>(1.0 - wo / we);
    return;
  }

  // MCC (Gorodkin R_K), with the reference's binary special cases
  double tk_pk = 0.0, pk2 = 0.0, tk2 = 0.0, correct = 0.0;
  for (int i = threadIdx.x; i < C; i += kThreads) {
    tk_pk += rows[i] * cols[i];
    pk2 += cols[i] * cols[i];
    tk2 += rows[i] * rows[i];
    correct += diag[i];
  }
  tk_pk = block_sum(tk_pk, red);
  pk2 = block_sum(pk2, red);
  tk2 = block_sum(tk2, red);
  correct = block_sum(correct, red);
  if (threadIdx.x != 0) return;
  const bool binary = C == 2;
  if (binary) {
    const double tn = static_cast<double>(cm[0]), fp = static_cast<double>(cm[1]);
    const double fn = static_cast<double>(cm[2]), tp = static_cast<double>(cm[3]);
    if (tp + tn != 0.0 && fp + fn == 0.0) {
      out[0] = 1.f;
      return;
    }
    if (tp + tn == 0.0 && fp + fn != 0.0) {
      out[0] = -1.f;
      return;
    }
  }
  double numer = correct * n - tk_pk;
  double denom = (n * n - pk2) * (n * n - tk2);
  if (denom == 0.0) {
    if (!binary) {
      out[0] = 0.f;
      return;
    }
    const double tn = static_cast<double>(cm[0]), fp = static_cast<double>(cm[1]);
    const double fn = static_cast<double>(cm[2]), tp = static_cast<double>(cm[3]);
    const double eps = 1.1920928955078125e-07;  // torch.finfo(float32).eps
    const double a = (tp == 0.0 || tn == 0.0) ? tp + tn : 0.0;
    const double b = (fp == 0.0 || fn == 0.0) ? fp + fn : 0.0;
    numer = sqrt(eps) * (a - b);
    denom = (tp + fp + eps) * (tp + fn + eps) * (tn + fp + eps) * (tn + fn + eps);
  }
  out[0] = static_cast<float>(numer / sqrt(denom));
}

// --------------------------------------------------------------------------------------- binned curve scores
// AUROC / AP of a binned [T, C, 2, 2] state.  Wave w scores classes w, w + 4, ...; lane-strided over thresholds +
// wave sum; then one wave reduces over classes.  out[0..C) = per-class score, out[C] = the reduced score;
// *nan_flag = 1 if any class is NaN.  sm: 2*C floats.
constexpr int kScoreAuroc = 0;
constexpr int kScoreAp = 1;

__device__ __forceinline__ float safe_div(long long a, long long b) {
  return static_cast<float>(a) / (b == 0 ? 1.f : static_cast<float>(b));
}

__device__ __forceinline__ void curve_score_block(const int64_t* __restrict__ st, int T, int C, int kind, int average,
                                                  float* __restrict__ out, int* __restrict__ nan_flag, float* sm) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave, nw = kThreads / kWave;
  auto at = [&](int t, int c, int a, int b) -> long long { return st[((static_cast<long long>(t) * C + c) * 2 + a) * 2 + b]; };
  for (int c = wave; c < C; c += nw) {
    float acc = 0.f;
    if (kind == kScoreAuroc) {
      // points i = 0..T-1 of the flipped curve: x_i = fpr(T-1-i), y_i = tpr(T-1-i); trapz over consecutive pairs
      for (int i = lane; i < T - 1; i += kWave) {
        const int t0 = T - 1 - i, t1 = T - 2 - i;
        const float x0 = safe_div(at(t0, c, 0, 1), at(t0, c, 0, 1) + at(t0, c, 0, 0));
        const float x1 = safe_div(at(t1, c, 0, 1), at(t1, c, 0, 1) + at(t1, c, 0, 0));
        const float y0 = safe_div(at(t0, c, 1, 1), at(t0, c, 1, 1) + at(t0, c, 1, 0));
        const float y1 = safe_div(at(t1, c, 1, 1), at(t1, c, 1, 1) + at(t1, c, 1, 0));
        acc += (x1 - x0) * (y1 + y0) / 2.f;
      }
    } else {
      // AP = -sum_k (recall[k+1] - recall[k]) * precision[k], with the appended point (precision 1, recall 0)
      for (int k = lane; k < T; k += kWave) {
        const long long tp = at(k, c, 1, 1), fp = at(k, c, 0, 1), fn = at(k, c, 1, 0);
        const float prec = safe_div(tp, tp + fp), rec = safe_div(tp, tp + fn);
        float rec_next = 0.f;
        if (k + 1 < T) {
          const long long tp1 = at(k + 1, c, 1, 1), fn1 = at(k + 1, c, 1, 0);
          rec_next = safe_div(tp1, tp1 + fn1);
        }
        acc += (rec_next - rec) * prec;
      }
      acc = -acc;
    }
    acc = wave_sum(acc);
    if (lane == 0) {
      sm[c] = acc;
      sm[C + c] = static_cast<float>(at(0, c, 1, 0) + at(0, c, 1, 1));  // positives per class (weights)
      out[c] = acc;
    }
  }
  __syncthreads();
  if (wave == 0) {
    float sum = 0.f, wsum = 0.f, cnt = 0.f;
    int nan = 0;
    for (int c = lane; c < C; c += kWave) {
      const float r = sm[c];
      if (r != r) {
        nan = 1;
        continue;
      }
      sum += r;
      cnt += 1.f;
      wsum += sm[C + c];
    }
    sum = wave_sum(sum);
    cnt = wave_sum(cnt);
    wsum = wave_sum(wsum);
    nan = __any(nan);
    float wred = 0.f;
    if (average == 2) {
      const float denom = wsum == 0.f ? 1.f : wsum;
      for (int c = lane; c < C; c += kWave) {
        const float r = sm[c];
        if (r == r) wred += r * (sm[C + c] / denom);
      }
      wred = wave_sum(wred);
    }
    if (lane == 0) {
      out[C] = average == 2 ? wred : sum / cnt;
      *nan_flag = nan;
    }
  }
}

// ------------------------------------------------------------------------------ streaming regression ratios
// Explained variance / R^2 / Pearson / concordance from running sums (reference regression/{explained_variance,
// r2,pearson,concordance}.py `_*_compute`).  Arithmetic in the states' dtype T.  red: 4 T of LDS.
enum RegKind : int { kExplainedVariance = 0, kR2 = 1, kPearson = 2, kConcordance = 3 };
enum MultiOut : int { kRaw = 0, kUniform = 1, kVarianceWeighted = 2 };
enum NKind : int { kNScalar = 0, kNFloat = 1, kNDouble = 2, kNLong = 3 };

template <typename T>
__device__ __forceinline__ T load_n(const void* p, int kind, int idx, double scalar) {
  switch (kind) {
    case kNFloat: return static_cast<T>(static_cast<const float*>(p)[idx]);
    case kNDouble: return static_cast<T>(static_cast<const double*>(p)[idx]);
    case kNLong: return static_cast<T>(static_cast<const int64_t*>(p)[idx]);
    default: return static_cast<T>(scalar);
  }
}

template <typename T>
__device__ __forceinline__ void regression_compute_block(int kind, int k, const T* __restrict__ s0,
                                                         const T* __restrict__ s1, const T* __restrict__ s2,
                                                         const T* __restrict__ s3, const T* __restrict__ s4,
                                                         const void* __restrict__ n_ptr, int n_kind, int n_per_col,
                                                         double n_scalar, int multioutput, T bound,
                                                         T* __restrict__ out, T* red) {
  T num_sum = 0, w_sum = 0, wscore = 0;
  int low_var = 0;
  for (int c = threadIdx.x; c < k; c += kThreads) {
    const T n = load_n<T>(n_ptr, n_kind, n_per_col ? c : 0, n_scalar);
    T score = 0, weight = 0;
    if (kind == kExplainedVariance) {
      // s0 = sum_error, s1 = sum_squared_error, s2 = sum_target, s3 = sum_squared_target
      const T diff_avg = s0[c] / n;
      const T numer = s1[c] / n - diff_avg * diff_avg;
      const T tavg = s2[c] / n;
      const T denom = s3[c] / n - tavg * tavg;
      score = (numer != T(0) && denom != T(0)) ? T(1) - numer / denom : (numer != T(0) ? T(0) : T(1));
      weight = denom;
    } else if (kind == kR2) {
      // s0 = sum_squared_obs, s1 = sum_obs, s2 = rss; nonzero = !isclose(x, 0, atol=1e-4) (NaN counts as nonzero)
      const T mean = s1[c] / n;
      const T tss = s0[c] - s1[c] * mean;
      const T rss = s2[c];
      const bool nz_rss = !(fabs(rss) <= T(1e-4)), nz_tss = !(fabs(tss) <= T(1e-4));
      score = (nz_rss && nz_tss) ? T(1) - rss / tss : (nz_rss ? T(0) : T(1));
      weight = tss;
      low_var |= n < T(2) ? 1 : 0;  // R^2's flag slot: fewer than two samples (the reference raises)
    } else {
      // s0 = mean_x, s1 = mean_y, s2 = m2_x, s3 = m2_y, s4 = c_xy (sums of squared deviations)
      const T vx = s2[c] / (n - T(1)), vy = s3[c] / (n - T(1)), cxy = s4[c] / (n - T(1));
      low_var |= (vx < bound || vy < bound) ? 1 : 0;
      T corr = cxy / sqrt(vx * vy);
      corr = corr != corr ? corr : fmin(fmax(corr, T(-1)), T(1));
      if (kind == kPearson) {
        score = corr;
      } else {
        const T dm = s0[c] - s1[c];
        score = T(2) * corr * sqrt(vx) * sqrt(vy) / (vx + vy + dm * dm);
      }
    }
    out[c] = score;
    num_sum += score;
    w_sum += weight;
    wscore += weight * score;
  }
  if (multioutput != kRaw) {
    num_sum = block_sum(num_sum, red);
    w_sum = block_sum(w_sum, red);
    wscore = block_sum(wscore, red);
  }
  low_var = __syncthreads_or(low_var);
  if (threadIdx.x == 0) {
    out[k + 1] = low_var ? T(1) : T(0);
    if (multioutput == kUniform) out[k] = num_sum / static_cast<T>(k);
    else if (multioutput == kVarianceWeighted) out[k] = wscore / w_sum;
  }
}

// ------------------------------------------------------------------------------------------ element ratios
// out[i] = a[i] / b (b a scalar or per element; int64 b converted to a's dtype first, as ATen's true_divide does), then
// optionally sqrt: MSE / RMSE / MAE / ... compute (reference regression/{mse,mae}.py `_*_compute`).
template <typename T>
__device__ __forceinline__ void ratio_block(const T* __restrict__ a, const void* __restrict__ b, int b_kind,
                                            int b_per_elem, int k, int take_sqrt, T* __restrict__ out) {
  for (int i = threadIdx.x; i < k; i += kThreads) {
    const T d = load_n<T>(b, b_kind, b_per_elem ? i : 0, 0.0);
    const T r = a[i] / d;
    out[i] = take_sqrt ? sqrt(r) : r;
  }
}

// ---------------------------------------------------------------------------------------- stat-scores output
// StatScores compute() for global multidim_average (reference F/classification/stat_scores.py
// `_multiclass_stat_scores_compute`): res = [tp, fp, tn, fn, tp + fn] per class; micro -> int64 sums over classes,
// macro -> float32 mean over classes, none -> int64 [C, 5].  Integer-valued fp32 sums are exact below 2^24, so the
// macro mean is bit-identical to ATen's whatever the summation order.
__device__ __forceinline__ void stat_scores_block(const int64_t* __restrict__ tp, const int64_t* __restrict__ fp,
                                                  const int64_t* __restrict__ tn, const int64_t* __restrict__ fn,
                                                  int C, int avg, void* __restrict__ out, double* red) {
  if (avg == kNone) {
    int64_t* o = static_cast<int64_t*>(out);
    for (int c = threadIdx.x; c < C; c += kThreads) {
      o[5 * c] = tp[c];
      o[5 * c + 1] = fp[c];
      o[5 * c + 2] = tn[c];
      o[5 * c + 3] = fn[c];
      o[5 * c + 4] = tp[c] + fn[c];
    }
    return;
  }
  long long s[5] = {0, 0, 0, 0, 0};
  for (int c = threadIdx.x; c < C; c += kThreads) {
    s[0] += tp[c];
    s[1] += fp[c];
    s[2] += tn[c];
    s[3] += fn[c];
    s[4] += tp[c] + fn[c];
  }
  for (int j = 0; j < 5; ++j) {
    // exact: int64 partial sums travel through the double-typed LDS scratch bit-cast
    long long v = wave_sum_ll(s[j]);
    const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    __syncthreads();
    if (lane == 0) reinterpret_cast<long long*>(red)[wave] = v;
    __syncthreads();
    long long tot = 0;
    for (int w = 0; w < kThreads / kWave; ++w) tot += reinterpret_cast<long long*>(red)[w];
    s[j] = tot;
  }
  if (threadIdx.x == 0) {
    for (int j = 0; j < 5; ++j) {
      if (avg == kMicro) static_cast<int64_t*>(out)[j] = s[j];
      else static_cast<float*>(out)[j] = static_cast<float>(s[j]) * (1.f / static_cast<float>(C));  // ATen MeanOps
    }
  }
}

}  // namespace cbody
}  // namespace tm_amd
