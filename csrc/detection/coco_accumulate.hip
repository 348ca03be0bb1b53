// COCO accumulation for every (category, IoU threshold, area range, max-dets) at once.
//
// Reference: pycocotools COCOeval.accumulate as driven by S/detection/mean_ap.py:513-588 -- per (k, a, m) a Python
// loop that concatenates the per-image matches, a mergesort by score, float cumulative sums, the precision envelope
// (a reverse running max) and a searchsorted of the 101 recall thresholds.  The round-2 device version ran that as
// ~40 batched torch ops and a host sync per max-dets value (~10 ms at 512 images x 100 detections).
//
// Here ONE WAVE per (k, t, a, m) sweeps its category's detections (sorted by category, then score; `seg` offsets) in
// chunks of 64, a lane per detection (r05: one thread per (k, t, a, m) walked the ~640 detections of its category
// serially twice -- 745 us per compute at 512 images x 100 detections x COCO-80):
//   counting pass (forward): the included detections (rank below the max-dets value: pycocotools truncates each
//             image's list) and their true / false positive flags are wave ballots; popcounts give the totals;
//   main pass (backward, from the last chunk): a detection's counts are the totals minus the popcounts of the
//             included flags after it, pr = tp / (tp + fp + eps) is the same fp64 formula on the same integers, the
//             precision envelope is a suffix max (wave scan + the carry of the later chunks), and the recall
//             thresholds in (rc of the previous included detection, rc] -- exactly those whose first position with
//             rc >= threshold is this detection (searchsorted 'left') -- take its envelope value and score.
// The per-detection match flags of all (t, a) pairs are packed into two 64-bit words (true / false positive bits), so
// a chunk loads three words shared by every wave of the category (broadcast from cache).  Outputs go straight into
// precision / scores [T, R, K, A, M] and recall [T, K, A, M]; categories without non-ignored ground truth get -1.
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kMaxM = 8, kMaxR = 1024;
constexpr int kAccThreads = 256;

struct AccArgs {
  int T, A, M, K, R;
  int max_dets[kMaxM];
};

// #{r : r_thr[r] <= x} (r_thr ascending)
__device__ __forceinline__ int thr_count(const double* __restrict__ r_thr, int R, double x) {
  int lo = 0, hi = R;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (r_thr[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ double wave_suffix_max(double v, int lane) {
  // inclusive max over lanes >= lane
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double u = __shfl_down(v, o, kWave);
    if (lane + o < kWave) v = u > v ? u : v;
  }
  return v;
}

__global__ void __launch_bounds__(kAccThreads) coco_accumulate_kernel(const int64_t* __restrict__ tpb,
                                                                      const int64_t* __restrict__ fpb,
                                                                      const int64_t* __restrict__ rank,
                                                                      const double* __restrict__ score,
                                                                      const int64_t* __restrict__ seg,
                                                                      const double* __restrict__ npig,
                                                                      const double* __restrict__ r_thr, AccArgs args,
                                                                      double* __restrict__ precision,
                                                                      double* __restrict__ recall,
                                                                      double* __restrict__ scores) {
  const int T = args.T, A = args.A, M = args.M, K = args.K, R = args.R;
  const int lane = threadIdx.x & (kWave - 1);
  const long long gid = (static_cast<long long>(blockIdx.x) * kAccThreads + threadIdx.x) / kWave;  // wave-uniform
  if (gid >= static_cast<long long>(K) * T * A * M) return;
  const int m = static_cast<int>(gid % M);
  const int a = static_cast<int>((gid / M) % A);
  const int t = static_cast<int>((gid / (static_cast<long long>(M) * A)) % T);
  const int k = static_cast<int>(gid / (static_cast<long long>(M) * A * T));
  const int md = args.max_dets[m];
  const long long bit = 1LL << (t * A + a);
  const double np = npig[static_cast<long long>(a) * K + k];
  // output addressing: precision / scores [T, R, K, A, M], recall [T, K, A, M]
  const long long pr_base = ((static_cast<long long>(t) * R) * K + k) * A * M + static_cast<long long>(a) * M + m;
  const long long pr_stride_r = static_cast<long long>(K) * A * M;
  const long long rc_idx = ((static_cast<long long>(t) * K + k) * A + a) * M + m;
  if (np <= 0.0) {  // no non-ignored ground truth: pycocotools skips the category
    for (int r = lane; r < R; r += kWave) {
      precision[pr_base + r * pr_stride_r] = -1.0;
      scores[pr_base + r * pr_stride_r] = -1.0;
    }
    if (lane == 0) recall[rc_idx] = -1.0;
    return;
  }
  const long long s = seg[k], e = seg[k + 1];
  const unsigned long long below = (1ull << lane) - 1ull;  // lanes before this one
  // counting pass: included detections and their flags
  long long tp_tot = 0, fp_tot = 0, nd = 0;
  for (long long c0 = s; c0 < e; c0 += kWave) {
    const long long i = c0 + lane;
    const bool inc = i < e && rank[i] < md;
    const bool tpf = inc && (tpb[i] & bit), fpf = inc && (fpb[i] & bit);
    tp_tot += __popcll(__ballot(tpf));
    fp_tot += __popcll(__ballot(fpf));
    nd += __popcll(__ballot(inc));
  }
  const int hi_last = nd ? thr_count(r_thr, R, static_cast<double>(tp_tot) / np) : 0;
  if (lane == 0) recall[rc_idx] = nd ? static_cast<double>(tp_tot) / np : 0.0;
  // thresholds above the last recall get 0 precision / score
  for (int q = hi_last + lane; q < R; q += kWave) {
    precision[pr_base + q * pr_stride_r] = 0.0;
    scores[pr_base + q * pr_stride_r] = 0.0;
  }
  if (hi_last == 0) return;
  // main pass, backward: suffix counts, envelope, each detection's threshold range
  const double eps = 2.220446049250313e-16;  // np.spacing(1)
  long long tp_after = 0, fp_after = 0, nd_after = 0;  // included flags / detections in later chunks
  double env_after = 0.0;
  const long long nchunks = (e - s + kWave - 1) / kWave;
  for (long long ci = nchunks - 1; ci >= 0; --ci) {
    const long long i = s + ci * kWave + lane;
    const bool inc = i < e && rank[i] < md;
    const bool tpf = inc && (tpb[i] & bit), fpf = inc && (fpb[i] & bit);
    const unsigned long long btp = __ballot(tpf), bfp = __ballot(fpf), binc = __ballot(inc);
    // counts up to and including this detection = totals - flags after it
    const long long tp_i = tp_tot - tp_after - __popcll(btp & ~below & ~(1ull << lane));
    const long long fp_i = fp_tot - fp_after - __popcll(bfp & ~below & ~(1ull << lane));
    const double p = inc ? static_cast<double>(tp_i) / (static_cast<double>(tp_i) + static_cast<double>(fp_i) + eps)
                         : 0.0;
    double env = wave_suffix_max(p, lane);
    env = env > env_after ? env : env_after;
    if (inc) {
      const double rc = static_cast<double>(tp_i) / np;
      const double rc_prev = static_cast<double>(tp_i - (tpf ? 1 : 0)) / np;
      // (the previous included detection's recall; before the first included detection of the category nothing
      // was assigned, whatever the thresholds at recall 0)
      const bool first = nd - nd_after - __popcll(binc & ~below) == 0;  // no included detection before it
      const int lo = first ? 0 : thr_count(r_thr, R, rc_prev);
      const int hi = thr_count(r_thr, R, rc);
      const double sc = score[i];
      for (int q = lo; q < hi; ++q) {
        precision[pr_base + q * pr_stride_r] = env;
        scores[pr_base + q * pr_stride_r] = sc;
      }
    }
    tp_after += __popcll(btp);
    fp_after += __popcll(bfp);
    nd_after += __popcll(binc);
    env_after = __shfl(env, 0, kWave);
  }
}

// per detection: bit q (= t * A + a) of tpb / fpb set when the detection is a true / false positive of
// (threshold t, area a) -- matched / unmatched and not ignored; reads the matcher's [T * A, D] flags coalesced
__global__ void __launch_bounds__(256) coco_pack_kernel(const uint8_t* __restrict__ match,
                                                        const uint8_t* __restrict__ ig, long long D, int TA,
                                                        int64_t* __restrict__ tpb, int64_t* __restrict__ fpb) {
  const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= D) return;
  long long tp = 0, fp = 0;
  for (int q = 0; q < TA; ++q) {
    const long long e = static_cast<long long>(q) * D + i;
    if (ig[e]) continue;
    if (match[e]) tp |= 1LL << q;
    else fp |= 1LL << q;
  }
  tpb[i] = tp;
  fpb[i] = fp;
}

// coco_pack_kernel in accumulation order, fused with the gathers around it: sorted position i takes detection
// j = o[i] (o: the (category, score) sort permutation of the matcher-order arrays) -- its true / false positive bit
// words, rank and score -- and the category segment starts seg [K + 1] (seg[c] = first position whose category is
// >= c; category K = not on the axis, sorted last) come from the boundaries between neighbours.  One launch instead
// of pack + five gathers + histogram + scan.
__global__ void __launch_bounds__(256) coco_pack_sorted_kernel(
    const uint8_t* __restrict__ match, const uint8_t* __restrict__ ig, const int64_t* __restrict__ o,
    const int64_t* __restrict__ rank_v, const double* __restrict__ score_v, const int64_t* __restrict__ cls_v,
    long long D, int TA, int K, int64_t* __restrict__ tpb, int64_t* __restrict__ fpb, int64_t* __restrict__ rank_s,
    double* __restrict__ score_s, int64_t* __restrict__ seg) {
  const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= D) return;
  const long long j = o[i];
  long long tp = 0, fp = 0;
  for (int q = 0; q < TA; ++q) {
    const long long e = static_cast<long long>(q) * D + j;
    if (ig[e]) continue;
    if (match[e]) tp |= 1LL << q;
    else fp |= 1LL << q;
  }
  tpb[i] = tp;
  fpb[i] = fp;
  rank_s[i] = rank_v[j];
  score_s[i] = score_v[j];
  const long long c = cls_v[j];
  const long long cp = i > 0 ? cls_v[o[i - 1]] : -1;
  for (long long x = cp + 1; x <= c && x <= K; ++x) seg[x] = i;
  if (i == D - 1)
    for (long long x = c + 1; x <= K; ++x) seg[x] = D;
}

// ------------------------------------------------------------------------------------------------ summary
// Every number COCOeval.summarize and the per-class mAP / mAR need, from precision [T, R, K, A, M] and recall
// [T, K, A, M], in ONE launch (it replaced ~10 masked-reduction launches over the 7.7 MB precision tensor plus a
// concatenation): sums and counts of the defined (> -1) entries.  Precision blocks: one per (t, group of kSumKC
// categories): for every r the group's kSumKC * A * M values are contiguous, so a thread keeps ONE (category, a, m)
// column over the whole R walk (sums in registers), the block folds its threads per column, then writes its
// categories' per-class sums at (area 0, max-dets m_ap) and its partial (t, a, m) sums.  Recall blocks: one per t.
// Every output is written exactly once, in a fixed order (deterministic); the host adds the partials.
constexpr int kSumThreads = 256;
constexpr int kSumKC = 4;  // categories per precision block

__global__ void __launch_bounds__(kSumThreads) coco_summary_kernel(const double* __restrict__ prec,
                                                                   const double* __restrict__ rec,
                                                                   const double* __restrict__ cprec,
                                                                   const double* __restrict__ crec, int T, int R, int K,
                                                                   int AM, int M, int m_ap, double* __restrict__ out) {
  __shared__ double s_sum[kSumThreads], s_cnt[kSumThreads], s_cls[kSumThreads], s_ccnt[kSumThreads];
  const int tid = threadIdx.x;
  const int NB = (K + kSumKC - 1) / kSumKC;
  const long long TAM = static_cast<long long>(T) * AM, TK = static_cast<long long>(T) * K;
  double* psp = out;                                    // [T][NB][AM]
  double* pcp = psp + static_cast<long long>(T) * NB * AM;  // [T][NB][AM]
  double* sr = pcp + static_cast<long long>(T) * NB * AM;   // [T][AM]
  double* cr = sr + TAM;
  double* mps = cr + TAM;  // [T][K]
  double* mpc = mps + TK;
  double* mrs = mpc + TK;
  double* mrc = mrs + TK;
  const int b = blockIdx.x;
  if (b < T * NB) {
    const int t = b / NB, kb = b - t * NB;
    const int k0 = kb * kSumKC, kc = min(kSumKC, K - k0);
    const int W = kc * AM;          // contiguous values per r
    const int G = kSumThreads / W;  // threads per column (>= 2: A * M <= 32)
    const int c = tid % W, g = tid / W;
    double sum = 0.0, cnt = 0.0, csum = 0.0, ccnt = 0.0;
    const bool cls_col = m_ap >= 0 && (c % AM) == m_ap;  // (area 0: column m_ap of its category)
    if (g < G) {
      for (int r = g; r < R; r += G) {
        const long long e = ((static_cast<long long>(t) * R + r) * K + k0) * AM + c;
        const double v = prec[e];
        if (v > -1.0) {
          sum += v;
          cnt += 1.0;
        }
        if (cls_col) {
          const double w = cprec[e];
          if (w > -1.0) {
            csum += w;
            ccnt += 1.0;
          }
        }
      }
    }
    s_sum[tid] = sum;
    s_cnt[tid] = cnt;
    s_cls[tid] = csum;
    s_ccnt[tid] = ccnt;
    __syncthreads();
    if (tid < W) {  // fold the G threads of column tid, in order
      for (int j = 1; j < G; ++j) {
        s_sum[tid] += s_sum[tid + j * W];
        s_cnt[tid] += s_cnt[tid + j * W];
        s_cls[tid] += s_cls[tid + j * W];
        s_ccnt[tid] += s_ccnt[tid + j * W];
      }
    }
    __syncthreads();
    if (tid < AM) {  // this block's partial (t, a, m) sums: its categories in order
      double a = 0.0, n = 0.0;
      for (int kk = 0; kk < kc; ++kk) {
        a += s_sum[kk * AM + tid];
        n += s_cnt[kk * AM + tid];
      }
      psp[(static_cast<long long>(t) * NB + kb) * AM + tid] = a;
      pcp[(static_cast<long long>(t) * NB + kb) * AM + tid] = n;
    }
    if (tid < kc) {
      const long long o = static_cast<long long>(t) * K + k0 + tid;
      mps[o] = m_ap >= 0 ? s_cls[tid * AM + m_ap] : 0.0;
      mpc[o] = m_ap >= 0 ? s_ccnt[tid * AM + m_ap] : 0.0;
    }
  } else {
    // recall slab t [K, A*M]: per (a, m) over k (a thread per column, as above), and per category the class recall at
    // (area 0, the last max-dets)
    const int t = b - T * NB;
    const int G = kSumThreads / AM;
    const int c = tid % AM, g = tid / AM;
    double sum = 0.0, cnt = 0.0;
    if (g < G) {
      for (int k = g; k < K; k += G) {
        const double v = rec[(static_cast<long long>(t) * K + k) * AM + c];
        if (v > -1.0) {
          sum += v;
          cnt += 1.0;
        }
      }
    }
    s_sum[tid] = sum;
    s_cnt[tid] = cnt;
    for (int k = tid; k < K; k += kSumThreads) {
      const double v = crec[(static_cast<long long>(t) * K + k) * AM + (M - 1)];
      const bool ok = v > -1.0;
      mrs[static_cast<long long>(t) * K + k] = ok ? v : 0.0;
      mrc[static_cast<long long>(t) * K + k] = ok ? 1.0 : 0.0;
    }
    __syncthreads();
    if (tid < AM) {
      double a = 0.0, n = 0.0;
      for (int j = 0; j < G; ++j) {
        a += s_sum[tid + j * AM];
        n += s_cnt[tid + j * AM];
      }
      sr[static_cast<long long>(t) * AM + tid] = a;
      cr[static_cast<long long>(t) * AM + tid] = n;
    }
  }
}

}  // namespace

// match / ig uint8 [T, A, D] (coco_match's outputs) -> packed true / false positive bits int64 [D] each
std::tuple<at::Tensor, at::Tensor> coco_pack_bits(const at::Tensor& match, const at::Tensor& ig) {
  TM_CHECK_CUDA(match);
  TM_SAME_DEVICE(match, ig);
  TM_CHECK_CONTIG(match);
  TM_CHECK_CONTIG(ig);
  TORCH_CHECK(match.scalar_type() == at::kByte && ig.scalar_type() == at::kByte && match.dim() == 3 &&
                  ig.sizes() == match.sizes(),
              "coco_pack_bits: uint8 [T, A, D] flags");
  const long long TA = match.size(0) * match.size(1), D = match.size(2);
  TORCH_CHECK(TA <= 63, "coco_pack_bits: T * A <= 63");
  at::Tensor tpb = at::empty({D}, match.options().dtype(at::kLong));
  at::Tensor fpb = at::empty({D}, match.options().dtype(at::kLong));
  if (D > 0)
    hipLaunchKernelGGL(coco_pack_kernel, dim3(static_cast<unsigned>((D + 255) / 256)), dim3(256), 0, stream(),
                       match.data_ptr<uint8_t>(), ig.data_ptr<uint8_t>(), D, static_cast<int>(TA),
                       tpb.data_ptr<int64_t>(), fpb.data_ptr<int64_t>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {tpb, fpb};
}

// match / ig uint8 [T, A, D] in matcher order, o int64 [D] the accumulation order, rank / cls int64 and score fp64 [D]
// in matcher order -> (tpb, fpb, rank, score) in accumulation order and seg int64 [K + 1]
std::vector<at::Tensor> coco_pack_sorted(const at::Tensor& match, const at::Tensor& ig, const at::Tensor& o,
                                         const at::Tensor& rank, const at::Tensor& score, const at::Tensor& cls,
                                         int64_t K) {
  TM_CHECK_CUDA(match);
  for (const at::Tensor* x : {&ig, &o, &rank, &score, &cls}) {
    TM_SAME_DEVICE(match, *x);
    TM_CHECK_CONTIG(*x);
  }
  TM_CHECK_CONTIG(match);
  TORCH_CHECK(match.scalar_type() == at::kByte && ig.scalar_type() == at::kByte && match.dim() == 3 &&
                  ig.sizes() == match.sizes(),
              "coco_pack_sorted: uint8 [T, A, D] flags");
  const long long TA = match.size(0) * match.size(1), D = match.size(2);
  TORCH_CHECK(TA <= 63, "coco_pack_sorted: T * A <= 63");
  TORCH_CHECK(o.scalar_type() == at::kLong && rank.scalar_type() == at::kLong && cls.scalar_type() == at::kLong &&
                  score.scalar_type() == at::kDouble && o.numel() == D && rank.numel() == D && cls.numel() == D &&
                  score.numel() == D,
              "coco_pack_sorted: o / rank / cls int64 [D], score fp64 [D]");
  auto l = match.options().dtype(at::kLong);
  at::Tensor tpb = at::empty({D}, l), fpb = at::empty({D}, l), rank_s = at::empty({D}, l);
  at::Tensor score_s = at::empty({D}, match.options().dtype(at::kDouble));
  at::Tensor seg = at::empty({K + 1}, l);
  if (D == 0) {
    seg.zero_();
  } else {
    hipLaunchKernelGGL(coco_pack_sorted_kernel, dim3(static_cast<unsigned>((D + 255) / 256)), dim3(256), 0, stream(),
                       match.data_ptr<uint8_t>(), ig.data_ptr<uint8_t>(), o.data_ptr<int64_t>(),
                       rank.data_ptr<int64_t>(), score.data_ptr<double>(), cls.data_ptr<int64_t>(), D,
                       static_cast<int>(TA), static_cast<int>(K), tpb.data_ptr<int64_t>(), fpb.data_ptr<int64_t>(),
                       rank_s.data_ptr<int64_t>(), score_s.data_ptr<double>(), seg.data_ptr<int64_t>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
  return {tpb, fpb, rank_s, score_s, seg};
}

// tpb / fpb int64 [D]: per detection (sorted by category, then score) bit t * A + a set for a true / false positive of
// (IoU threshold t, area range a); rank int64 [D] (rank within its image and category); score fp64 [D]; seg int64
// [K + 1]; npig fp64 [A, K]; r_thr fp64 [R]; max_dets int64 [M] (CPU); outputs fp64 precision / scores [T, R, K, A, M],
// recall [T, K, A, M].
void coco_accumulate(const at::Tensor& tpb, const at::Tensor& fpb, const at::Tensor& rank, const at::Tensor& score,
                     const at::Tensor& seg, const at::Tensor& npig, const at::Tensor& r_thr,
                     const at::Tensor& max_dets, int64_t T, at::Tensor precision, at::Tensor recall,
                     at::Tensor scores) {
  TM_CHECK_CUDA(tpb);
  for (const at::Tensor* x : {&fpb, &rank, &score, &seg, &npig, &r_thr}) {
    TM_SAME_DEVICE(tpb, *x);
    TM_CHECK_CONTIG(*x);
  }
  TM_SAME_DEVICE(tpb, precision);
  TM_SAME_DEVICE(tpb, recall);
  TM_SAME_DEVICE(tpb, scores);
  TM_CHECK_CONTIG(tpb);
  const long long D = tpb.numel();
  TORCH_CHECK(tpb.scalar_type() == at::kLong && fpb.scalar_type() == at::kLong && rank.scalar_type() == at::kLong &&
                  fpb.numel() == D && rank.numel() == D,
              "coco_accumulate: tpb / fpb / rank must be int64 [D]");
  TORCH_CHECK(score.scalar_type() == at::kDouble && score.numel() == D, "coco_accumulate: score fp64 [D]");
  TORCH_CHECK(npig.scalar_type() == at::kDouble && npig.dim() == 2, "coco_accumulate: npig fp64 [A, K]");
  const int A = static_cast<int>(npig.size(0)), K = static_cast<int>(npig.size(1));
  TORCH_CHECK(seg.scalar_type() == at::kLong && seg.numel() == K + 1, "coco_accumulate: seg int64 [K + 1]");
  TORCH_CHECK(r_thr.scalar_type() == at::kDouble, "coco_accumulate: r_thr fp64");
  const int R = static_cast<int>(r_thr.numel());
  TORCH_CHECK(!max_dets.is_cuda() && max_dets.scalar_type() == at::kLong, "coco_accumulate: max_dets CPU int64");
  const int M = static_cast<int>(max_dets.numel());
  TORCH_CHECK(M >= 1 && M <= kMaxM && R >= 1 && R <= kMaxR && T >= 1 && T * A <= 63,
              "coco_accumulate: 1 <= M <= 8, 1 <= R <= 1024, T * A <= 63");
  TORCH_CHECK(D < (1LL << 31), "coco_accumulate: too many detections");
  const long long nthr = static_cast<long long>(K) * T * A * M;
  TORCH_CHECK(precision.scalar_type() == at::kDouble && precision.is_contiguous() &&
                  precision.numel() == static_cast<long long>(T) * R * K * A * M &&
                  scores.scalar_type() == at::kDouble && scores.is_contiguous() && scores.numel() == precision.numel() &&
                  recall.scalar_type() == at::kDouble && recall.is_contiguous() && recall.numel() == nthr,
              "coco_accumulate: outputs must be fp64 [T, R, K, A, M] / [T, K, A, M]");
  if (nthr == 0) return;
  AccArgs args{};
  args.T = static_cast<int>(T);
  args.A = A;
  args.M = M;
  args.K = K;
  args.R = R;
  const int64_t* mdp = max_dets.data_ptr<int64_t>();
  for (int i = 0; i < M; ++i) args.max_dets[i] = static_cast<int>(std::min<int64_t>(mdp[i], 1 << 30));
  constexpr int kWavesPerBlock = kAccThreads / kWave;
  const unsigned blocks = static_cast<unsigned>((nthr + kWavesPerBlock - 1) / kWavesPerBlock);
  hipLaunchKernelGGL(coco_accumulate_kernel, dim3(blocks), dim3(kAccThreads), 0, stream(), tpb.data_ptr<int64_t>(),
                     fpb.data_ptr<int64_t>(), rank.data_ptr<int64_t>(), score.data_ptr<double>(),
                     seg.data_ptr<int64_t>(), npig.data_ptr<double>(), r_thr.data_ptr<double>(), args,
                     precision.data_ptr<double>(), recall.data_ptr<double>(), scores.data_ptr<double>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}


// The summary sums of coco_summary_kernel as one fp64 vector: psp, pcp [T, NB, A*M] (partial precision sums / counts
// of the defined entries per (t, category group of 4, a, m)), sr, cr [T, A*M] (recall over K), then mps, mpc, mrs, mrc
// [T, K] (per-category precision sums / counts at (area 0, max-dets m_ap; m_ap < 0: zeros) and recall at (area 0, last
// max-dets)).  cprec / crec: the per-class evaluation (the same tensors unless micro averaging evaluated twice).
at::Tensor coco_summary(const at::Tensor& prec, const at::Tensor& rec, const at::Tensor& cprec, const at::Tensor& crec,
                        int64_t m_ap) {
  TM_CHECK_CUDA(prec);
  for (const at::Tensor* x : {&rec, &cprec, &crec}) {
    TM_SAME_DEVICE(prec, *x);
    TM_CHECK_CONTIG(*x);
    TORCH_CHECK(x->scalar_type() == at::kDouble, "coco_summary: fp64 tensors");
  }
  TM_CHECK_CONTIG(prec);
  TORCH_CHECK(prec.scalar_type() == at::kDouble && prec.dim() == 5 && rec.dim() == 4 && cprec.sizes() == prec.sizes() &&
                  crec.sizes() == rec.sizes(),
              "coco_summary: precision [T, R, K, A, M], recall [T, K, A, M]");
  const int T = static_cast<int>(prec.size(0)), R = static_cast<int>(prec.size(1)), K = static_cast<int>(prec.size(2));
  const int A = static_cast<int>(prec.size(3)), M = static_cast<int>(prec.size(4));
  TORCH_CHECK(rec.size(0) == T && rec.size(1) == K && rec.size(2) == A && rec.size(3) == M, "coco_summary: shapes");
  TORCH_CHECK(A * M >= 1 && A * M * kSumKC <= kSumThreads / 2 && m_ap < M, "coco_summary: A * M <= 32");
  const int NB = (K + kSumKC - 1) / kSumKC;
  const long long TAM = static_cast<long long>(T) * A * M, TK = static_cast<long long>(T) * K;
  at::Tensor out = at::empty({2 * NB * TAM + 2 * TAM + 4 * TK}, prec.options());
  if (T == 0 || K == 0) return out.zero_();
  hipLaunchKernelGGL(coco_summary_kernel, dim3(T * NB + T), dim3(kSumThreads), 0, stream(), prec.data_ptr<double>(),
                     rec.data_ptr<double>(), cprec.data_ptr<double>(), crec.data_ptr<double>(), T, R, K, A * M, M,
                     static_cast<int>(m_ap), out.data_ptr<double>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("coco_pack_bits(Tensor match, Tensor ig) -> (Tensor, Tensor)");
  m.def("coco_pack_sorted(Tensor match, Tensor ig, Tensor o, Tensor rank, Tensor score, Tensor cls, int K) -> Tensor[]");
  m.def("coco_summary(Tensor prec, Tensor rec, Tensor cprec, Tensor crec, int m_ap) -> Tensor");
  m.def(
      "coco_accumulate(Tensor tpb, Tensor fpb, Tensor rank, Tensor score, Tensor seg, Tensor npig, Tensor r_thr, "
      "Tensor max_dets, int T, Tensor(a!) precision, Tensor(b!) recall, Tensor(c!) scores) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("coco_pack_bits", &coco_pack_bits);
  m.impl("coco_pack_sorted", &coco_pack_sorted);
  m.impl("coco_accumulate", &coco_accumulate);
  m.impl("coco_summary", &coco_summary);
}

}  // namespace tm_amd
