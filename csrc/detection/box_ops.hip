// Pairwise box-overlap family (IoU / GIoU / DIoU / CIoU) and the COCO greedy matcher used by MeanAveragePrecision.
//
// box_pairwise: reference F/detection/{iou,giou,diou,ciou}.py call torchvision.ops.{box_iou, generalized_box_iou,
// distance_box_iou, complete_box_iou}; here one kernel computes any of the four for an N x M grid (or for N aligned
// pairs), one thread per pair, boxes in xyxy.
//
// coco_match: reference S/detection/mean_ap.py hands everything to pycocotools COCOeval on the host (per image, per
// category, per area range, per IoU threshold Python/C loops).  Here every (image x category group, area range,
// IoU threshold) greedy matching problem is one thread: detections are pre-sorted by score (per group, truncated to
// the largest max-detections), ground truths keep annotation order, the "non-ignored first" COCO ordering is realised
// as two passes, IoU (COCO bbox definition, fp64, crowd => intersection / detection area) is evaluated on the fly.
// Outputs per detection: matched flag and ignore flag for every (threshold, area range).
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

enum BoxOp : int { kIoU = 0, kGIoU = 1, kDIoU = 2, kCIoU = 3 };

template <typename acc_t>
__device__ __forceinline__ acc_t pair_value(const acc_t* a, const acc_t* b, int op) {
  // a = pred xyxy, b = target xyxy
  const acc_t area_a = (a[2] - a[0]) * (a[3] - a[1]);
  const acc_t area_b = (b[2] - b[0]) * (b[3] - b[1]);
  const acc_t iw = max(min(a[2], b[2]) - max(a[0], b[0]), acc_t(0));
  const acc_t ih = max(min(a[3], b[3]) - max(a[1], b[1]), acc_t(0));
  const acc_t inter = iw * ih;
  const acc_t uni = area_a + area_b - inter;
  const acc_t iou = inter / uni;
  if (op == kIoU) return iou;
  const acc_t cw = max(a[2], b[2]) - min(a[0], b[0]);
  const acc_t ch = max(a[3], b[3]) - min(a[1], b[1]);
  if (op == kGIoU) {
    const acc_t area_c = cw * ch;
    return iou - (area_c - uni) / area_c;
  }
  const acc_t eps = acc_t(1e-7);
  const acc_t diag = cw * cw + ch * ch + eps;
  const acc_t dx = (a[0] + a[2]) / 2 - (b[0] + b[2]) / 2;
  const acc_t dy = (a[1] + a[3]) / 2 - (b[1] + b[3]) / 2;
  const acc_t diou = iou - (dx * dx + dy * dy) / diag;
  if (op == kDIoU) return diou;
  const acc_t wa = a[2] - a[0], ha = a[3] - a[1], wb = b[2] - b[0], hb = b[3] - b[1];
  const acc_t dv = atan(wb / hb) - atan(wa / ha);
  const acc_t v = acc_t(4.0 / (M_PI * M_PI)) * dv * dv;
  const acc_t alpha = v / (1 - iou + v + eps);
  return diou - alpha * v;
}

template <typename scalar_t, typename acc_t>
__global__ void __launch_bounds__(256) box_pairwise_kernel(const scalar_t* __restrict__ a,
                                                           const scalar_t* __restrict__ b, int n, int m, int op,
                                                           bool aligned, scalar_t* __restrict__ out) {
  const long long total = aligned ? n : static_cast<long long>(n) * m;
  for (long long idx = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; idx < total;
       idx += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long i = aligned ? idx : idx / m;
    const long long j = aligned ? idx : idx % m;
    acc_t pa[4], pb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pa[k] = static_cast<acc_t>(to_f32(a[i * 4 + k]));
      pb[k] = static_cast<acc_t>(to_f32(b[j * 4 + k]));
    }
    out[idx] = static_cast<scalar_t>(pair_value<acc_t>(pa, pb, op));
  }
}

template <>
__global__ void __launch_bounds__(256) box_pairwise_kernel<double, double>(const double* __restrict__ a,
                                                                           const double* __restrict__ b, int n, int m,
                                                                           int op, bool aligned,
                                                                           double* __restrict__ out) {
  const long long total = aligned ? n : static_cast<long long>(n) * m;
  for (long long idx = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; idx < total;
       idx += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long i = aligned ? idx : idx / m;
    const long long j = aligned ? idx : idx % m;
    out[idx] = pair_value<double>(a + i * 4, b + j * 4, op);
  }
}

// Ragged batch of images (IntersectionOverUnion & co. update): block i computes image i's [n_i, m_i] matrix into its
// slice of one flat output, with the reference's two in-place masks fused (F/detection/iou.py `_iou_update`:
// values below iou_threshold -> invalid; S/detection/iou.py:191-193 respect_labels: label mismatch -> invalid).
// One launch per update instead of one box_pairwise + 2 masked writes per image.
template <typename scalar_t, typename acc_t>
__global__ void __launch_bounds__(256) box_pairwise_ragged_kernel(
    const scalar_t* __restrict__ a, const scalar_t* __restrict__ b, const int64_t* __restrict__ a_off,
    const int64_t* __restrict__ b_off, const int64_t* __restrict__ o_off, const int64_t* __restrict__ a_lab,
    const int64_t* __restrict__ b_lab, int op, bool has_thr, acc_t thr, acc_t invalid, scalar_t* __restrict__ out) {
  const int img = blockIdx.x;
  const long long a0 = a_off[img], b0 = b_off[img], o0 = o_off[img];
  const long long m = b_off[img + 1] - b0;
  const long long total = o_off[img + 1] - o0;
  for (long long e = threadIdx.x; e < total; e += blockDim.x) {
    const long long i = a0 + e / m, j = b0 + e % m;
    acc_t pa[4], pb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pa[k] = static_cast<acc_t>(a[i * 4 + k]);
      pb[k] = static_cast<acc_t>(b[j * 4 + k]);
    }
    acc_t v = pair_value<acc_t>(pa, pb, op);
    if (has_thr && v < thr) v = invalid;
    if (a_lab != nullptr && a_lab[i] != b_lab[j]) v = invalid;
    out[o0 + e] = static_cast<scalar_t>(v);
  }
}

// compute() of the IoU family over the flat values of every image: one block per image; column j of image i belongs
// to class classes[k] == gt_lab[b_off[i] + j].  Sums (fp64) and counts of the valid (!= invalid) values, per class
// (slot k < K, LDS-privatised per block) and over everything (slot K).  Replaces the reference's per-image boolean
// indexing and per-class x per-image double loop (S/detection/iou.py:205-221).
template <typename scalar_t>
__global__ void __launch_bounds__(256) iou_class_reduce_kernel(
    const scalar_t* __restrict__ vals, const int64_t* __restrict__ o_off, const int64_t* __restrict__ b_off,
    const int64_t* __restrict__ gt_lab, const int64_t* __restrict__ classes, int K, double invalid,
    double* __restrict__ sums, int64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* lsum = reinterpret_cast<double*>(smem);
  int* lcnt = reinterpret_cast<int*>(lsum + K);
  const bool per_class = K > 0;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    lsum[k] = 0.0;
    lcnt[k] = 0;
  }
  __syncthreads();
  const int img = blockIdx.x;
  const long long o0 = o_off[img], b0 = b_off[img];
  const long long m = b_off[img + 1] - b0;
  const long long total = o_off[img + 1] - o0;
  double s = 0.0;
  long long c = 0;
  for (long long e = threadIdx.x; e < total; e += blockDim.x) {
    const double v = static_cast<double>(vals[o0 + e]);
    if (v == invalid) continue;
    s += v;
    ++c;
    if (per_class) {
      const long long lab = gt_lab[b0 + e % m];
      int lo = 0, hi = K;  // lower_bound: classes is the sorted unique set of all ground-truth labels
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (classes[mid] < lab) lo = mid + 1;
        else hi = mid;
      }
      atomicAdd(&lsum[lo], v);
      atomicAdd(&lcnt[lo], 1);
    }
  }
  __shared__ double rs[256 / kWave];
  __shared__ long long rc[256 / kWave];
  s = wave_sum(s);
  c = wave_sum_ll(c);
  if ((threadIdx.x & (kWave - 1)) == 0) {
    rs[threadIdx.x / kWave] = s;
    rc[threadIdx.x / kWave] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0;
    long long tc = 0;
    for (int w = 0; w < static_cast<int>(blockDim.x / kWave); ++w) {
      ts += rs[w];
      tc += rc[w];
    }
    if (tc) {
      atomicAdd(&sums[K], ts);
      atomic_add_i64(counts + K, tc);
    }
  }
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    if (lcnt[k]) {
      atomicAdd(&sums[k], lsum[k]);
      atomic_add_i64(counts + k, lcnt[k]);
    }
  }
}

// COCO bbox IoU (maskApi bbIou): boxes xywh, crowd ground truth => intersection over detection area.
__device__ __forceinline__ double coco_iou(const double* d, const double* g, bool crowd) {
  const double w = min(d[0] + d[2], g[0] + g[2]) - max(d[0], g[0]);
  if (w <= 0) return 0.0;
  const double h = min(d[1] + d[3], g[1] + g[3]) - max(d[1], g[1]);
  if (h <= 0) return 0.0;
  const double inter = w * h;
  const double da = d[2] * d[3];
  const double u = crowd ? da : da + g[2] * g[3] - inter;
  return inter / u;
}

__global__ void __launch_bounds__(256) coco_match_kernel(
    const double* __restrict__ dbox, const double* __restrict__ darea, const double* __restrict__ gbox,
    const double* __restrict__ garea, const uint8_t* __restrict__ gcrowd, const int* __restrict__ det_start,
    const int* __restrict__ det_cnt, const int* __restrict__ gt_start, const int* __restrict__ gt_cnt, int groups,
    const double* __restrict__ area_rng, int num_area, const double* __restrict__ iou_thr, int num_thr, int num_det,
    int num_gt, const double* __restrict__ iou_pre, const int64_t* __restrict__ iou_off,
    uint8_t* __restrict__ gt_used, uint8_t* __restrict__ dt_match, uint8_t* __restrict__ dt_ig) {
  const long long idx = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (idx >= static_cast<long long>(groups) * num_area * num_thr) return;
  const int t = static_cast<int>(idx % num_thr);
  const int a = static_cast<int>((idx / num_thr) % num_area);
  const int grp = static_cast<int>(idx / (static_cast<long long>(num_thr) * num_area));
  const int dn = det_cnt[grp];
  if (dn == 0) return;
  const int d0 = det_start[grp], g0 = gt_start[grp], gn = gt_cnt[grp];
  const double lo = area_rng[2 * a], hi = area_rng[2 * a + 1];
  const double thr = min(iou_thr[t], 1.0 - 1e-10);
  const long long plane_d = static_cast<long long>(t * num_area + a) * num_det;
  uint8_t* used = gt_used + static_cast<long long>(t * num_area + a) * num_gt;
  // groups of <= 64 ground truths (the usual case) keep the "already matched" flags in a register bitmask: no global
  // store -> load round trip between consecutive detections of the greedy loop
  const bool small = gn <= 64;
  unsigned long long used_bits = 0ull;
  for (int k = 0; k < dn; ++k) {
    const int di = d0 + k;
    const double* db = dbox + 4LL * di;
    double best = thr;
    int m = -1;
    bool m_ig = false;
    // pass 1: ground truths inside the area range and not crowd (COCO sorts these first)
    for (int j = 0; j < gn; ++j) {
      const int gi = g0 + j;
      const bool crowd = gcrowd[gi] != 0;
      const bool ig = crowd || garea[gi] < lo || garea[gi] > hi;
      if (ig || (small ? ((used_bits >> j) & 1ull) != 0 : used[gi] != 0)) continue;
      const double v = iou_pre ? iou_pre[iou_off[grp] + static_cast<long long>(k) * gn + j]
                               : coco_iou(db, gbox + 4LL * gi, false);
      if (v < best) continue;
      best = v;
      m = gi;
    }
    if (m < 0) {  // pass 2: ignored ground truths (crowd ones may be matched repeatedly)
      for (int j = 0; j < gn; ++j) {
        const int gi = g0 + j;
        const bool crowd = gcrowd[gi] != 0;
        const bool ig = crowd || garea[gi] < lo || garea[gi] > hi;
        const bool u = small ? ((used_bits >> j) & 1ull) != 0 : used[gi] != 0;
        if (!ig || (u && !crowd)) continue;
        const double v = iou_pre ? iou_pre[iou_off[grp] + static_cast<long long>(k) * gn + j]
                                 : coco_iou(db, gbox + 4LL * gi, crowd);
        if (v < best) continue;
        best = v;
        m = gi;
        m_ig = true;
      }
    }
    if (m >= 0) {
      if (small) used_bits |= 1ull << (m - g0);
      else used[m] = 1;
      dt_match[plane_d + di] = 1;
      dt_ig[plane_d + di] = m_ig ? 1 : 0;
    } else {
      dt_match[plane_d + di] = 0;
      dt_ig[plane_d + di] = (darea[di] < lo || darea[di] > hi) ? 1 : 0;
    }
  }
}

}  // namespace

// a [N, 4], b [M, 4] xyxy (same float dtype); op 0 iou, 1 giou, 2 diou, 3 ciou; aligned -> [N] (N == M) else [N, M]
at::Tensor box_pairwise(const at::Tensor& a, const at::Tensor& b, int64_t op, bool aligned) {
  TM_CHECK_CUDA(a);
  TM_CHECK_CONTIG(a);
  TM_CHECK_CONTIG(b);
  TORCH_CHECK(a.dim() == 2 && a.size(1) == 4 && b.dim() == 2 && b.size(1) == 4, "box_pairwise: boxes must be [*, 4]");
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "box_pairwise: dtype mismatch");
  TORCH_CHECK(op >= 0 && op <= 3, "box_pairwise: unknown op");
  const int n = static_cast<int>(a.size(0)), m = static_cast<int>(b.size(0));
  if (aligned) TORCH_CHECK(n == m, "box_pairwise: aligned mode needs N == M");
  at::Tensor out = aligned ? at::empty({n}, a.options()) : at::empty({n, m}, a.options());
  const long long total = aligned ? n : static_cast<long long>(n) * m;
  if (total == 0) return out;
  auto s = stream();
  TM_DISPATCH_FLOAT(a.scalar_type(), "box_pairwise", [&] {
    using acc_t = typename std::conditional<std::is_same<scalar_t, double>::value, double, float>::type;
    hipLaunchKernelGGL((box_pairwise_kernel<scalar_t, acc_t>), dim3(grid_cap((total + 255) / 256, 8192)), dim3(256),
                       0, s, reinterpret_cast<const scalar_t*>(a.data_ptr()),
                       reinterpret_cast<const scalar_t*>(b.data_ptr()), n, m, static_cast<int>(op), aligned,
                       reinterpret_cast<scalar_t*>(out.data_ptr()));
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// Ragged batch: a [sum n_i, 4], b [sum m_i, 4] xyxy; a_off / b_off / o_off int64 [I + 1] (o_off: prefix sums of
// n_i * m_i); labels int64 (empty tensors: respect_labels off).  Returns the flat [sum n_i m_i] values.
at::Tensor box_pairwise_ragged(const at::Tensor& a, const at::Tensor& b, const at::Tensor& a_off,
                               const at::Tensor& b_off, const at::Tensor& o_off, const at::Tensor& a_lab,
                               const at::Tensor& b_lab, int64_t op, double threshold, bool has_thr, double invalid,
                               int64_t total) {
  TM_CHECK_CUDA(a);
  for (const at::Tensor* t : {&b, &a_off, &b_off, &o_off, &a_lab, &b_lab}) TM_SAME_DEVICE(a, (*t));
  for (const at::Tensor* t : {&a, &b, &a_off, &b_off, &o_off, &a_lab, &b_lab})
    TORCH_CHECK(t->is_contiguous(), "box_pairwise_ragged: contiguous inputs expected");
  TORCH_CHECK(a.dim() == 2 && a.size(1) == 4 && b.dim() == 2 && b.size(1) == 4, "box_pairwise_ragged: [*, 4] boxes");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && (a.scalar_type() == at::kFloat || a.scalar_type() == at::kDouble),
              "box_pairwise_ragged: float32 / float64 boxes of one dtype");
  TORCH_CHECK(op >= 0 && op <= 3, "box_pairwise_ragged: unknown op");
  for (const at::Tensor* t : {&a_off, &b_off, &o_off})
    TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() == a_off.numel() && t->numel() >= 1,
                "box_pairwise_ragged: offsets int64 [I + 1]");
  const bool labels = a_lab.numel() > 0 || b_lab.numel() > 0;
  if (labels)
    TORCH_CHECK(a_lab.scalar_type() == at::kLong && b_lab.scalar_type() == at::kLong && a_lab.numel() == a.size(0) &&
                    b_lab.numel() == b.size(0),
                "box_pairwise_ragged: int64 labels, one per box");
  const long long I = a_off.numel() - 1;  // total = o_off[I], passed by the caller (no device read)
  at::Tensor out = at::empty({total}, a.options());
  if (total == 0 || I == 0) return out;
  TM_DISPATCH_FLOAT(a.scalar_type(), "box_pairwise_ragged", [&] {
    using acc_t = typename std::conditional<std::is_same<scalar_t, double>::value, double, float>::type;
    hipLaunchKernelGGL((box_pairwise_ragged_kernel<scalar_t, acc_t>), dim3(static_cast<unsigned>(I)), dim3(256), 0,
                       stream(), reinterpret_cast<const scalar_t*>(a.data_ptr()),
                       reinterpret_cast<const scalar_t*>(b.data_ptr()), a_off.data_ptr<int64_t>(),
                       b_off.data_ptr<int64_t>(), o_off.data_ptr<int64_t>(),
                       labels ? a_lab.data_ptr<int64_t>() : nullptr, labels ? b_lab.data_ptr<int64_t>() : nullptr,
                       static_cast<int>(op), has_thr, static_cast<acc_t>(threshold), static_cast<acc_t>(invalid),
                       reinterpret_cast<scalar_t*>(out.data_ptr()));
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// (sums f64 [K + 1], counts int64 [K + 1]) of the valid values, per class (k < K) and overall (K); see the kernel.
std::tuple<at::Tensor, at::Tensor> iou_class_reduce(const at::Tensor& vals, const at::Tensor& o_off,
                                                    const at::Tensor& b_off, const at::Tensor& gt_lab,
                                                    const at::Tensor& classes, double invalid) {
  TM_CHECK_CUDA(vals);
  for (const at::Tensor* t : {&o_off, &b_off, &gt_lab, &classes}) {
    TM_SAME_DEVICE(vals, (*t));
    TORCH_CHECK(t->scalar_type() == at::kLong && t->is_contiguous(), "iou_class_reduce: int64 contiguous tables");
  }
  TORCH_CHECK(vals.is_contiguous() && (vals.scalar_type() == at::kFloat || vals.scalar_type() == at::kDouble),
              "iou_class_reduce: float32 / float64 values");
  TORCH_CHECK(o_off.numel() == b_off.numel() && o_off.numel() >= 1, "iou_class_reduce: offsets [I + 1]");
  const long long I = o_off.numel() - 1;
  const int K = static_cast<int>(classes.numel());
  const size_t lds = static_cast<size_t>(K) * (sizeof(double) + sizeof(int));
  TORCH_CHECK(lds <= 60 * 1024, "iou_class_reduce: at most ~5000 classes");
  at::Tensor sums = at::zeros({K + 1}, vals.options().dtype(at::kDouble));
  at::Tensor counts = at::zeros({K + 1}, vals.options().dtype(at::kLong));
  if (I == 0) return {sums, counts};
  AT_DISPATCH_FLOATING_TYPES(vals.scalar_type(), "iou_class_reduce", [&] {
    hipLaunchKernelGGL(iou_class_reduce_kernel<scalar_t>, dim3(static_cast<unsigned>(I)), dim3(256), lds, stream(),
                       vals.data_ptr<scalar_t>(), o_off.data_ptr<int64_t>(), b_off.data_ptr<int64_t>(),
                       gt_lab.data_ptr<int64_t>(), classes.data_ptr<int64_t>(), K, invalid, sums.data_ptr<double>(),
                       counts.data_ptr<int64_t>());
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {sums, counts};
}

// Greedy COCO matching for all groups / area ranges / thresholds.  Returns (dt_match, dt_ig), each uint8 [T, A, D].
std::tuple<at::Tensor, at::Tensor> coco_match(const at::Tensor& dbox, const at::Tensor& darea, const at::Tensor& gbox,
                                              const at::Tensor& garea, const at::Tensor& gcrowd,
                                              const at::Tensor& det_start, const at::Tensor& det_cnt,
                                              const at::Tensor& gt_start, const at::Tensor& gt_cnt,
                                              const at::Tensor& area_rng, const at::Tensor& iou_thr,
                                              const c10::optional<at::Tensor>& iou_pre,
                                              const c10::optional<at::Tensor>& iou_off) {
  TM_CHECK_CUDA(dbox);
  for (const auto* t : {&dbox, &darea, &gbox, &garea, &area_rng, &iou_thr})
    TORCH_CHECK(t->scalar_type() == at::kDouble && t->is_contiguous(), "coco_match: f64 contiguous inputs expected");
  for (const auto* t : {&det_start, &det_cnt, &gt_start, &gt_cnt})
    TORCH_CHECK(t->scalar_type() == at::kInt && t->is_contiguous(), "coco_match: int32 group tables expected");
  TORCH_CHECK(gcrowd.scalar_type() == at::kByte && gcrowd.is_contiguous(), "coco_match: crowd must be uint8");
  const int num_det = static_cast<int>(dbox.size(0)), num_gt = static_cast<int>(gbox.size(0));
  const int groups = static_cast<int>(det_start.numel());
  const int num_area = static_cast<int>(area_rng.numel() / 2), num_thr = static_cast<int>(iou_thr.numel());
  auto opts = dbox.options().dtype(at::kByte);
  // the two flag arrays and the matcher's "ground truth used" scratch from ONE zero-filled allocation (one fill
  // launch instead of three: compute() is launch-bound)
  const long long tad = static_cast<long long>(num_thr) * num_area * num_det;
  at::Tensor zbuf = at::zeros({2 * tad + static_cast<long long>(num_thr) * num_area * std::max(num_gt, 1)}, opts);
  at::Tensor dt_match = zbuf.narrow(0, 0, tad).view({num_thr, num_area, num_det});
  at::Tensor dt_ig = zbuf.narrow(0, tad, tad).view({num_thr, num_area, num_det});
  at::Tensor used = zbuf.narrow(0, 2 * tad, zbuf.numel() - 2 * tad);
  const bool pre = iou_pre.has_value() && iou_pre->defined();
  if (pre) {
    TORCH_CHECK(iou_off.has_value() && iou_off->scalar_type() == at::kLong && iou_off->numel() == groups,
                "coco_match: iou_off must be int64 [groups]");
    TORCH_CHECK(iou_pre->scalar_type() == at::kDouble && iou_pre->is_contiguous(), "coco_match: iou_pre f64");
  }
  const long long total = static_cast<long long>(groups) * num_area * num_thr;
  if (total > 0 && num_det > 0) {
    hipLaunchKernelGGL(coco_match_kernel, dim3((total + 255) / 256), dim3(256), 0, stream(), dbox.data_ptr<double>(),
                       darea.data_ptr<double>(), gbox.data_ptr<double>(), garea.data_ptr<double>(),
                       gcrowd.data_ptr<uint8_t>(), det_start.data_ptr<int>(), det_cnt.data_ptr<int>(),
                       gt_start.data_ptr<int>(), gt_cnt.data_ptr<int>(), groups, area_rng.data_ptr<double>(), num_area,
                       iou_thr.data_ptr<double>(), num_thr, num_det, std::max(num_gt, 1),
                       pre ? iou_pre->data_ptr<double>() : nullptr, pre ? iou_off->data_ptr<int64_t>() : nullptr,
                       used.data_ptr<uint8_t>(),
                       dt_match.data_ptr<uint8_t>(), dt_ig.data_ptr<uint8_t>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
  return {dt_match, dt_ig};
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("box_pairwise(Tensor a, Tensor b, int op, bool aligned) -> Tensor");
  m.def(
      "box_pairwise_ragged(Tensor a, Tensor b, Tensor a_off, Tensor b_off, Tensor o_off, Tensor a_lab, Tensor b_lab, "
      "int op, float threshold, bool has_thr, float invalid, int total) -> Tensor");
  m.def(
      "iou_class_reduce(Tensor vals, Tensor o_off, Tensor b_off, Tensor gt_lab, Tensor classes, float invalid) -> "
      "(Tensor, Tensor)");
  m.def(
      "coco_match(Tensor dbox, Tensor darea, Tensor gbox, Tensor garea, Tensor gcrowd, Tensor det_start, "
      "Tensor det_cnt, Tensor gt_start, Tensor gt_cnt, Tensor area_rng, Tensor iou_thr, Tensor? iou_pre=None, "
      "Tensor? iou_off=None) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("box_pairwise", &tm_amd::box_pairwise);
  m.impl("box_pairwise_ragged", &tm_amd::box_pairwise_ragged);
  m.impl("iou_class_reduce", &tm_amd::iou_class_reduce);
  m.impl("coco_match", &tm_amd::coco_match);
}
