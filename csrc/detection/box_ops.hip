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
      if (ig || used[gi]) continue;
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
        if (!ig || (used[gi] && !crowd)) continue;
        const double v = iou_pre ? iou_pre[iou_off[grp] + static_cast<long long>(k) * gn + j]
                                 : coco_iou(db, gbox + 4LL * gi, crowd);
        if (v < best) continue;
        best = v;
        m = gi;
        m_ig = true;
      }
    }
    if (m >= 0) {
      used[m] = 1;
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
  at::Tensor dt_match = at::zeros({num_thr, num_area, num_det}, opts);
  at::Tensor dt_ig = at::zeros({num_thr, num_area, num_det}, opts);
  at::Tensor used = at::zeros({static_cast<long long>(num_thr) * num_area * std::max(num_gt, 1)}, opts);
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
      "coco_match(Tensor dbox, Tensor darea, Tensor gbox, Tensor garea, Tensor gcrowd, Tensor det_start, "
      "Tensor det_cnt, Tensor gt_start, Tensor gt_cnt, Tensor area_rng, Tensor iou_thr, Tensor? iou_pre=None, "
      "Tensor? iou_off=None) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("box_pairwise", &tm_amd::box_pairwise);
  m.impl("coco_match", &tm_amd::coco_match);
}
