// Greedy COCO matching on the host (CPU dispatch key of `tm_amd::coco_match`; the ROCm key is the kernel in
// box_ops.hip).  Same semantics as pycocotools COCOeval.evaluateImg (reference S/detection/mean_ap.py:513-588 hands
// every image x class to it): per (image x class group, area range, IoU threshold), detections in score order take the
// best still-free ground truth with IoU >= threshold, non-ignored ground truths first, crowd ground truths
// reusable and matched with IoU over the detection area.
//
// Host layout: the IoU block of a group (det_cnt x gt_cnt) is computed once and reused by all A x T matchings (the
// GPU kernel recomputes it per thread instead -- there arithmetic is free and memory is not); groups are spread over
// threads with at::parallel_for.  Outputs are bitwise identical to the kernel's (same fp64 IoU formula, same order).
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdint>
#include <tuple>
#include <vector>

namespace tm_amd {
namespace {

inline double coco_iou_host(const double* d, const double* g, bool crowd) {
  const double w = std::min(d[0] + d[2], g[0] + g[2]) - std::max(d[0], g[0]);
  if (w <= 0) return 0.0;
  const double h = std::min(d[1] + d[3], g[1] + g[3]) - std::max(d[1], g[1]);
  if (h <= 0) return 0.0;
  const double inter = w * h;
  const double da = d[2] * d[3];
  const double u = crowd ? da : da + g[2] * g[3] - inter;
  return inter / u;
}

}  // namespace

std::tuple<at::Tensor, at::Tensor> coco_match_cpu(const at::Tensor& dbox_, const at::Tensor& darea_,
                                                  const at::Tensor& gbox_, const at::Tensor& garea_,
                                                  const at::Tensor& gcrowd_, const at::Tensor& det_start_,
                                                  const at::Tensor& det_cnt_, const at::Tensor& gt_start_,
                                                  const at::Tensor& gt_cnt_, const at::Tensor& area_rng_,
                                                  const at::Tensor& iou_thr_, const c10::optional<at::Tensor>& iou_pre,
                                                  const c10::optional<at::Tensor>& iou_off) {
  const at::Tensor dbox = dbox_.to(at::kDouble).contiguous(), darea = darea_.to(at::kDouble).contiguous();
  const at::Tensor gbox = gbox_.to(at::kDouble).contiguous(), garea = garea_.to(at::kDouble).contiguous();
  const at::Tensor gcrowd = gcrowd_.to(at::kByte).contiguous();
  const at::Tensor det_start = det_start_.to(at::kLong).contiguous(), det_cnt = det_cnt_.to(at::kLong).contiguous();
  const at::Tensor gt_start = gt_start_.to(at::kLong).contiguous(), gt_cnt = gt_cnt_.to(at::kLong).contiguous();
  const at::Tensor area_rng = area_rng_.to(at::kDouble).contiguous(), iou_thr = iou_thr_.to(at::kDouble).contiguous();
  const int64_t num_det = dbox.size(0), num_gt = gbox.size(0), groups = det_start.numel();
  const int64_t num_area = area_rng.numel() / 2, num_thr = iou_thr.numel();
  TORCH_CHECK(dbox.dim() == 2 && dbox.size(1) == 4 && gbox.dim() == 2 && gbox.size(1) == 4,
              "coco_match: boxes must be [*, 4] (xywh)");
  TORCH_CHECK(darea.numel() == num_det && garea.numel() == num_gt && gcrowd.numel() == num_gt,
              "coco_match: per-box tables must match the box counts");
  TORCH_CHECK(det_cnt.numel() == groups && gt_start.numel() == groups && gt_cnt.numel() == groups,
              "coco_match: group tables must have one entry per group");
  const bool pre = iou_pre.has_value() && iou_pre->defined();
  at::Tensor pre_t, off_t;
  if (pre) {
    TORCH_CHECK(iou_off.has_value() && iou_off->defined() && iou_off->numel() == groups,
                "coco_match: iou_off must be int64 [groups]");
    pre_t = iou_pre->to(at::kDouble).contiguous();
    off_t = iou_off->to(at::kLong).contiguous();
  }
  auto opts = at::TensorOptions().dtype(at::kByte);
  at::Tensor dt_match = at::zeros({num_thr, num_area, num_det}, opts);
  at::Tensor dt_ig = at::zeros({num_thr, num_area, num_det}, opts);
  if (groups == 0 || num_det == 0) return {dt_match, dt_ig};

  const double* db = dbox.data_ptr<double>();
  const double* da = darea.data_ptr<double>();
  const double* gb = gbox.data_ptr<double>();
  const double* ga = garea.data_ptr<double>();
  const uint8_t* gc = gcrowd.data_ptr<uint8_t>();
  const int64_t* ds = det_start.data_ptr<int64_t>();
  const int64_t* dc = det_cnt.data_ptr<int64_t>();
  const int64_t* gs = gt_start.data_ptr<int64_t>();
  const int64_t* gcnt = gt_cnt.data_ptr<int64_t>();
  const double* rng = area_rng.data_ptr<double>();
  const double* thr = iou_thr.data_ptr<double>();
  const double* pre_p = pre ? pre_t.data_ptr<double>() : nullptr;
  const int64_t* off_p = pre ? off_t.data_ptr<int64_t>() : nullptr;
  const int64_t pre_n = pre ? pre_t.numel() : 0;
  uint8_t* match = dt_match.data_ptr<uint8_t>();
  uint8_t* ign = dt_ig.data_ptr<uint8_t>();
  for (int64_t grp = 0; grp < groups; ++grp) {
    TORCH_CHECK(ds[grp] >= 0 && dc[grp] >= 0 && ds[grp] + dc[grp] <= num_det && gs[grp] >= 0 && gcnt[grp] >= 0 &&
                    gs[grp] + gcnt[grp] <= num_gt,
                "coco_match: group ", grp, " is out of range");
    if (pre && dc[grp] > 0 && gcnt[grp] > 0)
      TORCH_CHECK(off_p[grp] >= 0 && off_p[grp] + dc[grp] * gcnt[grp] <= pre_n, "coco_match: iou_pre block ", grp,
                  " out of range");
  }

  at::parallel_for(0, groups, 1, [&](int64_t lo_g, int64_t hi_g) {
    std::vector<double> iou;
    std::vector<uint8_t> used, ig_gt;
    for (int64_t grp = lo_g; grp < hi_g; ++grp) {
      const int64_t dn = dc[grp], gn = gcnt[grp], d0 = ds[grp], g0 = gs[grp];
      if (dn == 0) continue;
      iou.resize(static_cast<size_t>(dn * gn));
      for (int64_t k = 0; k < dn; ++k)
        for (int64_t j = 0; j < gn; ++j)
          iou[k * gn + j] = pre ? pre_p[off_p[grp] + k * gn + j]
                                : coco_iou_host(db + 4 * (d0 + k), gb + 4 * (g0 + j), gc[g0 + j] != 0);
      used.resize(static_cast<size_t>(gn));
      ig_gt.resize(static_cast<size_t>(gn));
      for (int64_t a = 0; a < num_area; ++a) {
        const double lo = rng[2 * a], hi = rng[2 * a + 1];
        for (int64_t j = 0; j < gn; ++j) ig_gt[j] = (gc[g0 + j] != 0 || ga[g0 + j] < lo || ga[g0 + j] > hi) ? 1 : 0;
        for (int64_t t = 0; t < num_thr; ++t) {
          const double th = std::min(thr[t], 1.0 - 1e-10);
          const int64_t plane = (t * num_area + a) * num_det;
          std::fill(used.begin(), used.end(), 0);
          for (int64_t k = 0; k < dn; ++k) {
            const double* row = iou.data() + k * gn;
            double best = th;
            int64_t m = -1;
            bool m_ig = false;
            for (int64_t j = 0; j < gn; ++j) {  // pass 1: regular ground truths
              if (ig_gt[j] || used[j] || row[j] < best) continue;
              best = row[j];
              m = j;
            }
            if (m < 0) {
              for (int64_t j = 0; j < gn; ++j) {  // pass 2: ignored ones (crowd: reusable)
                if (!ig_gt[j] || (used[j] && gc[g0 + j] == 0) || row[j] < best) continue;
                best = row[j];
                m = j;
                m_ig = true;
              }
            }
            const int64_t di = d0 + k;
            if (m >= 0) {
              used[m] = 1;
              match[plane + di] = 1;
              ign[plane + di] = m_ig ? 1 : 0;
            } else {
              ign[plane + di] = (da[di] < lo || da[di] > hi) ? 1 : 0;
            }
          }
        }
      }
    }
  });
  return {dt_match, dt_ig};
}

}  // namespace tm_amd

TORCH_LIBRARY_IMPL(tm_amd, CPU, m) { m.impl("coco_match", &tm_amd::coco_match_cpu); }
