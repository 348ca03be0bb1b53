// Greedy NMS on the host (CPU dispatch key of `tm_amd::nms`; the ROCm key is the bitmask kernel in nms.hip).
// Same rule and arithmetic as the kernel: boxes in stable descending-score order, fp32 IoU, a box is dropped when a
// kept higher-scored box of the same class overlaps it with IoU > threshold.  Kept boxes are compared against the
// candidate (O(n * kept)) instead of materialising the n x n suppression matrix.
#include <ATen/ATen.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdint>
#include <vector>

namespace tm_amd {

at::Tensor nms_cpu(const at::Tensor& boxes, const at::Tensor& scores, const at::Tensor& idxs, double iou_threshold) {
  TORCH_CHECK(boxes.dim() == 2 && boxes.size(1) == 4, "nms: boxes must be [N, 4]");
  TORCH_CHECK(scores.dim() == 1 && scores.size(0) == boxes.size(0), "nms: scores must be [N]");
  const int64_t n = boxes.size(0);
  auto lopt = at::TensorOptions().dtype(at::kLong);
  if (n == 0) return at::empty({0}, lopt);
  const bool batched = idxs.numel() > 0;
  if (batched) TORCH_CHECK(idxs.numel() == n, "nms: idxs must be [N]");
  const at::Tensor order = std::get<1>(scores.sort(/*stable=*/true, /*dim=*/0, /*descending=*/true)).contiguous();
  const at::Tensor b = boxes.index_select(0, order).to(at::kFloat).contiguous();
  const at::Tensor c = batched ? idxs.index_select(0, order).to(at::kLong).contiguous() : at::Tensor();
  const float* bp = b.data_ptr<float>();
  const int64_t* cp = batched ? c.data_ptr<int64_t>() : nullptr;
  const int64_t* op = order.data_ptr<int64_t>();
  const float thr = static_cast<float>(iou_threshold);
  std::vector<float> area(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) area[i] = (bp[4 * i + 2] - bp[4 * i]) * (bp[4 * i + 3] - bp[4 * i + 1]);
  std::vector<int64_t> kept;
  for (int64_t i = 0; i < n; ++i) {
    const float* bi = bp + 4 * i;
    bool drop = false;
    for (int64_t k : kept) {
      if (cp && cp[k] != cp[i]) continue;
      const float* bk = bp + 4 * k;
      const float iw = std::max(std::min(bk[2], bi[2]) - std::max(bk[0], bi[0]), 0.f);
      const float ih = std::max(std::min(bk[3], bi[3]) - std::max(bk[1], bi[1]), 0.f);
      const float inter = iw * ih;
      if (inter / (area[k] + area[i] - inter) > thr) {
        drop = true;
        break;
      }
    }
    if (!drop) kept.push_back(i);
  }
  at::Tensor out = at::empty({static_cast<int64_t>(kept.size())}, lopt);
  int64_t* o = out.data_ptr<int64_t>();
  for (size_t j = 0; j < kept.size(); ++j) o[j] = op[kept[j]];
  return out;
}

}  // namespace tm_amd

TORCH_LIBRARY_IMPL(tm_amd, CPU, m) { m.impl("nms", &tm_amd::nms_cpu); }
