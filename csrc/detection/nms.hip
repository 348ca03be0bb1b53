// Non-maximum suppression (greedy, score-ordered), optionally class-aware ("batched"): keep a box unless a
// higher-scored kept box of the same class overlaps it with IoU > threshold.
//
// Not a reference capability (the reference has no NMS); it is the detection post-processing step that
// usually precedes MeanAveragePrecision and is named by BASELINE config #3.  Layout for wave64:
//   * suppression mask: for boxes sorted by descending score, bit c of word mask[r][w] says "box r suppresses box
//     64w + c" (c > r, IoU > thr, same class).  A 64-thread workgroup owns a 64 x 64 tile (row block, column block
//     >= row block): the column block's boxes are staged in LDS, each lane evaluates its row against all 64 and
//     produces the whole 64-bit word with no atomics -- one wave per tile is exactly one word per lane.
//   * greedy scan: a single wave walks the rows in 64-row chunks.  The chunk's diagonal words are resolved
//     sequentially in registers (lane shuffles, no LDS traffic), then every kept row's mask words are OR-ed into the
//     removed bitset, lanes striding the words with 8 independent loads in flight.  Kept indices are written in
//     score order and their count to a device word.
// IoU in fp32 with the torchvision box convention (area = (x2 - x1) * (y2 - y1), inter / union).
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kTile = 64;
constexpr int kMaxWords = 4096;  // n <= 262144 boxes per call (removed bitset: 32 KiB of LDS)

__device__ __forceinline__ float box_iou(const float4 a, const float4 b) {
  const float area_a = (a.z - a.x) * (a.w - a.y);
  const float area_b = (b.z - b.x) * (b.w - b.y);
  const float iw = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x), 0.f);
  const float ih = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y), 0.f);
  const float inter = iw * ih;
  return inter / (area_a + area_b - inter);
}

// grid (col_blocks, row_blocks), block 64: boxes / classes already in score order
__global__ void __launch_bounds__(kTile) nms_mask_kernel(const float4* __restrict__ boxes,
                                                         const int64_t* __restrict__ cls, int n, float thr,
                                                         unsigned long long* __restrict__ mask, int words) {
  const int rb = blockIdx.y, cb = blockIdx.x;
  if (cb < rb) return;  // block-uniform: suppressions only go to later (lower-scored) boxes
  __shared__ float4 cbox[kTile];
  __shared__ int64_t ccls[kTile];
  const int lane = threadIdx.x;
  const int col0 = cb * kTile;
  if (col0 + lane < n) {
    cbox[lane] = boxes[col0 + lane];
    ccls[lane] = cls ? cls[col0 + lane] : 0;
  }
  __syncthreads();
  const int row = rb * kTile + lane;
  if (row >= n) return;
  const float4 rbox = boxes[row];
  const int64_t rcls = cls ? cls[row] : 0;
  const int ncol = min(kTile, n - col0);
  unsigned long long bits = 0ull;
  for (int c = (cb == rb ? lane + 1 : 0); c < ncol; ++c) {
    if (ccls[c] == rcls && box_iou(rbox, cbox[c]) > thr) bits |= 1ull << c;
  }
  mask[static_cast<long long>(row) * words + cb] = bits;
}

// one wave: greedy scan over the mask
__global__ void __launch_bounds__(kTile) nms_scan_kernel(const unsigned long long* __restrict__ mask, int n,
                                                         int words, const int64_t* __restrict__ order,
                                                         int64_t* __restrict__ keep, int* __restrict__ nkeep) {
  __shared__ unsigned long long removed[kMaxWords];
  const int lane = threadIdx.x;
  for (int w = lane; w < words; w += kTile) removed[w] = 0ull;
  __syncthreads();
  int count = 0;
  for (int cb = 0; cb < words; ++cb) {
    const int r0 = cb * kTile;
    const int nrow = min(kTile, n - r0);
    // lane l holds the diagonal word of row r0 + l
    const unsigned long long diag = lane < nrow ? mask[static_cast<long long>(r0 + lane) * words + cb] : 0ull;
    unsigned long long rem = removed[cb];  // the same value in every lane
    unsigned long long kept = 0ull;
    for (int l = 0; l < nrow; ++l) {  // sequential inside the chunk, in registers
      const unsigned long long dl = __shfl(diag, l, kTile);
      if (!((rem >> l) & 1ull)) {
        kept |= 1ull << l;
        rem |= dl;
      }
    }
    if ((kept >> lane) & 1ull) {
      const int rank = __popcll(kept & ((1ull << lane) - 1ull));
      keep[count + rank] = order[r0 + lane];
    }
    count += __popcll(kept);
    // fold the kept rows' suppressions into the later words, 8 independent row loads in flight per lane
    for (int w = cb + 1 + lane; w < words; w += kTile) {
      unsigned long long acc = removed[w];
      unsigned long long k = kept;
      while (k) {
        int rows[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          rows[u] = -1;
          if (k) {
            rows[u] = __ffsll(static_cast<long long>(k)) - 1;
            k &= k - 1ull;
          }
        }
        unsigned long long v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[u] = rows[u] >= 0 ? mask[static_cast<long long>(r0 + rows[u]) * words + w] : 0ull;
#pragma unroll
        for (int u = 0; u < 8; ++u) acc |= v[u];
      }
      removed[w] = acc;
    }
    __syncthreads();
  }
  if (lane == 0) *nkeep = count;
}

}  // namespace

// boxes: [N, 4] xyxy; scores: [N]; idxs: i64 [N] class ids or empty (class-agnostic).
// Returns i64 [K] indices of the kept boxes in descending score order (equal scores: lower index first).
at::Tensor nms(const at::Tensor& boxes, const at::Tensor& scores, const at::Tensor& idxs, double iou_threshold) {
  TM_CHECK_CUDA(boxes);
  TORCH_CHECK(boxes.dim() == 2 && boxes.size(1) == 4, "nms: boxes must be [N, 4]");
  TORCH_CHECK(scores.dim() == 1 && scores.size(0) == boxes.size(0), "nms: scores must be [N]");
  const long long n = boxes.size(0);
  auto lopt = boxes.options().dtype(at::kLong);
  if (n == 0) return at::empty({0}, lopt);
  const int words = static_cast<int>((n + kTile - 1) / kTile);
  TORCH_CHECK(words <= kMaxWords, "nms: at most ", kMaxWords * kTile, " boxes per call");
  const bool batched = idxs.numel() > 0;
  if (batched) TORCH_CHECK(idxs.numel() == n, "nms: idxs must be [N]");
  at::Tensor order = std::get<1>(scores.sort(/*stable=*/true, /*dim=*/0, /*descending=*/true));
  at::Tensor sboxes = boxes.index_select(0, order).to(at::kFloat).contiguous();
  at::Tensor scls = batched ? idxs.index_select(0, order).to(at::kLong).contiguous() : at::Tensor();
  at::Tensor mask = at::empty({n, words}, lopt);
  auto s = stream();
  hipLaunchKernelGGL(nms_mask_kernel, dim3(words, words), dim3(kTile), 0, s,
                     reinterpret_cast<const float4*>(sboxes.data_ptr<float>()),
                     batched ? scls.data_ptr<int64_t>() : nullptr, static_cast<int>(n),
                     static_cast<float>(iou_threshold),
                     reinterpret_cast<unsigned long long*>(mask.data_ptr<int64_t>()), words);
  at::Tensor keep = at::empty({n}, lopt);
  at::Tensor nkeep = at::zeros({1}, boxes.options().dtype(at::kInt));
  hipLaunchKernelGGL(nms_scan_kernel, dim3(1), dim3(kTile), 0, s,
                     reinterpret_cast<const unsigned long long*>(mask.data_ptr<int64_t>()), static_cast<int>(n),
                     words, order.data_ptr<int64_t>(), keep.data_ptr<int64_t>(), nkeep.data_ptr<int>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  const int k = nkeep.item<int>();  // the output size is data dependent: the op's one host read
  return keep.narrow(0, 0, k);
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("nms(Tensor boxes, Tensor scores, Tensor idxs, float iou_threshold) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("nms", &tm_amd::nms); }
