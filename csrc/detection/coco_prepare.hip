// COCO evaluation front end in ONE launch (torchmetrics_amd/detection/_coco_eval.py coco_evaluate, bbox path).
//
// Replaces ~120 small ATen launches of the grouping stage (image-index expansion, category lookup, keep masks,
// (group, -score) sort, group histograms / starts, ranks, the gathers of boxes / areas / crowds into matcher order,
// the non-ignored ground-truth histogram) -- compute() was host-bound on their launch cost (~1.8 ms for config #3's
// 512 images, ~1 ms of device work).  Behavioural reference: pycocotools COCOeval.evaluateImg's per (image, category)
// detection order (score descending, mergesort-stable) and ground-truth order, as driven by
// S/detection/mean_ap.py:513-588.
//
// Layout: one block per image for its detections (blocks [0, n_img)) and one per image for its ground truths
// (blocks [n_img, 2 n_img)).  The block stages the image's sort keys in LDS -- detections (category index, descending-
// score key), ground truths (category index) -- and every element ranks itself against them: its output slot is the
// image's first slot + the number of elements ordered before it (key, then index: a stable sort), so the arrays come
// out grouped by (image, category) in score order, each image in its own flat range, categories not on the K axis
// (index K) at the end of the image's range.  The element ranked first in its group writes the group's start and
// count (detections: at most max_dets[-1]).  Detections write box / area / score / within-group rank / category and
// the (category, score) key of the accumulation sort; ground truths write box / area / crowd and add their
// (area range, category) to the non-ignored histogram.  Image sizes are bounded by the LDS key buffer
// (kPrepMaxPerImage); the caller keeps the ATen path beyond it.
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kPrepThreads = 256;
constexpr int kPrepMaxPerImage = 2048;  // 16 KiB of LDS keys; the ranking loop is O(n^2) per image

enum FloatCode : int { kF32 = 0, kF64 = 1, kF16 = 2, kBF16 = 3 };
enum IntCode : int { kI64 = 0, kI32 = 1, kU8 = 2, kI16 = 3 };

__device__ __forceinline__ double ld_f(const void* p, int code, long long i) {
  switch (code) {
    case kF64: return static_cast<const double*>(p)[i];
    case kF16: return static_cast<double>(to_f32(static_cast<const c10::Half*>(p)[i]));
    case kBF16: return static_cast<double>(to_f32(static_cast<const c10::BFloat16*>(p)[i]));
    default: return static_cast<double>(static_cast<const float*>(p)[i]);
  }
}

__device__ __forceinline__ long long ld_i(const void* p, int code, long long i) {
  switch (code) {
    case kI32: return static_cast<const int32_t*>(p)[i];
    case kU8: return static_cast<const uint8_t*>(p)[i];
    case kI16: return static_cast<const int16_t*>(p)[i];
    default: return static_cast<const int64_t*>(p)[i];
  }
}

// _coco_eval._desc_key32: the score as f32 (-0 -> +0), its bits made order-preserving and reversed (larger score ->
// smaller key); NaN -> 0xffffffff (last)
__device__ __forceinline__ uint32_t desc_key(double s) {
  const float f = static_cast<float>(s) + 0.0f;
  if (f != f) return 0xffffffffu;
  const uint32_t b = __float_as_uint(f);
  const uint32_t ordered = b >= 0x80000000u ? 0xffffffffu - b : (b | 0x80000000u);
  return 0xffffffffu - ordered;
}

// index of `v` in the sorted category ids, or K when absent
__device__ __forceinline__ int class_index(const int64_t* __restrict__ classes, int K, long long v) {
  int lo = 0, hi = K;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (classes[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return (lo < K && classes[lo] == v) ? lo : K;
}

struct PrepArgs {
  const int64_t* classes;
  const int64_t* off;  // [2 * (n_img + 1)]: detection offsets, then ground-truth offsets
  const void* d_lab;
  const void* d_score;
  const void* d_box;
  const void* g_lab;
  const void* g_box;
  const void* g_crowd;
  const void* g_area;
  const double* areas;  // [A, 2]
  int lab_code, g_lab_code, score_code, dbox_code, gbox_code, crowd_code, garea_code;
  int n_img, K, A;
  long long max_det;
  // outputs
  int* det_start;
  int* det_cnt;
  int* gt_start;
  int* gt_cnt;
  int* npig;  // [A, K]
  double* o_dbox;
  double* o_darea;
  int64_t* o_rank;
  int64_t* o_cls;
  double* o_score;
  int64_t* o_key2;
  double* o_gbox;
  double* o_garea;
  uint8_t* o_gcrowd;
};

__global__ void __launch_bounds__(kPrepThreads) coco_prepare_kernel(PrepArgs a) {
  extern __shared__ unsigned long long keys[];
  const bool gt = static_cast<int>(blockIdx.x) >= a.n_img;
  const int img = gt ? blockIdx.x - a.n_img : blockIdx.x;
  const int64_t* off = a.off + (gt ? a.n_img + 1 : 0);
  const long long b = off[img];
  const int n = static_cast<int>(off[img + 1] - b);
  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += kPrepThreads) {
    if (gt) {
      keys[i] = static_cast<unsigned long long>(class_index(a.classes, a.K, ld_i(a.g_lab, a.g_lab_code, b + i)));
    } else {
      const unsigned long long c = class_index(a.classes, a.K, ld_i(a.d_lab, a.lab_code, b + i));
      keys[i] = (c << 32) | desc_key(ld_f(a.d_score, a.score_code, b + i));
    }
  }
  __syncthreads();
  for (int i = tid; i < n; i += kPrepThreads) {
    const unsigned long long key = keys[i];
    const unsigned long long grp = gt ? key : key >> 32;
    int before = 0, lower_grp = 0, same = 0;
    for (int k = 0; k < n; ++k) {  // (every lane reads the same LDS word: a broadcast)
      const unsigned long long kk = keys[k];
      const unsigned long long kg = gt ? kk : kk >> 32;
      before += (kk < key) || (kk == key && k < i);
      lower_grp += kg < grp;
      same += kg == grp;
    }
    const long long pos = b + before;
    const int cls = static_cast<int>(grp);
    const bool valid = cls < a.K;
    const int rank = before - lower_grp;  // within (image, category)
    const long long g = static_cast<long long>(img) * a.K + cls;
    if (gt) {
      const double x = ld_f(a.g_box, a.gbox_code, 4 * (b + i)), y = ld_f(a.g_box, a.gbox_code, 4 * (b + i) + 1);
      const double w = ld_f(a.g_box, a.gbox_code, 4 * (b + i) + 2), h = ld_f(a.g_box, a.gbox_code, 4 * (b + i) + 3);
      const double ain = ld_f(a.g_area, a.garea_code, b + i);
      const double area = ain > 0.0 ? ain : w * h;
      const long long cr = ld_i(a.g_crowd, a.crowd_code, b + i);
      const uint8_t crowd = cr <= 0 ? 0 : 1;
      a.o_gbox[4 * pos] = x;
      a.o_gbox[4 * pos + 1] = y;
      a.o_gbox[4 * pos + 2] = w;
      a.o_gbox[4 * pos + 3] = h;
      a.o_garea[pos] = area;
      a.o_gcrowd[pos] = crowd;
      if (valid) {
        if (rank == 0) {
          a.gt_start[g] = static_cast<int>(pos);
          a.gt_cnt[g] = same;
        }
        if (!crowd)
          for (int r = 0; r < a.A; ++r)
            if (!(area < a.areas[2 * r]) && !(area > a.areas[2 * r + 1])) atomicAdd(a.npig + r * a.K + cls, 1);
      }
    } else {
      const long long src = 4 * (b + i);
      const double w = ld_f(a.d_box, a.dbox_code, src + 2), h = ld_f(a.d_box, a.dbox_code, src + 3);
      a.o_dbox[4 * pos] = ld_f(a.d_box, a.dbox_code, src);
      a.o_dbox[4 * pos + 1] = ld_f(a.d_box, a.dbox_code, src + 1);
      a.o_dbox[4 * pos + 2] = w;
      a.o_dbox[4 * pos + 3] = h;
      a.o_darea[pos] = w * h;
      a.o_score[pos] = ld_f(a.d_score, a.score_code, b + i);
      a.o_rank[pos] = valid ? rank : (0x7fffffffffffffffLL / 2);
      a.o_cls[pos] = cls;
      a.o_key2[pos] = static_cast<int64_t>((static_cast<unsigned long long>(cls) << 32) | (key & 0xffffffffull));
      if (valid && rank == 0) {
        a.det_start[g] = static_cast<int>(pos);
        a.det_cnt[g] = static_cast<int>(same < a.max_det ? same : a.max_det);
      }
    }
  }
}

// Sorted distinct values of two integer label arrays in [0, kUniqRange), in ONE single-block launch (the K axis of
// every COCO evaluation: torch.unique was a radix sort + merges + a partition, ~15 launches): an LDS bitmap of the
// range, then a block scan of the words' popcounts writes the values in order.  out int64 [1 + kUniqMax]: out[0] =
// the count, or -1 when a value is outside the range, -2 when more than kUniqMax values are distinct (the caller
// falls back to torch.unique).
constexpr int kUniqRange = 1 << 16;
constexpr int kUniqMax = 4096;
constexpr int kUniqThreads = 1024;

__global__ void __launch_bounds__(kUniqThreads) small_unique_kernel(const void* __restrict__ a, int acode,
                                                                    long long na, const void* __restrict__ b,
                                                                    int bcode, long long nb,
                                                                    int64_t* __restrict__ out) {
  constexpr int kWords = kUniqRange / 32;
  constexpr int kPer = kWords / kUniqThreads;  // bitmap words per thread in the compaction
  __shared__ uint32_t bits[kWords];
  __shared__ int scan[kUniqThreads];
  __shared__ int bad;
  const int tid = threadIdx.x;
  for (int w = tid; w < kWords; w += kUniqThreads) bits[w] = 0u;
  if (tid == 0) bad = 0;
  __syncthreads();
  for (long long i = tid; i < na + nb; i += kUniqThreads) {
    const long long v = i < na ? ld_i(a, acode, i) : ld_i(b, bcode, i - na);
    if (v < 0 || v >= kUniqRange) bad = 1;
    else atomicOr(&bits[v >> 5], 1u << (v & 31));
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) out[0] = -1;
    return;
  }
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) cnt += __popc(bits[tid * kPer + k]);
  scan[tid] = cnt;
  __syncthreads();
  for (int off = 1; off < kUniqThreads; off <<= 1) {  // inclusive Hillis-Steele scan of the popcounts
    const int v = tid >= off ? scan[tid - off] : 0;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  const int total = scan[kUniqThreads - 1];
  if (tid == 0) out[0] = total > kUniqMax ? -2 : total;
  if (total > kUniqMax) return;
  int pos = scan[tid] - cnt;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    uint32_t w = bits[tid * kPer + k];
    while (w) {
      const int bit = __ffs(w) - 1;
      w &= w - 1;
      out[1 + pos++] = static_cast<long long>(tid * kPer + k) * 32 + bit;
    }
  }
}

int float_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return kF32;
    case at::kDouble: return kF64;
    case at::kHalf: return kF16;
    case at::kBFloat16: return kBF16;
    default: TORCH_CHECK(false, "coco_prepare: unsupported floating dtype ", t.scalar_type());
  }
  return kF32;
}

int int_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kLong: return kI64;
    case at::kInt: return kI32;
    case at::kByte:
    case at::kBool: return kU8;
    case at::kShort: return kI16;
    default: TORCH_CHECK(false, "coco_prepare: unsupported integer dtype ", t.scalar_type());
  }
  return kI64;
}

}  // namespace

// classes int64 [K] sorted; off int64 [2 (n_img + 1)] (detection then ground-truth exclusive offsets, each ending in
// its total); max_per_image: the largest image size (host-known; <= kPrepMaxPerImage).  Returns [tables int32
// [4 G + A K] (det_start | det_cnt | gt_start | gt_cnt | npig), d_box f64 [D, 4], d_area, rank int64, cls int64,
// score f64, key2 int64, g_box f64 [N, 4], g_area, g_crowd uint8].
std::vector<at::Tensor> coco_prepare(const at::Tensor& classes, const at::Tensor& off, const at::Tensor& d_lab,
                                     const at::Tensor& d_score, const at::Tensor& d_box, const at::Tensor& g_lab,
                                     const at::Tensor& g_box, const at::Tensor& g_crowd, const at::Tensor& g_area,
                                     const at::Tensor& areas, int64_t n_img, int64_t max_det, int64_t max_per_image) {
  TM_CHECK_CUDA(classes);
  for (const at::Tensor* t : {&off, &d_lab, &d_score, &d_box, &g_lab, &g_box, &g_crowd, &g_area, &areas}) {
    TM_SAME_DEVICE(classes, (*t));
    TORCH_CHECK(t->is_contiguous(), "coco_prepare: contiguous inputs expected");
  }
  TORCH_CHECK(classes.scalar_type() == at::kLong && off.scalar_type() == at::kLong, "coco_prepare: int64 tables");
  TORCH_CHECK(areas.scalar_type() == at::kDouble && areas.numel() % 2 == 0, "coco_prepare: areas f64 [A, 2]");
  TORCH_CHECK(off.numel() == 2 * (n_img + 1), "coco_prepare: offsets [2 (n_img + 1)]");
  TORCH_CHECK(max_per_image >= 0 && max_per_image <= kPrepMaxPerImage, "coco_prepare: image too large");
  const long long D = d_lab.numel(), N = g_lab.numel();
  TORCH_CHECK(d_score.numel() == D && d_box.numel() == 4 * D, "coco_prepare: detection shapes");
  TORCH_CHECK(g_box.numel() == 4 * N && g_crowd.numel() == N && g_area.numel() == N, "coco_prepare: gt shapes");
  const int K = static_cast<int>(classes.numel()), A = static_cast<int>(areas.numel() / 2);
  const long long G = n_img * K;
  TORCH_CHECK(G < (1LL << 31) && D < (1LL << 31) && N < (1LL << 31), "coco_prepare: sizes");
  auto f64 = classes.options().dtype(at::kDouble);
  auto i64 = classes.options();
  at::Tensor tables = at::zeros({4 * G + static_cast<long long>(A) * K}, classes.options().dtype(at::kInt));
  at::Tensor o_dbox = at::empty({D, 4}, f64), o_darea = at::empty({D}, f64), o_rank = at::empty({D}, i64);
  at::Tensor o_cls = at::empty({D}, i64), o_score = at::empty({D}, f64), o_key2 = at::empty({D}, i64);
  at::Tensor o_gbox = at::empty({N, 4}, f64), o_garea = at::empty({N}, f64);
  at::Tensor o_gcrowd = at::empty({N}, classes.options().dtype(at::kByte));
  if (n_img > 0 && K > 0 && (D > 0 || N > 0)) {
    PrepArgs a;
    a.classes = classes.data_ptr<int64_t>();
    a.off = off.data_ptr<int64_t>();
    a.d_lab = d_lab.data_ptr();
    a.d_score = d_score.data_ptr();
    a.d_box = d_box.data_ptr();
    a.g_lab = g_lab.data_ptr();
    a.g_box = g_box.data_ptr();
    a.g_crowd = g_crowd.data_ptr();
    a.g_area = g_area.data_ptr();
    a.areas = areas.data_ptr<double>();
    a.lab_code = int_code(d_lab);
    a.g_lab_code = int_code(g_lab);
    a.score_code = float_code(d_score);
    a.dbox_code = float_code(d_box);
    a.gbox_code = float_code(g_box);
    a.crowd_code = int_code(g_crowd);
    a.garea_code = float_code(g_area);
    a.n_img = static_cast<int>(n_img);
    a.K = K;
    a.A = A;
    a.max_det = max_det;
    int* tp = tables.data_ptr<int>();
    a.det_start = tp;
    a.det_cnt = tp + G;
    a.gt_start = tp + 2 * G;
    a.gt_cnt = tp + 3 * G;
    a.npig = tp + 4 * G;
    a.o_dbox = o_dbox.data_ptr<double>();
    a.o_darea = o_darea.data_ptr<double>();
    a.o_rank = o_rank.data_ptr<int64_t>();
    a.o_cls = o_cls.data_ptr<int64_t>();
    a.o_score = o_score.data_ptr<double>();
    a.o_key2 = o_key2.data_ptr<int64_t>();
    a.o_gbox = o_gbox.data_ptr<double>();
    a.o_garea = o_garea.data_ptr<double>();
    a.o_gcrowd = o_gcrowd.data_ptr<uint8_t>();
    const size_t smem = static_cast<size_t>(std::max<int64_t>(max_per_image, 1)) * sizeof(unsigned long long);
    hipLaunchKernelGGL(coco_prepare_kernel, dim3(static_cast<unsigned>(2 * n_img)), dim3(kPrepThreads), smem, stream(),
                       a);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
  return {tables, o_dbox, o_darea, o_rank, o_cls, o_score, o_key2, o_gbox, o_garea, o_gcrowd};
}

// a, b: integer label arrays on one device -> int64 [1 + kUniqMax] (see small_unique_kernel)
at::Tensor small_unique(const at::Tensor& a, const at::Tensor& b) {
  TM_CHECK_CUDA(a);
  TM_SAME_DEVICE(a, b);
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous(), "small_unique: contiguous inputs expected");
  at::Tensor out = at::empty({1 + kUniqMax}, a.options().dtype(at::kLong));
  hipLaunchKernelGGL(small_unique_kernel, dim3(1), dim3(kUniqThreads), 0, stream(), a.data_ptr(), int_code(a),
                     static_cast<long long>(a.numel()), b.data_ptr(), int_code(b), static_cast<long long>(b.numel()),
                     out.data_ptr<int64_t>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("small_unique(Tensor a, Tensor b) -> Tensor");
  m.def(
      "coco_prepare(Tensor classes, Tensor off, Tensor d_lab, Tensor d_score, Tensor d_box, Tensor g_lab, "
      "Tensor g_box, Tensor g_crowd, Tensor g_area, Tensor areas, int n_img, int max_det, int max_per_image) "
      "-> Tensor[]");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("coco_prepare", &coco_prepare);
  m.impl("small_unique", &small_unique);
}

}  // namespace tm_amd
