// Run-length encoded masks for `MeanAveragePrecision(iou_type="segm")` (K21 segm path).
//
// Reference: S/detection/mean_ap.py:825-829 encodes every mask on the host with pycocotools (`mask_utils.encode` of a
// Fortran-ordered numpy copy), keeps (size, counts-bytes) tuples in state, gathers them with all_gather_object
// (:1007-1038) and lets COCOeval compute mask IoUs with `rleIou` on the CPU.
//
// Here a mask is stored by its *change positions*: the column-major (COCO order, index x*H + y) pixel indices where
// the value flips, starting from background.  That is COCO's RLE in cumulative form (counts = successive differences),
// so areas, IoUs and the COCO counts string all follow from it, and it makes IoU a merge of two sorted interval lists.
// One image's masks live in a single int32 "pack" tensor (device-resident state, gathered by the sync engine like any
// list state):
//     [n, H, W, area_0 .. area_{n-1}, off_0 .. off_n, positions...]      off: start of mask l's positions
//
// rle_encode   two kernels over all masks of an update call (one block per mask): (1) per-column change counts and
//              the mask area; one D2H copy of the per-mask totals sizes the packs; (2) a block scan of the column
//              counts (tiles of 1024 columns with a carry) and an ordered write of the positions.  A thread owns 4
//              adjacent columns and walks them row by row with one 4-byte load per row, so a wave reads 256
//              contiguous bytes per row (byte loads when rows are not 4-byte aligned).
// rle_iou      one thread per (detection, ground truth) pair: two-pointer merge of the foreground intervals; crowd
//              ground truths divide by the detection area; size mismatch -> -1 (pycocotools rleIou semantics).
// The CPU dispatch key runs the same algorithms on host threads.
#include "common/tm_common.h"

#include <ATen/Parallel.h>

#include <vector>

namespace tm_amd {
namespace {

constexpr int kThreads = 256;
constexpr int kRows = 8;  // rows loaded per batch in the encode kernels

// foreground interval i of a mask with k change positions: [pos[2i], pos[2i+1]) (open end -> hw)
__host__ __device__ inline long long rle_intersection(const int* a, int ka, const int* b, int kb, long long hw) {
  const int na = (ka + 1) / 2, nb = (kb + 1) / 2;
  int i = 0, j = 0;
  long long inter = 0;
  while (i < na && j < nb) {
    const long long a0 = a[2 * i], a1 = (2 * i + 1 < ka) ? a[2 * i + 1] : hw;
    const long long b0 = b[2 * j], b1 = (2 * j + 1 < kb) ? b[2 * j + 1] : hw;
    const long long lo = a0 > b0 ? a0 : b0, hi = a1 < b1 ? a1 : b1;
    if (hi > lo) inter += hi - lo;
    if (a1 < b1) ++i;
    else ++j;
  }
  return inter;
}

__host__ __device__ inline double rle_iou_value(const int* dbuf, const int64_t* dd, const int* gbuf, const int64_t* gd,
                                                bool crowd) {
  // desc row: pos_start, k, area, H, W
  if (dd[3] != gd[3] || dd[4] != gd[4]) return -1.0;
  const long long inter = rle_intersection(dbuf + dd[0], static_cast<int>(dd[1]), gbuf + gd[0],
                                           static_cast<int>(gd[1]), dd[3] * dd[4]);
  if (inter == 0) return 0.0;
  const long long uni = crowd ? dd[2] : dd[2] + gd[2] - inter;
  return static_cast<double>(inter) / static_cast<double>(uni);
}

__device__ inline int block_exclusive_scan(int v, int* lds_wave) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  int inc = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int o = __shfl_up(inc, off, kWave);
    if (lane >= off) inc += o;
  }
  if (lane == kWave - 1) lds_wave[wid] = inc;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wid; ++w) base += lds_wave[w];
  return base + inc - v;
}

// Column strips: a thread owns VW consecutive columns of a tile of kThreads * VW columns and walks them row by row,
// one VW-byte load per row (VW = 4 when rows are 4-byte aligned: a wave reads 256 contiguous bytes per row; else 1).
// Column x's value sequence in COCO order is rows 0..H-1 of column x, preceded by pixel (x-1, H-1).
template <int VW>
struct Strip {
  static __device__ __forceinline__ uint32_t load(const uint8_t* p) {
    if constexpr (VW == 4) return *reinterpret_cast<const uint32_t*>(p);
    else return *p;
  }
  static __device__ __forceinline__ int bit(uint32_t word, int j) { return ((word >> (8 * j)) & 0xffu) != 0; }
};

// table row: ptr, H, W, colcnt offset.  colcnt [N, W]: changes per column; stats [N, 2]: total changes, area.
template <int VW>
__global__ void __launch_bounds__(kThreads) rle_count_kernel(const int64_t* __restrict__ table,
                                                              int* __restrict__ colcnt, int* __restrict__ stats) {
  const int mid = blockIdx.x, tid = threadIdx.x;
  const uint8_t* m = reinterpret_cast<const uint8_t*>(table[mid * 4]);
  const int H = static_cast<int>(table[mid * 4 + 1]), W = static_cast<int>(table[mid * 4 + 2]);
  int* cc = colcnt + static_cast<long long>(table[mid * 4 + 3]);
  int chg_all = 0, ones = 0;
  for (int x0 = tid * VW; x0 < W && H > 0; x0 += kThreads * VW) {
    int prev[VW], chg[VW];
    const uint32_t last = Strip<VW>::load(m + static_cast<long long>(H - 1) * W + x0);
    prev[0] = x0 == 0 ? 0 : (m[static_cast<long long>(H - 1) * W + x0 - 1] != 0);
#pragma unroll
    for (int j = 1; j < VW; ++j) prev[j] = Strip<VW>::bit(last, j - 1);
#pragma unroll
    for (int j = 0; j < VW; ++j) chg[j] = 0;
    for (int y0 = 0; y0 < H; y0 += kRows) {  // kRows independent loads in flight per lane
      uint32_t w[kRows];
#pragma unroll
      for (int r = 0; r < kRows; ++r)
        w[r] = y0 + r < H ? Strip<VW>::load(m + static_cast<long long>(y0 + r) * W + x0) : 0u;
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        if (y0 + r >= H) break;
#pragma unroll
        for (int j = 0; j < VW; ++j) {
          const int v = Strip<VW>::bit(w[r], j);
          chg[j] += v != prev[j];
          ones += v;
          prev[j] = v;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      cc[x0 + j] = chg[j];
      chg_all += chg[j];
    }
  }
  __shared__ int red[2][kThreads / kWave];
  const int wc = wave_sum(chg_all), wo = wave_sum(ones);
  if ((tid & (kWave - 1)) == 0) {
    red[0][tid / kWave] = wc;
    red[1][tid / kWave] = wo;
  }
  __syncthreads();
  if (tid < 2) {
    int s = 0;
    for (int w = 0; w < kThreads / kWave; ++w) s += red[tid][w];
    stats[mid * 2 + tid] = s;
  }
}

// table row: ptr, H, W, colcnt offset, pack_base, l, n, off_rel, nchg, area
template <int VW>
__global__ void __launch_bounds__(kThreads) rle_write_kernel(const int64_t* __restrict__ table,
                                                              const int* __restrict__ colcnt, int* __restrict__ out) {
  const int mid = blockIdx.x, tid = threadIdx.x;
  const int64_t* row = table + mid * 10;
  const uint8_t* m = reinterpret_cast<const uint8_t*>(row[0]);
  const int H = static_cast<int>(row[1]), W = static_cast<int>(row[2]);
  const int* cc = colcnt + row[3];
  const long long n = row[6], l = row[5], off_rel = row[7];
  int* pack = out + row[4];
  if (tid == 0) {
    if (l == 0) {
      pack[0] = static_cast<int>(n);
      pack[1] = H;
      pack[2] = W;
    }
    pack[3 + l] = static_cast<int>(row[9]);
    pack[3 + n + l] = static_cast<int>(off_rel);
    if (l == n - 1) pack[3 + 2 * n] = static_cast<int>(off_rel + row[8]);
  }
  int* pos = pack + 3 + 2 * n + 1 + off_rel;
  __shared__ int wsum[kThreads / kWave];
  __shared__ int carry_s;
  int carry = 0;
  for (int t0 = 0; t0 < W; t0 += kThreads * VW) {  // tiles of columns; uniform trip count across the block
    const int x0 = t0 + tid * VW;
    int cnt[VW];
    int mine = 0;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      cnt[j] = x0 + j < W ? cc[x0 + j] : 0;
      mine += cnt[j];
    }
    const int excl = block_exclusive_scan(mine, wsum);
    if (tid == kThreads - 1) carry_s = excl + mine;
    __syncthreads();
    const int tile_total = carry_s;
    if (x0 < W && H > 0) {
      int k[VW], prev[VW];
      int acc = carry + excl;
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        k[j] = acc;
        acc += cnt[j];
      }
      const uint32_t last = Strip<VW>::load(m + static_cast<long long>(H - 1) * W + x0);
      prev[0] = x0 == 0 ? 0 : (m[static_cast<long long>(H - 1) * W + x0 - 1] != 0);
#pragma unroll
      for (int j = 1; j < VW; ++j) prev[j] = Strip<VW>::bit(last, j - 1);
      for (int y0 = 0; y0 < H; y0 += kRows) {
        uint32_t w[kRows];
#pragma unroll
        for (int r = 0; r < kRows; ++r)
          w[r] = y0 + r < H ? Strip<VW>::load(m + static_cast<long long>(y0 + r) * W + x0) : 0u;
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
          if (y0 + r >= H) break;
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const int v = Strip<VW>::bit(w[r], j);
            if (v != prev[j]) pos[k[j]++] = (x0 + j) * H + y0 + r;
            prev[j] = v;
          }
        }
      }
    }
    carry += tile_total;
    __syncthreads();  // wsum / carry_s reuse by the next tile
  }
}

__global__ void rle_iou_kernel(const int* __restrict__ dbuf, const int64_t* __restrict__ ddesc,
                               const int* __restrict__ gbuf, const int64_t* __restrict__ gdesc,
                               const int64_t* __restrict__ pd, const int64_t* __restrict__ pg,
                               const uint8_t* __restrict__ gcrowd, long long P, double* __restrict__ out) {
  for (long long p = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; p < P;
       p += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int64_t d = pd[p], g = pg[p];
    out[p] = rle_iou_value(dbuf, ddesc + d * 5, gbuf, gdesc + g * 5, gcrowd[g] != 0);
  }
}

struct MaskRef {
  const uint8_t* ptr;
  int64_t h, w;
  int64_t image, local, n;
};

std::vector<MaskRef> mask_refs(at::TensorList masks, std::vector<at::Tensor>& keep) {
  std::vector<MaskRef> refs;
  for (size_t i = 0; i < masks.size(); ++i) {
    TORCH_CHECK(masks[i].dim() == 3, "rle_encode: masks must be [n, H, W]");
    at::Tensor m = masks[i];
    if (m.scalar_type() != at::kBool && m.scalar_type() != at::kByte) m = m.ne(0);
    m = m.contiguous();
    keep.push_back(m);
    const int64_t n = m.size(0), h = m.size(1), w = m.size(2);
    TORCH_CHECK(h * w < (1LL << 31), "rle_encode: H * W must be < 2^31");
    for (int64_t l = 0; l < n; ++l)
      refs.push_back({reinterpret_cast<const uint8_t*>(m.data_ptr()) + l * h * w, h, w, static_cast<int64_t>(i), l, n});
  }
  return refs;
}

// per-image pack sizes / bases from the per-mask change counts
int64_t pack_layout(at::TensorList masks, const std::vector<MaskRef>& refs, const int* nchg,
                    std::vector<int64_t>& base, std::vector<int64_t>& off_rel) {
  base.assign(masks.size(), 0);
  off_rel.assign(refs.size(), 0);
  std::vector<int64_t> tot(masks.size(), 0);
  for (size_t r = 0; r < refs.size(); ++r) {
    off_rel[r] = tot[refs[r].image];
    tot[refs[r].image] += nchg[r];
  }
  int64_t total = 0;
  for (size_t i = 0; i < masks.size(); ++i) {
    base[i] = total;
    total += 3 + 2 * masks[i].size(0) + 1 + tot[i];
  }
  TORCH_CHECK(total < (1LL << 31), "rle_encode: packed masks of one call exceed 2^31 words");
  return total;
}

std::vector<at::Tensor> split_packs(const at::Tensor& buf, at::TensorList masks, const std::vector<int64_t>& base) {
  std::vector<at::Tensor> out;
  for (size_t i = 0; i < masks.size(); ++i) {
    const int64_t end = i + 1 < masks.size() ? base[i + 1] : buf.numel();
    out.push_back(buf.narrow(0, base[i], end - base[i]));
  }
  return out;
}

}  // namespace

std::vector<at::Tensor> rle_encode_cuda(at::TensorList masks) {
  TORCH_CHECK(!masks.empty(), "rle_encode: empty list");
  TM_CHECK_CUDA(masks[0]);
  for (const auto& m : masks) TM_SAME_DEVICE(masks[0], m);
  std::vector<at::Tensor> keep;
  const std::vector<MaskRef> refs = mask_refs(masks, keep);
  const int64_t N = static_cast<int64_t>(refs.size());
  auto i64 = at::TensorOptions().dtype(at::kLong);
  auto dev_i32 = masks[0].options().dtype(at::kInt);
  std::vector<int64_t> base, off_rel;
  at::Tensor buf;
  if (N > 0) {
    TORCH_CHECK(N < (1LL << 31), "rle_encode: too many masks");
    // 4-byte column groups when every mask row is 4-byte aligned (W % 4 == 0 and 4-aligned mask starts)
    bool vec4 = true;
    std::vector<int64_t> col_off(N);
    int64_t cols = 0;
    for (int64_t r = 0; r < N; ++r) {
      vec4 = vec4 && refs[r].w % 4 == 0 && reinterpret_cast<uintptr_t>(refs[r].ptr) % 4 == 0;
      col_off[r] = cols;
      cols += refs[r].w + 4;  // + padding: a 4-wide group may straddle W only when W % 4 != 0 (byte path then)
    }
    at::Tensor t1 = at::empty({N, 4}, i64);
    int64_t* t1p = t1.data_ptr<int64_t>();
    for (int64_t r = 0; r < N; ++r) {
      t1p[r * 4] = reinterpret_cast<int64_t>(refs[r].ptr);
      t1p[r * 4 + 1] = refs[r].h;
      t1p[r * 4 + 2] = refs[r].w;
      t1p[r * 4 + 3] = col_off[r];
    }
    at::Tensor t1d = t1.to(masks[0].device());
    at::Tensor colcnt = at::empty({cols}, dev_i32);
    at::Tensor stats = at::empty({N, 2}, dev_i32);
    if (vec4)
      hipLaunchKernelGGL(rle_count_kernel<4>, dim3(static_cast<unsigned>(N)), dim3(kThreads), 0, stream(),
                         t1d.data_ptr<int64_t>(), colcnt.data_ptr<int>(), stats.data_ptr<int>());
    else
      hipLaunchKernelGGL(rle_count_kernel<1>, dim3(static_cast<unsigned>(N)), dim3(kThreads), 0, stream(),
                         t1d.data_ptr<int64_t>(), colcnt.data_ptr<int>(), stats.data_ptr<int>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
    at::Tensor st = stats.cpu();  // the one host sync of an update: sizes the packs
    const int* sp = st.data_ptr<int>();
    std::vector<int> nchg(N);
    for (int64_t r = 0; r < N; ++r) nchg[r] = sp[r * 2];
    const int64_t total = pack_layout(masks, refs, nchg.data(), base, off_rel);
    buf = at::empty({total}, dev_i32);
    at::Tensor t2 = at::empty({N, 10}, i64);
    int64_t* t2p = t2.data_ptr<int64_t>();
    for (int64_t r = 0; r < N; ++r) {
      const MaskRef& f = refs[r];
      const int64_t row[10] = {reinterpret_cast<int64_t>(f.ptr), f.h, f.w, col_off[r], base[f.image], f.local, f.n,
                               off_rel[r], nchg[r], sp[r * 2 + 1]};
      for (int c = 0; c < 10; ++c) t2p[r * 10 + c] = row[c];
    }
    at::Tensor t2d = t2.to(masks[0].device());
    if (vec4)
      hipLaunchKernelGGL(rle_write_kernel<4>, dim3(static_cast<unsigned>(N)), dim3(kThreads), 0, stream(),
                         t2d.data_ptr<int64_t>(), colcnt.data_ptr<int>(), buf.data_ptr<int>());
    else
      hipLaunchKernelGGL(rle_write_kernel<1>, dim3(static_cast<unsigned>(N)), dim3(kThreads), 0, stream(),
                         t2d.data_ptr<int64_t>(), colcnt.data_ptr<int>(), buf.data_ptr<int>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    pack_layout(masks, refs, nullptr, base, off_rel);
    buf = at::empty({static_cast<int64_t>(4 * masks.size())}, dev_i32);
  }
  // images without masks: [0, H, W, 0] headers written from the host (rare; one small copy each)
  for (size_t i = 0; i < masks.size(); ++i) {
    if (masks[i].size(0) != 0) continue;
    at::Tensor h = at::tensor({0, static_cast<int>(masks[i].size(1)), static_cast<int>(masks[i].size(2)), 0},
                              at::TensorOptions().dtype(at::kInt));
    buf.narrow(0, base[i], 4).copy_(h, /*non_blocking=*/false);
  }
  return split_packs(buf, masks, base);
}

std::vector<at::Tensor> rle_encode_cpu(at::TensorList masks) {
  TORCH_CHECK(!masks.empty(), "rle_encode: empty list");
  std::vector<at::Tensor> keep;
  const std::vector<MaskRef> refs = mask_refs(masks, keep);
  const int64_t N = static_cast<int64_t>(refs.size());
  std::vector<int> nchg(N), area(N);
  at::parallel_for(0, N, 1, [&](int64_t b, int64_t e) {
    for (int64_t r = b; r < e; ++r) {
      const MaskRef& f = refs[r];
      int prev = 0, c = 0, a = 0;
      for (int64_t x = 0; x < f.w; ++x)
        for (int64_t y = 0; y < f.h; ++y) {
          const int v = f.ptr[y * f.w + x] != 0;
          c += v != prev;
          a += v;
          prev = v;
        }
      nchg[r] = c;
      area[r] = a;
    }
  });
  std::vector<int64_t> base, off_rel;
  const int64_t total = pack_layout(masks, refs, nchg.data(), base, off_rel);
  at::Tensor buf = at::empty({total}, at::TensorOptions().dtype(at::kInt));
  int* out = buf.data_ptr<int>();
  for (size_t i = 0; i < masks.size(); ++i) {
    int* pack = out + base[i];
    const int64_t n = masks[i].size(0);
    pack[0] = static_cast<int>(n);
    pack[1] = static_cast<int>(masks[i].size(1));
    pack[2] = static_cast<int>(masks[i].size(2));
    pack[3 + 2 * n] = 0;
  }
  at::parallel_for(0, N, 1, [&](int64_t b, int64_t e) {
    for (int64_t r = b; r < e; ++r) {
      const MaskRef& f = refs[r];
      int* pack = out + base[f.image];
      pack[3 + f.local] = area[r];
      pack[3 + f.n + f.local] = static_cast<int>(off_rel[r]);
      if (f.local == f.n - 1) pack[3 + 2 * f.n] = static_cast<int>(off_rel[r] + nchg[r]);
      int* pos = pack + 3 + 2 * f.n + 1 + off_rel[r];
      int prev = 0, k = 0;
      for (int64_t x = 0; x < f.w; ++x)
        for (int64_t y = 0; y < f.h; ++y) {
          const int v = f.ptr[y * f.w + x] != 0;
          if (v != prev) pos[k++] = static_cast<int>(x * f.h + y);
          prev = v;
        }
    }
  });
  return split_packs(buf, masks, base);
}

static void check_iou_args(const at::Tensor& dbuf, const at::Tensor& ddesc, const at::Tensor& gbuf,
                           const at::Tensor& gdesc, const at::Tensor& pd, const at::Tensor& pg,
                           const at::Tensor& gcrowd) {
  TORCH_CHECK(dbuf.scalar_type() == at::kInt && gbuf.scalar_type() == at::kInt, "rle_iou: int32 buffers");
  TORCH_CHECK(ddesc.scalar_type() == at::kLong && gdesc.scalar_type() == at::kLong && ddesc.dim() == 2 &&
                  gdesc.dim() == 2 && ddesc.size(1) == 5 && gdesc.size(1) == 5,
              "rle_iou: descriptors must be int64 [N, 5]");
  TORCH_CHECK(pd.scalar_type() == at::kLong && pg.scalar_type() == at::kLong && pd.numel() == pg.numel(),
              "rle_iou: int64 pair indices of equal length");
  TORCH_CHECK(gcrowd.scalar_type() == at::kByte && gcrowd.numel() == gdesc.size(0), "rle_iou: uint8 crowd per gt");
  for (const at::Tensor* t : {&dbuf, &ddesc, &gbuf, &gdesc, &pd, &pg, &gcrowd}) TM_CHECK_CONTIG(*t);
}

// pair indices are trusted to be in range: the caller builds them from the descriptor row counts
at::Tensor rle_iou_cuda(const at::Tensor& dbuf, const at::Tensor& ddesc, const at::Tensor& gbuf,
                        const at::Tensor& gdesc, const at::Tensor& pd, const at::Tensor& pg,
                        const at::Tensor& gcrowd) {
  TM_CHECK_CUDA(pd);
  for (const at::Tensor* t : {&dbuf, &ddesc, &gbuf, &gdesc, &pg, &gcrowd}) TM_SAME_DEVICE(pd, *t);
  check_iou_args(dbuf, ddesc, gbuf, gdesc, pd, pg, gcrowd);
  const long long P = pd.numel();
  at::Tensor out = at::empty({P}, pd.options().dtype(at::kDouble));
  if (P == 0) return out;
  hipLaunchKernelGGL(rle_iou_kernel, dim3(grid_cap((P + 255) / 256, 256 * 64)), dim3(256), 0, stream(),
                     dbuf.data_ptr<int>(), ddesc.data_ptr<int64_t>(), gbuf.data_ptr<int>(), gdesc.data_ptr<int64_t>(),
                     pd.data_ptr<int64_t>(), pg.data_ptr<int64_t>(), gcrowd.data_ptr<uint8_t>(), P,
                     out.data_ptr<double>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

at::Tensor rle_iou_cpu(const at::Tensor& dbuf, const at::Tensor& ddesc, const at::Tensor& gbuf,
                       const at::Tensor& gdesc, const at::Tensor& pd, const at::Tensor& pg, const at::Tensor& gcrowd) {
  check_iou_args(dbuf, ddesc, gbuf, gdesc, pd, pg, gcrowd);
  const int64_t P = pd.numel();
  at::Tensor out = at::empty({P}, at::TensorOptions().dtype(at::kDouble));
  const int* db = dbuf.data_ptr<int>();
  const int* gb = gbuf.data_ptr<int>();
  const int64_t *dd = ddesc.data_ptr<int64_t>(), *gd = gdesc.data_ptr<int64_t>();
  const int64_t *pdp = pd.data_ptr<int64_t>(), *pgp = pg.data_ptr<int64_t>();
  const uint8_t* cr = gcrowd.data_ptr<uint8_t>();
  double* o = out.data_ptr<double>();
  const int64_t nd = ddesc.size(0), ng = gdesc.size(0);
  at::parallel_for(0, P, 256, [&](int64_t b, int64_t e) {
    for (int64_t p = b; p < e; ++p) {
      TORCH_CHECK(pdp[p] >= 0 && pdp[p] < nd && pgp[p] >= 0 && pgp[p] < ng, "rle_iou: pair index out of range");
      o[p] = rle_iou_value(db, dd + pdp[p] * 5, gb, gd + pgp[p] * 5, cr[pgp[p]] != 0);
    }
  });
  return out;
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("rle_encode(Tensor[] masks) -> Tensor[]");
  m.def("rle_iou(Tensor dbuf, Tensor ddesc, Tensor gbuf, Tensor gdesc, Tensor pd, Tensor pg, Tensor gcrowd) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("rle_encode", &rle_encode_cuda);
  m.impl("rle_iou", &rle_iou_cuda);
}
TORCH_LIBRARY_IMPL(tm_amd, CPU, m) {
  m.impl("rle_encode", &rle_encode_cpu);
  m.impl("rle_iou", &rle_iou_cpu);
}

}  // namespace tm_amd
