// Panoptic quality segment statistics (K22): per image, the pixel area of every predicted segment,
// every target segment and every (predicted, target) segment pair.
//
// Reference (F/detection/_panoptic_quality_common.py:50-62, 214-251): per sample `torch.unique(dim=0)` over the
// flattened color maps plus a Python dict walk over every intersecting pair.  The previous version here sorted all
// B*P pixel keys three times (`torch.unique` on packed keys).  Here one block owns one image: three open-addressing
// hash tables in LDS (pairs, predicted segments, target segments) count the pixels, with wave-level aggregation of
// equal keys first (neighbouring pixels mostly share a segment, so a wave usually issues 1-3 LDS atomics per table
// instead of 64 contended ones).  The tables are written out whole (empty slots keep the sentinel); an image with
// more distinct keys than a table holds raises its overflow flag and the caller takes the sort path for the batch.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 1024;
constexpr int kPairCap = 4096;  // distinct (pred, target) segment pairs per image
constexpr int kSegCap = 1024;   // distinct segments per image and side
constexpr unsigned kEmpty32 = 0xffffffffu;
constexpr unsigned long long kEmpty64 = ~0ull;

__device__ __forceinline__ unsigned hash32(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return static_cast<unsigned>(k);
}

// wave-aggregated insert-or-add of `add` for `key` into an LDS table (linear probing); false on overflow
template <typename K>
__device__ __forceinline__ bool wave_insert(K* keys, unsigned* counts, int cap, K key, bool active, K empty) {
  bool ok = true;
  unsigned long long todo = __ballot(active);
  while (todo) {
    const int leader = __ffsll(static_cast<long long>(todo)) - 1;
    const K lk = static_cast<K>(__shfl(static_cast<unsigned long long>(key), leader, kWave));
    const unsigned long long same = __ballot(active && key == lk) & todo;
    if ((threadIdx.x & (kWave - 1)) == leader) {
      unsigned h = hash32(static_cast<unsigned long long>(lk)) & (cap - 1);
      int probes = 0;
      while (true) {
        const K prev = atomicCAS(&keys[h], empty, lk);
        if (prev == empty || prev == lk) {
          atomicAdd(&counts[h], static_cast<unsigned>(__popcll(same)));
          break;
        }
        h = (h + 1) & (cap - 1);
        if (++probes >= cap) {
          ok = false;
          break;
        }
      }
    }
    todo &= ~same;
  }
  return ok;
}

__global__ void __launch_bounds__(kThreads) panoptic_tables_kernel(const int* __restrict__ pcode,
                                                                   const int* __restrict__ tcode, long long P,
                                                                   unsigned long long* __restrict__ out_pair_keys,
                                                                   unsigned* __restrict__ out_pair_cnt,
                                                                   unsigned* __restrict__ out_p_keys,
                                                                   unsigned* __restrict__ out_p_cnt,
                                                                   unsigned* __restrict__ out_t_keys,
                                                                   unsigned* __restrict__ out_t_cnt,
                                                                   int* __restrict__ overflow) {
  __shared__ unsigned long long pk[kPairCap];
  __shared__ unsigned pc[kPairCap];
  __shared__ unsigned sk[2][kSegCap];
  __shared__ unsigned sc[2][kSegCap];
  __shared__ int bad;
  const int tid = threadIdx.x;
  for (int i = tid; i < kPairCap; i += kThreads) {
    pk[i] = kEmpty64;
    pc[i] = 0;
  }
  for (int i = tid; i < kSegCap; i += kThreads) {
    sk[0][i] = sk[1][i] = kEmpty32;
    sc[0][i] = sc[1][i] = 0;
  }
  if (tid == 0) bad = 0;
  __syncthreads();
  const long long img = blockIdx.x;
  const int* pp = pcode + img * P;
  const int* tt = tcode + img * P;
  bool ok = true;
  // every lane of a wave runs the same trip count (ballots need the whole wave)
  for (long long base = 0; base < P; base += kThreads) {
    const long long e = base + tid;
    const bool active = e < P;
    const unsigned a = active ? static_cast<unsigned>(pp[e]) : 0u;
    const unsigned b = active ? static_cast<unsigned>(tt[e]) : 0u;
    const unsigned long long pair = (static_cast<unsigned long long>(a) << 32) | b;
    ok &= wave_insert<unsigned long long>(pk, pc, kPairCap, pair, active, kEmpty64);
    ok &= wave_insert<unsigned>(sk[0], sc[0], kSegCap, a, active, kEmpty32);
    ok &= wave_insert<unsigned>(sk[1], sc[1], kSegCap, b, active, kEmpty32);
  }
  if (!ok) atomicOr(&bad, 1);
  __syncthreads();
  for (int i = tid; i < kPairCap; i += kThreads) {
    out_pair_keys[img * kPairCap + i] = pk[i];
    out_pair_cnt[img * kPairCap + i] = pc[i];
  }
  for (int i = tid; i < kSegCap; i += kThreads) {
    out_p_keys[img * kSegCap + i] = sk[0][i];
    out_p_cnt[img * kSegCap + i] = sc[0][i];
    out_t_keys[img * kSegCap + i] = sk[1][i];
    out_t_cnt[img * kSegCap + i] = sc[1][i];
  }
  if (tid == 0 && bad) atomicOr(overflow, 1);
}

}  // namespace

// pcode / tcode: int32 [B, P] segment codes (category index * n_inst + instance, < 2^32 - 1).  Returns
// (pair_keys u64-as-int64 [B, 4096], pair_counts i32 [B, 4096], pred_keys i32 [B, 1024], pred_counts,
//  target_keys, target_counts, overflow i32 [1]); empty slots hold key -1 and count 0.
std::vector<at::Tensor> panoptic_tables(const at::Tensor& pcode, const at::Tensor& tcode) {
  TM_CHECK_CUDA(pcode);
  TM_SAME_DEVICE(pcode, tcode);
  TORCH_CHECK(pcode.scalar_type() == at::kInt && tcode.scalar_type() == at::kInt && pcode.dim() == 2 &&
                  pcode.sizes() == tcode.sizes() && pcode.is_contiguous() && tcode.is_contiguous(),
              "panoptic_tables: int32 [B, P] contiguous codes");
  const long long B = pcode.size(0), P = pcode.size(1);
  auto i64 = pcode.options().dtype(at::kLong);
  auto i32 = pcode.options();
  at::Tensor pair_keys = at::empty({B, kPairCap}, i64), pair_cnt = at::empty({B, kPairCap}, i32);
  at::Tensor p_keys = at::empty({B, kSegCap}, i32), p_cnt = at::empty({B, kSegCap}, i32);
  at::Tensor t_keys = at::empty({B, kSegCap}, i32), t_cnt = at::empty({B, kSegCap}, i32);
  at::Tensor overflow = at::zeros({1}, i32);
  if (B > 0) {
    TORCH_CHECK(B < (1LL << 31), "panoptic_tables: too many images");
    hipLaunchKernelGGL(panoptic_tables_kernel, dim3(static_cast<unsigned>(B)), dim3(kThreads), 0, stream(),
                       pcode.data_ptr<int>(), tcode.data_ptr<int>(), P,
                       reinterpret_cast<unsigned long long*>(pair_keys.data_ptr<int64_t>()),
                       reinterpret_cast<unsigned*>(pair_cnt.data_ptr<int>()),
                       reinterpret_cast<unsigned*>(p_keys.data_ptr<int>()), reinterpret_cast<unsigned*>(p_cnt.data_ptr<int>()),
                       reinterpret_cast<unsigned*>(t_keys.data_ptr<int>()), reinterpret_cast<unsigned*>(t_cnt.data_ptr<int>()),
                       overflow.data_ptr<int>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
  return {pair_keys, pair_cnt, p_keys, p_cnt, t_keys, t_cnt, overflow};
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("panoptic_tables(Tensor pcode, Tensor tcode) -> Tensor[]"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("panoptic_tables", &panoptic_tables); }

}  // namespace tm_amd
