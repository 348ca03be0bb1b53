// Top-k multiclass predictions (K3): top_k > 1 stat scores fused with the top-k selection, plus the
// bare top-k labels.
//
// Reference (F/classification/stat_scores.py `_refine_preds_oh` / `_multiclass_stat_scores_update`):
// `preds.topk(k, dim=1)` + a one-hot scatter of [N, C] + the tp/fp/fn algebra over dense [N, C] tensors.  Here one wave
// owns one row and nothing row-sized leaves registers:
//   * every score becomes a 64-bit packed key (order-preserving u32 of the fp32 value, NaN highest, -0 == +0) << 32 |
//     ~column, so "larger key" is exactly torch's order with ties to the smaller column and one u64 compare decides;
//   * each lane keeps a sorted top-k of the keys it sees (KP register slots, KP = k rounded up to 2 / 4 / 8 / 16, all
//     indices compile-time) behind an admission threshold; loads go 4 x 16 B per lane per step so a row's loads are in
//     flight together (a single dependent load chain per wave made the first version of this kernel latency-bound),
//     and a per-step wave bound (K-th largest lane maximum) filters what reaches the lists;
//   * k rounds of a wave u64 max pop the row's top-k in descending order; lane r keeps the r-th label;
//   * stats: hit = any(label_r == target); lanes with a miss add fp[label], lane 0 adds tp/fn[target] -- the same
//     [G, 3C+1] workspace as mc_update, finalised by mc_stats_finalize.  Histogram privatised in LDS.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kMaxK = 16;
constexpr int kBlockT = 256;
constexpr int kLoads = 4;  // 16-byte loads in flight per lane per step
constexpr int kLdsBinsT = 12288;
using u64 = unsigned long long;

__device__ __forceinline__ u64 pack_key(float f, int col) {
  unsigned u = __float_as_uint(f == 0.f ? 0.f : f);
  u = (f != f) ? 0xffffffffu : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
  return (static_cast<u64>(u) << 32) | static_cast<unsigned>(~col);
}

__device__ __forceinline__ int key_col(u64 key) { return static_cast<int>(~static_cast<unsigned>(key)); }

template <int KP>
struct LaneTopK {
  u64 s[KP];  // descending; unused slots 0 (below every real key)
  u64 thr;    // slot K-1: a key must beat it to enter

  __device__ __forceinline__ void init() {
#pragma unroll
    for (int q = 0; q < KP; ++q) s[q] = 0;
    thr = 0;
  }
  __device__ __forceinline__ void offer(u64 key, int K) {
    if (key <= thr) return;
#pragma unroll
    for (int q = KP - 1; q >= 1; --q) {
      if (q < K) {
        const u64 up = s[q - 1];
        s[q] = key > up ? up : (key > s[q] ? key : s[q]);
      }
    }
    s[0] = key > s[0] ? key : s[0];
#pragma unroll
    for (int q = 0; q < KP; ++q)
      if (q == K - 1) thr = s[q];
  }
  // k rounds of a wave max over the lanes' heads; lane r returns the r-th label (lanes >= K return -1)
  __device__ __forceinline__ int pop_wave(int K, int lane) {
    int mine = -1;
    for (int r = 0; r < K; ++r) {
      u64 w = s[0];
#pragma unroll
      for (int off = kWave / 2; off > 0; off >>= 1) {
        const u64 o = __shfl_xor(w, off, kWave);
        w = o > w ? o : w;
      }
      if (lane == r) mine = key_col(w);
      if (s[0] == w) {  // keys are unique (the column is in them): exactly one lane owned the winner
#pragma unroll
        for (int q = 0; q < KP - 1; ++q) s[q] = s[q + 1];
        s[KP - 1] = 0;
      }
    }
    return mine;
  }
};

// K-th largest of the lanes' values (0 when fewer than K lanes hold one): K rounds of a wave max
__device__ __forceinline__ u64 wave_kth(u64 v, int K) {
  u64 w = 0;
  for (int r = 0; r < K; ++r) {
    w = v;
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
      const u64 o = __shfl_xor(w, off, kWave);
      w = o > w ? o : w;
    }
    if (v == w) v = 0;
  }
  return w;
}

// scan one [C] row into the lane's list (vec: 16-B aligned rows with C * sizeof % 16 == 0).  Per step: all loads
// first, then a bound = the K-th largest lane maximum of the step (K distinct elements reach it, so every top-k
// element of the row that lies in this step does too); only keys >= bound are offered, which leaves most offer
// slots with an empty exec mask.
template <typename scalar_t, int KP>
__device__ __forceinline__ void scan_row(const scalar_t* __restrict__ rp, int C, int K, bool vec, int lane,
                                         LaneTopK<KP>& tk) {
  if (vec) {
    constexpr int kVec = 16 / sizeof(scalar_t);
    for (int base = 0; base < C; base += kWave * kVec * kLoads) {
      uint4 raw[kLoads];
#pragma unroll
      for (int u = 0; u < kLoads; ++u) {
        const int c0 = base + (u * kWave + lane) * kVec;
        raw[u] = c0 < C ? *reinterpret_cast<const uint4*>(rp + c0) : make_uint4(0, 0, 0, 0);
      }
      u64 lm = 0;
#pragma unroll
      for (int u = 0; u < kLoads; ++u) {
        const int c0 = base + (u * kWave + lane) * kVec;
        const scalar_t* e = reinterpret_cast<const scalar_t*>(&raw[u]);
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
          const u64 key = c0 < C ? pack_key(to_f32(e[j]), c0 + j) : 0;
          lm = key > lm ? key : lm;
        }
      }
      const u64 bound = wave_kth(lm, K);
#pragma unroll
      for (int u = 0; u < kLoads; ++u) {
        const int c0 = base + (u * kWave + lane) * kVec;
        const scalar_t* e = reinterpret_cast<const scalar_t*>(&raw[u]);
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
          const u64 key = c0 < C ? pack_key(to_f32(e[j]), c0 + j) : 0;
          if (key != 0 && key >= bound) tk.offer(key, K);
        }
      }
    }
  } else {
    constexpr int kE = 8;
    for (int base = 0; base < C; base += kWave * kE) {
      u64 key[kE];
      u64 lm = 0;
#pragma unroll
      for (int u = 0; u < kE; ++u) {
        const int c = base + u * kWave + lane;
        key[u] = c < C ? pack_key(to_f32(rp[c]), c) : 0;
      }
#pragma unroll
      for (int u = 0; u < kE; ++u) lm = key[u] > lm ? key[u] : lm;
      const u64 bound = wave_kth(lm, K);
#pragma unroll
      for (int u = 0; u < kE; ++u)
        if (key[u] != 0 && key[u] >= bound) tk.offer(key[u], K);
    }
  }
}

template <typename scalar_t, int KP>
__global__ void __launch_bounds__(kBlockT) topk_labels_kernel(const scalar_t* __restrict__ preds, long long N, int C,
                                                              int K, bool vec, int* __restrict__ out) {
  const int lane = threadIdx.x & (kWave - 1);
  const long long wave = (static_cast<long long>(blockIdx.x) * kBlockT + threadIdx.x) / kWave;
  const long long nwaves = static_cast<long long>(gridDim.x) * (kBlockT / kWave);
  for (long long row = wave; row < N; row += nwaves) {
    LaneTopK<KP> tk;
    tk.init();
    scan_row<scalar_t, KP>(preds + row * C, C, K, vec, lane, tk);
    const int lab = tk.pop_wave(K, lane);
    if (lane < K) out[row * K + lane] = lab;
  }
}

template <typename scalar_t, typename target_t, int KP>
__global__ void __launch_bounds__(kBlockT) topk_stats_kernel(const scalar_t* __restrict__ preds,
                                                             const target_t* __restrict__ target, long long N, int C,
                                                             int K, bool vec, long long ignore, bool has_ignore,
                                                             bool samplewise, bool use_lds, int64_t* __restrict__ ws,
                                                             int* __restrict__ flag) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const int nbins = 3 * C + 1;
  if (use_lds) {
    for (int b = threadIdx.x; b < nbins; b += kBlockT) lds[b] = 0;
    __syncthreads();
  }
  const int lane = threadIdx.x & (kWave - 1);
  const long long wave = (static_cast<long long>(blockIdx.x) * kBlockT + threadIdx.x) / kWave;
  const long long nwaves = static_cast<long long>(gridDim.x) * (kBlockT / kWave);
  for (long long row = wave; row < N; row += nwaves) {
    const long long tv = static_cast<long long>(target[row]);  // same address in every lane: one fetch
    LaneTopK<KP> tk;
    tk.init();
    scan_row<scalar_t, KP>(preds + row * C, C, K, vec, lane, tk);
    const int lab = tk.pop_wave(K, lane);
    if (has_ignore && tv == ignore) continue;
    if (tv < 0 || tv >= C) {
      if (lane == 0) raise_flag(flag, kErrTargetOutOfRange);
      continue;
    }
    const int t = static_cast<int>(tv);
    const bool hit = __any(lane < K && lab == t);
    const int slot = hit ? t : 2 * C + t;
    if (use_lds) {
      if (lane < K && lab != t) atomicAdd(&lds[C + lab], 1);
      if (lane == 0) atomicAdd(&lds[slot], 1);
    } else {
      int64_t* g = ws + (samplewise ? row : 0) * static_cast<long long>(nbins);
      if (lane < K && lab != t) atomic_add_i64(g + C + lab, 1);
      if (lane == 0) atomic_add_i64(g + slot, 1);  // the row count is derived from tp + fn at finalize
    }
  }
  if (use_lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += kBlockT) {
      const int v = lds[b];
      if (v) atomic_add_i64(ws + b, v);
    }
  }
}

int slots_for(int k) { return k <= 2 ? 2 : (k <= 4 ? 4 : (k <= 8 ? 8 : 16)); }

template <typename F>
void with_slots(int k, F&& f) {
  switch (slots_for(k)) {
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    default: f(std::integral_constant<int, 16>{}); break;
  }
}

#define TM_DISPATCH_HALF_FLOAT(dtype, NAME, ...)                                  \
  [&] {                                                                           \
    switch (dtype) {                                                              \
      case at::kFloat: { using scalar_t = float; return __VA_ARGS__(); }          \
      case at::kHalf: { using scalar_t = c10::Half; return __VA_ARGS__(); }       \
      case at::kBFloat16: { using scalar_t = c10::BFloat16; return __VA_ARGS__(); } \
      default: TORCH_CHECK(false, NAME ": f32 / f16 / bf16 scores, got ", dtype); \
    }                                                                             \
  }()

void check_scores(const at::Tensor& preds, int64_t k, const char* name) {
  TM_CHECK_CUDA(preds);
  TM_CHECK_CONTIG(preds);
  TORCH_CHECK(preds.dim() == 2, name, ": preds must be [N, C]");
  TORCH_CHECK(preds.size(1) < (1LL << 30), name, ": too many classes");
  TORCH_CHECK(k >= 1 && k <= kMaxK && k <= preds.size(1), name, ": 1 <= k <= min(16, C)");
}

bool rows_vectorisable(const at::Tensor& preds) {
  return (preds.size(1) * preds.element_size()) % 16 == 0 && reinterpret_cast<uintptr_t>(preds.data_ptr()) % 16 == 0;
}

int waves_grid(long long rows, int device) {
  const long long want = (rows + kBlockT / kWave - 1) / (kBlockT / kWave);
  return static_cast<int>(std::max<long long>(1, std::min<long long>(want, 8LL * cu_count(device))));
}

}  // namespace

// preds: [N, C] f32 / f16 / bf16 scores (f64 stays on ATen: the fp32 key could merge distinct doubles).  Returns int32
// [N, k] column indices in descending score order.
at::Tensor topk_labels(const at::Tensor& preds, int64_t k) {
  check_scores(preds, k, "topk_labels");
  const long long N = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  at::Tensor out = at::empty({N, k}, preds.options().dtype(at::kInt));
  if (N == 0) return out;
  const bool vec = rows_vectorisable(preds);
  const int grid = waves_grid(N, preds.get_device());
  TM_DISPATCH_HALF_FLOAT(preds.scalar_type(), "topk_labels", [&] {
    with_slots(static_cast<int>(k), [&](auto kp) {
      constexpr int KP = decltype(kp)::value;
      hipLaunchKernelGGL((topk_labels_kernel<scalar_t, KP>), dim3(grid), dim3(kBlockT), 0, stream(),
                         preds.data_ptr<scalar_t>(), N, C, static_cast<int>(k), vec, out.data_ptr<int>());
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// Fused top-k multiclass stats: ws int64 [G, 3C + 1] (G = N if samplewise else 1), the mc_update stats workspace.
void mc_topk_update(const at::Tensor& preds, const at::Tensor& target, at::Tensor ws, at::Tensor flag, int64_t k,
                    int64_t ignore_index, bool has_ignore, bool samplewise) {
  check_scores(preds, k, "mc_topk_update");
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, ws);
  TM_SAME_DEVICE(preds, flag);
  TM_CHECK_CONTIG(target);
  TM_CHECK_CONTIG(ws);
  const long long N = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  TORCH_CHECK(target.numel() == N, "mc_topk_update: target must be [N]");
  TORCH_CHECK(ws.scalar_type() == at::kLong && ws.numel() == (samplewise ? N : 1) * (3LL * C + 1),
              "mc_topk_update: workspace int64 [G, 3C + 1]");
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "mc_topk_update: flag int32 [1]");
  if (N == 0) return;
  const bool vec = rows_vectorisable(preds);
  const int grid = waves_grid(N, preds.get_device());
  const bool use_lds = !samplewise && 3LL * C + 1 <= kLdsBinsT;
  const size_t lds_bytes = use_lds ? (3 * C + 1) * sizeof(int) : 0;
  TM_DISPATCH_TARGET(target.scalar_type(), "mc_topk_update", [&] {
    TM_DISPATCH_HALF_FLOAT(preds.scalar_type(), "mc_topk_update", [&] {
      with_slots(static_cast<int>(k), [&](auto kp) {
        constexpr int KP = decltype(kp)::value;
        hipLaunchKernelGGL((topk_stats_kernel<scalar_t, target_t, KP>), dim3(grid), dim3(kBlockT), lds_bytes,
                           stream(), preds.data_ptr<scalar_t>(), target.data_ptr<target_t>(), N, C,
                           static_cast<int>(k), vec, ignore_index, has_ignore, samplewise, use_lds,
                           ws.data_ptr<int64_t>(), flag.data_ptr<int>());
      });
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("topk_labels(Tensor preds, int k) -> Tensor");
  m.def("mc_topk_update(Tensor preds, Tensor target, Tensor(a!) ws, Tensor(b!) flag, int k, int ignore_index, "
        "bool has_ignore, bool samplewise) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("topk_labels", &topk_labels);
  m.impl("mc_topk_update", &mc_topk_update);
}

}  // namespace tm_amd
