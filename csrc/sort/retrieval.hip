// Retrieval metrics for every query at once: (query, score desc) radix sort + one wave per query (gfx950).
//
// Reference behaviour: S/retrieval/base.py:147-190 sorts by query index, copies the group sizes to the host and
// loops over queries in Python, calling one small ``F/retrieval/*.py`` function per query (a topk/argsort each).
// Here:
//   1. two stable rocPRIM radix sorts order the documents by (query id, score descending): the first over the
//      order-preserving score key (value = document id), the second over the sign-flipped 64-bit query id;
//   2. ``retrieval_segments_kernel`` flags query starts, and a rocPRIM inclusive scan turns the flags into query ids;
//      query begin offsets and the query count stay on the device;
//   3. ``retrieval_metric_kernel``: one 64-lane wave per query (grid-stride over the device-side query count) walks
//      its documents in 64-wide chunks with wave scans -- relevant counts, first hit, top-k windows and, for AUROC
//      and NDCG, the tie-run scan (tie-averaged gains / trapezoids over groups of equal scores, as sklearn);
//   4. NDCG's ideal DCG reads a second (query, target desc) key sort.
// Result: per-query value + "empty" flag (no relevant -- or for fall-out no non-relevant -- document); aggregation
// and the empty-query policy are applied on the device by the caller.
#include <rocprim/device/device_scan.hpp>

#include "sort/sortscan.h"

namespace tm_amd {
namespace {

using sortscan::desc_key32;
using sortscan::desc_key32_decode;
using sortscan::desc_key64;

enum Kind : int { kMAP = 0, kMRR, kPrecision, kRecall, kFallOut, kHitRate, kRPrecision, kNDCG, kAUROC };

// 3-channel tie-run record (same algebra as csrc/sort/clf_curve.hip's RunRec)
struct Rec3 {
  double v[3];
  double s[3];
  int starts, has;
};

__device__ __forceinline__ Rec3 rec3_identity() {
  Rec3 r;
#pragma unroll
  for (int k = 0; k < 3; ++k) r.v[k] = r.s[k] = 0.0;
  r.starts = r.has = 0;
  return r;
}

struct Rec3Op {
  __device__ __forceinline__ Rec3 operator()(const Rec3& a, const Rec3& b) const {
    Rec3 r;
#pragma unroll
    for (int k = 0; k < 3; ++k) r.v[k] = a.v[k] + b.v[k];
    r.starts = a.starts + b.starts;
    if (b.has) {
#pragma unroll
      for (int k = 0; k < 3; ++k) r.s[k] = a.v[k] + b.s[k];
      r.has = 1;
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) r.s[k] = a.s[k];
      r.has = a.has;
    }
    return r;
  }
};

template <typename scalar_t>
__global__ void score_keys_kernel(const scalar_t* __restrict__ preds, int64_t n, uint64_t* __restrict__ keys,
                                  int32_t* __restrict__ vals) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if constexpr (std::is_same<scalar_t, double>::value) keys[i] = desc_key64(preds[i]);
    else keys[i] = static_cast<uint64_t>(desc_key32(to_f32(preds[i])));
    vals[i] = static_cast<int32_t>(i);
  }
}

__global__ void query_keys_kernel(const int64_t* __restrict__ indexes, const int32_t* __restrict__ vals, int64_t n,
                                  uint64_t* __restrict__ keys) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = static_cast<uint64_t>(indexes[vals[i]]) ^ 0x8000000000000000ULL;
}

// start flags of the sorted query keys (int32 1/0) -> scanned into query ids by rocPRIM
__global__ void query_flags_kernel(const uint64_t* __restrict__ qkeys, int64_t n, int32_t* __restrict__ flags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flags[i] = (i == 0 || qkeys[i] != qkeys[i - 1]) ? 1 : 0;
}

// qid[i] = inclusive count - 1; begin[qid] = i at starts; begin[nq] = n written by the last element
__global__ void query_offsets_kernel(const int32_t* __restrict__ incl, int64_t n, int32_t* __restrict__ begin,
                                     int32_t* __restrict__ nq) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = incl[i] - 1;
    if (i == 0 || incl[i] != incl[i - 1]) begin[q] = static_cast<int32_t>(i);
    if (i == n - 1) {
      begin[q + 1] = static_cast<int32_t>(n);
      nq[0] = q + 1;
    }
  }
}

// (query id << 32 | desc(target)) keys for the ideal-DCG order
template <typename target_t>
__global__ void ideal_keys_kernel(const target_t* __restrict__ target, const int32_t* __restrict__ vals,
                                  const int32_t* __restrict__ incl, int64_t n, uint64_t* __restrict__ keys) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = (static_cast<uint64_t>(incl[i] - 1) << 32) |
              static_cast<uint64_t>(desc_key32(static_cast<float>(to_f32(target[vals[i]]))));
}

template <typename T>
__device__ __forceinline__ double tval(const T* t, int64_t i) {
  return static_cast<double>(to_f32(t[i]));
}
__device__ __forceinline__ double tval(const double* t, int64_t i) { return t[i]; }
__device__ __forceinline__ double tval(const int64_t* t, int64_t i) { return static_cast<double>(t[i]); }
__device__ __forceinline__ double tval(const int32_t* t, int64_t i) { return static_cast<double>(t[i]); }
__device__ __forceinline__ double tval(const uint8_t* t, int64_t i) { return static_cast<double>(t[i]); }

template <typename scalar_t>
__device__ __forceinline__ uint64_t score_key(const scalar_t* p, int64_t i) {
  if constexpr (std::is_same<scalar_t, double>::value) return desc_key64(p[i]);
  else return static_cast<uint64_t>(desc_key32(to_f32(p[i])));
}

__device__ __forceinline__ double wave_min_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off, kWave));
  return v;
}

template <typename scalar_t, typename target_t>
__global__ __launch_bounds__(256) void retrieval_metric_kernel(const scalar_t* __restrict__ preds,
                                                               const target_t* __restrict__ target,
                                                               const int32_t* __restrict__ vals,
                                                               const int32_t* __restrict__ begin,
                                                               const int32_t* __restrict__ nq_ptr,
                                                               const uint64_t* __restrict__ ideal, int kind,
                                                               int64_t top_k, bool adaptive_k,
                                                               double* __restrict__ out, uint8_t* __restrict__ empty) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  const int nq = nq_ptr[0];
  Rec3Op op;
  for (int64_t q = wave; q < nq; q += nwaves) {
    const int64_t b = begin[q], e = begin[q + 1];
    const int64_t size = e - b;
    const int64_t K = top_k > 0 ? top_k : size;
    // pass A: totals
    double rel = 0.0, nonrel = 0.0;
    for (int64_t c = b; c < e; c += kWave) {
      const int64_t i = c + lane;
      if (i < e) {
        const double t = tval(target, vals[i]);
        rel += t > 0.0 ? 1.0 : 0.0;
        nonrel += t > 0.0 ? 0.0 : 1.0;
      }
    }
    rel = wave_sum(rel);
    nonrel = wave_sum(nonrel);
    double value = 0.0;
    const int64_t Kw = kind == kRPrecision ? static_cast<int64_t>(rel) : K;
    if (kind == kNDCG || kind == kAUROC) {
      // tie-run scan: NDCG channels (gain, discount, count); AUROC channels (pos, neg, -) inside the top K
      Rec3 carry = rec3_identity();
      double acc = 0.0;
      for (int64_t c = b; c < e; c += kWave) {
        const int64_t i = c + lane;
        const bool in = i < e;
        const int64_t pos = i - b;
        uint64_t key = 0, nkey = 0, pkey = 0;
        double t = 0.0;
        if (in) {
          key = score_key(preds, vals[i]);
          t = tval(target, vals[i]);
          if (i > b) pkey = score_key(preds, vals[i - 1]);
          if (i + 1 < e) nkey = score_key(preds, vals[i + 1]);
        }
        const bool start = in && (i == b || pkey != key);
        const bool end = in && (i + 1 == e || nkey != key);
        Rec3 r = rec3_identity();
        if (in) {
          if (kind == kNDCG) {
            r.v[0] = t;
            r.v[1] = pos < K ? 1.0 / log2(static_cast<double>(pos) + 2.0) : 0.0;
            r.v[2] = 1.0;
          } else {
            const double w = pos < K ? 1.0 : 0.0;
            r.v[0] = t > 0.0 ? w : 0.0;
            r.v[1] = t > 0.0 ? 0.0 : w;
          }
          r.starts = r.has = start ? 1 : 0;
        }
        Rec3 inc = sortscan::wave_inclusive_scan(r, op);
        const Rec3 run = op(carry, inc);
        if (end) {
          if (kind == kNDCG) {
            const double g = run.v[0] - run.s[0], d = run.v[1] - run.s[1], n = run.v[2] - run.s[2];
            acc += g / n * d;
          } else {
            const double pr = run.v[0] - run.s[0], nr = run.v[1] - run.s[1];
            acc += nr * (run.s[0] + 0.5 * pr);
          }
        }
        Rec3 last;
        {
          // broadcast lane 63's inclusive record (the chunk aggregate)
          const int* src = reinterpret_cast<const int*>(&inc);
          int* dst = reinterpret_cast<int*>(&last);
#pragma unroll
          for (int w = 0; w < static_cast<int>(sizeof(Rec3) / 4); ++w) dst[w] = __shfl(src[w], kWave - 1, kWave);
        }
        carry = op(carry, last);
      }
      acc = wave_sum(acc);
      if (kind == kNDCG) {
        double idcg = 0.0;
        for (int64_t c = b; c < e; c += kWave) {
          const int64_t i = c + lane;
          const int64_t pos = i - b;
          if (i < e && pos < K)
            idcg += static_cast<double>(desc_key32_decode(static_cast<uint32_t>(ideal[i] & 0xffffffffULL))) /
                    log2(static_cast<double>(pos) + 2.0);
        }
        idcg = wave_sum(idcg);
        value = idcg == 0.0 ? 0.0 : acc / idcg;
      } else {
        const double P = carry.v[0], N = carry.v[1];
        value = (P > 0.0 && N > 0.0) ? acc / (P * N) : 0.0;
      }
    } else {
      double hits = 0.0, misses = 0.0, ap = 0.0, first = 1e300, cum = 0.0;
      for (int64_t c = b; c < e; c += kWave) {
        const int64_t i = c + lane;
        const int64_t pos = i - b;
        const bool in = i < e && pos < Kw;
        const double t = i < e ? tval(target, vals[i]) : 0.0;
        const bool h = in && t > 0.0;
        double hv = h ? 1.0 : 0.0;
        // inclusive count of hits (MAP)
        double incl = hv;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
          const double o = __shfl_up(incl, d, kWave);
          if (lane >= d) incl += o;
        }
        if (h) {
          ap += (cum + incl) / static_cast<double>(pos + 1);
          first = fmin(first, static_cast<double>(pos));
        }
        if (in && !(t > 0.0)) misses += 1.0;
        cum += __shfl(incl, kWave - 1, kWave);
        hits += hv;
      }
      hits = wave_sum(hits);
      misses = wave_sum(misses);
      ap = wave_sum(ap);
      first = wave_min_d(first);
      switch (kind) {
        case kMAP: value = hits > 0.0 ? ap / hits : 0.0; break;
        case kMRR: value = first < 1e300 ? 1.0 / (first + 1.0) : 0.0; break;
        case kPrecision: {
          const double k = (adaptive_k && top_k > 0) ? static_cast<double>(K < size ? K : size) : static_cast<double>(K);
          value = hits / k;
          break;
        }
        case kRecall: value = rel > 0.0 ? hits / rel : 0.0; break;
        case kFallOut: value = nonrel > 0.0 ? misses / nonrel : 0.0; break;
        case kHitRate: value = hits > 0.0 ? 1.0 : 0.0; break;
        case kRPrecision: value = rel > 0.0 ? hits / rel : 0.0; break;
        default: break;
      }
    }
    if (lane == 0) {
      out[q] = value;
      empty[q] = kind == kFallOut ? (nonrel == 0.0) : (rel == 0.0);
    }
  }
}

// largest query size -> nq[1] (vector atomics; nq[1] zeroed by the caller)
__global__ void query_max_size_kernel(const int32_t* __restrict__ begin, int32_t* __restrict__ nq) {
  const int n_q = nq[0];
  int m = 0;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n_q; q += gridDim.x * blockDim.x)
    m = max(m, begin[q + 1] - begin[q]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off, kWave));
  if ((threadIdx.x & (kWave - 1)) == 0 && m > 0) atomicMax(nq + 1, m);
}

// Precision@k / recall@k for k = 1..K of every query (reference F/retrieval/precision_recall_curve.py:87-99 per
// query).  One wave per query walks k in 64-wide chunks: a wave inclusive scan of the relevance of the documents at
// rank k gives the hit count of the top k; ranks past the query's size add nothing (the reference pads with zeros).
// Denominators: k, or min(k, size) with adaptive_k; recall divides by the query's relevant count.  Queries without a
// relevant document write zeros and set ``empty`` (the empty-target policy is applied by the caller).
template <typename target_t>
__global__ __launch_bounds__(256) void retrieval_pr_curve_kernel(const target_t* __restrict__ target,
                                                                 const int32_t* __restrict__ order,
                                                                 const int32_t* __restrict__ begin, int n_q,
                                                                 int64_t K, bool adaptive_k, float* __restrict__ prec,
                                                                 float* __restrict__ rec, uint8_t* __restrict__ empty) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t q = wave; q < n_q; q += nwaves) {
    const int64_t b = begin[q], e = begin[q + 1];
    const int64_t size = e - b;
    double rel = 0.0;
    for (int64_t i = b + lane; i < e; i += kWave) rel += tval(target, order[i]) > 0.0 ? 1.0 : 0.0;
    rel = wave_sum(rel);
    float* pq = prec + q * K;
    float* rq = rec + q * K;
    double cum = 0.0;
    for (int64_t c = 0; c < K; c += kWave) {
      const int64_t k = c + lane;  // rank k (0-based) -> top (k + 1)
      double hv = (k < size && k < K && tval(target, order[b + k]) > 0.0) ? 1.0 : 0.0;
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const double o = __shfl_up(hv, d, kWave);
        if (lane >= d) hv += o;
      }
      const double hits = cum + hv;
      if (k < K) {
        const double denom = adaptive_k ? static_cast<double>(k + 1 < size ? k + 1 : size) : static_cast<double>(k + 1);
        pq[k] = rel > 0.0 ? static_cast<float>(hits / denom) : 0.0f;
        rq[k] = rel > 0.0 ? static_cast<float>(hits / rel) : 0.0f;
      }
      cum += __shfl(hv, kWave - 1, kWave);
      if (c + kWave >= size) {
        // every document of the query is counted: the rest of the row only changes through its denominator
        for (int64_t k2 = c + kWave + lane; k2 < K; k2 += kWave) {
          const double denom =
              adaptive_k ? static_cast<double>(k2 + 1 < size ? k2 + 1 : size) : static_cast<double>(k2 + 1);
          pq[k2] = rel > 0.0 ? static_cast<float>(cum / denom) : 0.0f;
          rq[k2] = rel > 0.0 ? static_cast<float>(cum / rel) : 0.0f;
        }
        break;
      }
    }
    if (lane == 0) empty[q] = rel == 0.0;
  }
}

}  // namespace

namespace {

// Documents ordered by (query id, score descending) plus the device-side query table.
struct QuerySegments {
  at::Tensor order;   // int32 [n]: document ids in (query, score desc) order
  at::Tensor begin;   // int32 [n + 1]: first sorted position of each query (first nq + 1 valid)
  at::Tensor nq;      // int32 [2]: query count, largest query size (the latter filled by retrieval_pr_curve only)
  at::Tensor incl;    // int32 [n]: 1-based query id of each sorted position
  at::Tensor scratch; // int64 [n]: free 64-bit key buffer after segmentation
};

void check_flat_inputs(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& indexes,
                       const char* name) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, indexes);
  TORCH_CHECK(preds.dim() == 1 && target.numel() == preds.numel() && indexes.numel() == preds.numel(), name,
              ": flat inputs of equal size expected");
  TORCH_CHECK(indexes.scalar_type() == at::kLong, name, ": indexes must be int64");
  TORCH_CHECK(preds.is_contiguous() && target.is_contiguous() && indexes.is_contiguous(), name,
              ": contiguous inputs expected");
  TORCH_CHECK(preds.numel() > 0 && preds.numel() < (1LL << 31), name, ": 0 < n < 2^31 documents");
}

QuerySegments segment_queries(const at::Tensor& preds, const at::Tensor& indexes, hipStream_t st) {
  const int64_t n = preds.numel();
  const auto dev = preds.device();
  auto i64 = at::TensorOptions().dtype(at::kLong).device(dev);
  auto i32 = at::TensorOptions().dtype(at::kInt).device(dev);
  QuerySegments s;
  s.nq = at::zeros({2}, i32);
  auto ka = at::empty({n}, i64), kb = at::empty({n}, i64);
  auto va = at::empty({n}, i32), vb = at::empty({n}, i32);
  auto* a = reinterpret_cast<uint64_t*>(ka.data_ptr());
  auto* bk = reinterpret_cast<uint64_t*>(kb.data_ptr());
  const int grid = grid_cap((n + 255) / 256);
  const bool f64 = preds.scalar_type() == at::kDouble;
  TM_DISPATCH_FLOAT(preds.scalar_type(), "retrieval", [&] {
    hipLaunchKernelGGL((score_keys_kernel<scalar_t>), dim3(grid), dim3(256), 0, st, preds.data_ptr<scalar_t>(), n, a,
                       va.data_ptr<int32_t>());
  });
  sortscan::sort_pairs<uint64_t, int32_t>(a, bk, va.data_ptr<int32_t>(), vb.data_ptr<int32_t>(), n, 0, f64 ? 64 : 32,
                                          dev, st);
  hipLaunchKernelGGL(query_keys_kernel, dim3(grid), dim3(256), 0, st, indexes.data_ptr<int64_t>(),
                     vb.data_ptr<int32_t>(), n, a);
  sortscan::sort_pairs<uint64_t, int32_t>(a, bk, vb.data_ptr<int32_t>(), va.data_ptr<int32_t>(), n, 0, 64, dev, st);
  // va: document ids in (query, score desc) order; bk: sorted query keys
  auto flags = at::empty({n}, i32);
  s.incl = at::empty({n}, i32);
  s.begin = at::empty({n + 1}, i32);
  hipLaunchKernelGGL(query_flags_kernel, dim3(grid), dim3(256), 0, st, bk, n, flags.data_ptr<int32_t>());
  {
    size_t bytes = 0;
    TORCH_CHECK(rocprim::inclusive_scan(nullptr, bytes, flags.data_ptr<int32_t>(), s.incl.data_ptr<int32_t>(),
                                        static_cast<size_t>(n), rocprim::plus<int32_t>(), st) == hipSuccess,
                "retrieval: scan size query failed");
    auto tmp = at::empty({static_cast<int64_t>(bytes) + 16}, at::TensorOptions().dtype(at::kByte).device(dev));
    TORCH_CHECK(rocprim::inclusive_scan(tmp.data_ptr(), bytes, flags.data_ptr<int32_t>(), s.incl.data_ptr<int32_t>(),
                                        static_cast<size_t>(n), rocprim::plus<int32_t>(), st) == hipSuccess,
                "retrieval: scan failed");
  }
  hipLaunchKernelGGL(query_offsets_kernel, dim3(grid), dim3(256), 0, st, s.incl.data_ptr<int32_t>(), n,
                     s.begin.data_ptr<int32_t>(), s.nq.data_ptr<int32_t>());
  s.order = va;
  s.scratch = ka;
  return s;
}

}  // namespace

// preds [n] float, target [n] (int/bool/float), indexes [n] int64.
// Returns (values fp64 [n] (first n_queries valid), empty uint8 [n], n_queries int32 [1]).
std::vector<at::Tensor> retrieval_metric(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& indexes,
                                         int64_t kind, int64_t top_k, bool adaptive_k) {
  check_flat_inputs(preds, target, indexes, "retrieval_metric");
  const int64_t n = preds.numel();
  const auto dev = preds.device();
  auto st = stream();
  auto values = at::empty({n}, at::TensorOptions().dtype(at::kDouble).device(dev));
  auto empty = at::empty({n}, at::TensorOptions().dtype(at::kByte).device(dev));
  QuerySegments s = segment_queries(preds, indexes, st);
  auto nq = s.nq.narrow(0, 0, 1);
  auto va = s.order;
  auto incl = s.incl;
  auto begin = s.begin;
  auto* a = reinterpret_cast<uint64_t*>(s.scratch.data_ptr());
  auto i64 = at::TensorOptions().dtype(at::kLong).device(dev);
  const int grid = grid_cap((n + 255) / 256);
  const uint64_t* ideal = nullptr;
  at::Tensor ik_sorted;
  if (kind == kNDCG) {
    ik_sorted = at::empty({n}, i64);
    TM_DISPATCH_PREDS(target.scalar_type(), "retrieval_metric", [&] {
      hipLaunchKernelGGL((ideal_keys_kernel<scalar_t>), dim3(grid), dim3(256), 0, st,
                         reinterpret_cast<const scalar_t*>(target.data_ptr()), va.data_ptr<int32_t>(),
                         incl.data_ptr<int32_t>(), n, a);
    });
    sortscan::sort_keys<uint64_t>(a, reinterpret_cast<uint64_t*>(ik_sorted.data_ptr()), n, 0,
                                  32 + sortscan::ceil_log2(n + 1), dev, st);
    ideal = reinterpret_cast<const uint64_t*>(ik_sorted.data_ptr());
  }
  const int mgrid = grid_cap((n * kWave + 255) / 256, cu_count(dev.index()) * 8);
  TM_DISPATCH_FLOAT(preds.scalar_type(), "retrieval_metric", [&] {
    using pscalar_t = scalar_t;
    TM_DISPATCH_PREDS(target.scalar_type(), "retrieval_metric", [&] {
      hipLaunchKernelGGL((retrieval_metric_kernel<pscalar_t, scalar_t>), dim3(mgrid), dim3(256), 0, st,
                         preds.data_ptr<pscalar_t>(), reinterpret_cast<const scalar_t*>(target.data_ptr()),
                         va.data_ptr<int32_t>(), begin.data_ptr<int32_t>(), nq.data_ptr<int32_t>(), ideal,
                         static_cast<int>(kind), top_k, adaptive_k, values.data_ptr<double>(),
                         empty.data_ptr<uint8_t>());
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {values, empty, nq};
}

// Precision / recall curves of every query: (precision f32 [nq, K], recall f32 [nq, K], empty uint8 [nq]).
// max_k <= 0 means K = the largest query size.  The query count (and largest size) is the one host read, as the
// output shape depends on it (the reference reads all group sizes, S/retrieval/precision_recall_curve.py:198).
std::vector<at::Tensor> retrieval_pr_curve(const at::Tensor& preds, const at::Tensor& target,
                                           const at::Tensor& indexes, int64_t max_k, bool adaptive_k) {
  check_flat_inputs(preds, target, indexes, "retrieval_pr_curve");
  const auto dev = preds.device();
  auto st = stream();
  QuerySegments s = segment_queries(preds, indexes, st);
  hipLaunchKernelGGL(query_max_size_kernel, dim3(grid_cap((preds.numel() + 255) / 256, 1024)), dim3(256), 0, st,
                     s.begin.data_ptr<int32_t>(), s.nq.data_ptr<int32_t>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  const auto host = s.nq.to(at::kCPU);  // the one device->host read
  const int n_q = host.data_ptr<int32_t>()[0];
  const int64_t K = max_k > 0 ? max_k : static_cast<int64_t>(host.data_ptr<int32_t>()[1]);
  TORCH_CHECK(static_cast<double>(n_q) * static_cast<double>(K) < 9.0e18, "retrieval_pr_curve: output too large");
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
  auto prec = at::empty({n_q, K}, f32);
  auto rec = at::empty({n_q, K}, f32);
  auto empty = at::empty({n_q}, at::TensorOptions().dtype(at::kByte).device(dev));
  if (n_q > 0 && K > 0) {
    const int grid = grid_cap((static_cast<int64_t>(n_q) * kWave + 255) / 256, cu_count(dev.index()) * 8);
    TM_DISPATCH_PREDS(target.scalar_type(), "retrieval_pr_curve", [&] {
      hipLaunchKernelGGL((retrieval_pr_curve_kernel<scalar_t>), dim3(grid), dim3(256), 0, st,
                         reinterpret_cast<const scalar_t*>(target.data_ptr()), s.order.data_ptr<int32_t>(),
                         s.begin.data_ptr<int32_t>(), n_q, K, adaptive_k, prec.data_ptr<float>(),
                         rec.data_ptr<float>(), empty.data_ptr<uint8_t>());
    });
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
  return {prec, rec, empty};
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("retrieval_metric(Tensor preds, Tensor target, Tensor indexes, int kind, int top_k, bool adaptive_k) -> Tensor[]");
  m.def("retrieval_pr_curve(Tensor preds, Tensor target, Tensor indexes, int max_k, bool adaptive_k) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("retrieval_metric", &tm_amd::retrieval_metric);
  m.impl("retrieval_pr_curve", &tm_amd::retrieval_pr_curve);
}
