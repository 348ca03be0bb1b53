// Unbinned classification curves on a segmented radix sort + a tie-run scan engine (gfx950).
//
// Reference behaviour: F/classification/precision_recall_curve.py:28-80 (``_binary_clf_curve``: argsort, distinct
// thresholds, cumsum), F/classification/auroc.py:45-106 and average_precision.py:43-80 (a Python loop over classes,
// one argsort + curve + trapezoid per class).  Here every column of a [M, S] score matrix is one *segment* and all
// segments are processed by the same few launches:
//
//   1. key build: one radix key per element, [ segment | desc-score(32) ] (invalid -> sentinel) + a positive-flag byte
//      -- the sort carries everything the scan needs, no payload and no gathers.  fp64 scores / sample weights use the
//      payload path instead: (desc-score64 -> flat index) sort, then a stable (segment, invalid) sort.
//   2. rocPRIM radix sort over exactly the key bits in use (32 + ceil(log2 S)).
//   3. run_tile_aggregate / run_tile_scan / run_tile_epilogue: a tile-decomposed segmented scan whose element is the
//      associative "tie-run" record {cum pos, cum neg, #run starts, cum (pos, neg) before the latest run start}.
//      At every run end (last element of a group of equal scores) the epilogue knows the run's TP/FP before and after
//      and accumulates: trapezoid AUROC area, step AP, max rank of a positive (coverage), and optionally emits the
//      compacted curve point (fps, tps, threshold) at index run_id -- sklearn's ``_binary_clf_curve`` for every
//      segment at once -- or per-element run ids / run ends for average ranks (Spearman).
//   4. run_finalize: deterministic fixed-order per-segment reduction of the tile partials.
//
// No host synchronisation anywhere: segment/tile counts are shapes; the number of distinct thresholds stays on the
// device (stats[:, 6]) until a caller needs it to size a returned curve.
#include "sort/sortscan.h"

namespace tm_amd {
namespace {

using sortscan::desc_key32;
using sortscan::desc_key32_decode;
using sortscan::desc_key64;

constexpr int kStatCols = 8;  // P, N, area, ap, coverage, spare, nruns, spare

// target interpretation
constexpr int kTgtBinary = 0;      // target[e] == pos_label                          (one segment)
constexpr int kTgtOneVsRest = 1;   // target[e] == segment                            (multiclass columns)
constexpr int kTgtElementwise = 2; // target at the score's own address == pos_label  (multilabel / rows)

// C = int32_t for unit weights (exact counts, half the scan traffic of fp64), double for sample weights
template <typename C>
struct RunRec {
  C p, n;    // inclusive positive / negative weight
  C sp, sn;  // cumulative (p, n) just before the latest run start in range
  int starts;  // number of run starts in range
  int has;     // range contains a run start
};

struct RunOp {
  template <typename C>
  __device__ __forceinline__ RunRec<C> operator()(const RunRec<C>& a, const RunRec<C>& b) const {
    RunRec<C> r;
    r.p = a.p + b.p;
    r.n = a.n + b.n;
    r.starts = a.starts + b.starts;
    if (b.has) {
      r.sp = a.p + b.sp;
      r.sn = a.n + b.sn;
      r.has = 1;
    } else {
      r.sp = a.sp;
      r.sn = a.sn;
      r.has = a.has;
    }
    return r;
  }
};

template <typename C>
__device__ __forceinline__ RunRec<C> run_identity() {
  return RunRec<C>{C(0), C(0), C(0), C(0), 0, 0};
}

template <typename C>
struct Elem {
  uint64_t rk;  // run key: equal rk <=> same score (compared inside one segment only)
  C pw, nw;
  bool valid;
};

// Packed path: the sorted key is [segment | desc-score32] (32-bit key when S == 1) with an invalid element's score
// replaced by the 0xffffffff sentinel (sorts last in its segment; no real score maps to it: the only float whose
// key it would be is a non-canonical NaN), and the sort's 1-byte value carries the positive flag.  Tiles are staged
// through LDS with coalesced loads.
template <typename K>
struct KV8Loader {
  static constexpr bool kStaged = true;
  using key_type = K;
  using count_t = int32_t;
  const K* keys;
  const uint8_t* flags;
  __device__ __forceinline__ Elem<count_t> make(K k, uint8_t f) const {
    Elem<count_t> e;
    const uint32_t lo = static_cast<uint32_t>(k & 0xffffffffULL);
    e.valid = lo != 0xffffffffu && !(f & 0x80);
    e.rk = lo;
    const bool pos = (f & 1) != 0;
    e.pw = (e.valid && pos) ? 1 : 0;
    e.nw = (e.valid && !pos) ? 1 : 0;
    return e;
  }
  __device__ __forceinline__ Elem<count_t> load(int64_t gi) const { return make(keys[gi], flags[gi]); }
  __device__ __forceinline__ double threshold(int64_t gi) const {
    return static_cast<double>(desc_key32_decode(static_cast<uint32_t>(keys[gi] & 0xffffffffULL)));
  }
  __device__ __forceinline__ int64_t origin(int64_t) const { return -1; }
};

// Payload path: the sort carries the flat element id (s * M + e).
//   kKeyed: non-fp64 scores -- the sorted 64-bit key [segment | invalid | desc-score32] gives run key and validity;
//           otherwise (fp64) both come from gathers of the original score / target.
//   kNeedPN: positive / negative weights are needed (curves, AUROC); ranks-only callers skip the target gathers.
template <typename scalar_t, typename target_t, bool kKeyed, bool kNeedPN, typename KT = uint64_t>
struct PayloadLoader {
  static constexpr bool kStaged = false;
  using key_type = KT;
  using count_t = double;
  const KT* keys;  // kKeyed only: [segment | invalid | desc32] (64-bit) or desc32 alone (one segment, no ignore)
  const int32_t* vals;
  const scalar_t* scores;
  const target_t* target;
  const double* weights;  // per element e (binary / one-vs-rest), nullable
  sortscan::FastDiv divM;
  int64_t M, seg_stride, elem_stride;
  int tmode;
  int64_t pos_label, ignore_index;
  bool has_ignore;

  __device__ __forceinline__ void se(int64_t v, int64_t& s, int64_t& e) const {
    s = divM.div(static_cast<uint32_t>(v));
    e = v - s * M;
  }
  __device__ __forceinline__ Elem<double> load(int64_t gi) const {
    const int64_t v = vals[gi];
    int64_t s, e;
    se(v, s, e);
    Elem<double> r;
    bool valid = true;
    int64_t t = 0;
    if (kNeedPN || !kKeyed)
      t = static_cast<int64_t>(tmode == kTgtElementwise ? target[s * seg_stride + e * elem_stride] : target[e]);
    if constexpr (kKeyed) {
      const uint64_t k = keys[gi];
      r.rk = k & 0xffffffffULL;
      if constexpr (sizeof(KT) == 8) valid = ((k >> 32) & 1ULL) == 0ULL;
    } else {
      r.rk = desc_key64(static_cast<double>(scores[s * seg_stride + e * elem_stride]));
      valid = !(has_ignore && t == ignore_index);
    }
    r.valid = valid;
    if constexpr (kNeedPN) {
      const bool pos = tmode == kTgtOneVsRest ? (t == s) : (t == pos_label);
      const double w = weights ? weights[e] : 1.0;
      r.pw = (valid && pos) ? w : 0.0;
      r.nw = (valid && !pos) ? w : 0.0;
    } else {
      r.pw = valid ? 1.0 : 0.0;
      r.nw = 0.0;
    }
    return r;
  }
  __device__ __forceinline__ double threshold(int64_t gi) const {
    if constexpr (kKeyed) {
      return static_cast<double>(desc_key32_decode(static_cast<uint32_t>(keys[gi] & 0xffffffffULL)));
    } else {
      int64_t s, e;
      se(vals[gi], s, e);
      return static_cast<double>(scores[s * seg_stride + e * elem_stride]);
    }
  }
  __device__ __forceinline__ int64_t origin(int64_t gi) const { return vals[gi]; }
};

struct Partial {
  double area, ap, cov, spare;
};

// ----------------------------------------------------------------------------------------------- key building
// Keys are written in INPUT memory order (flat address a, coalesced reads and writes); the segment / element of an
// address comes from one fast division.  Two layouts: column segments (seg_stride 1, elem_stride S: a = e * S + s)
// and row segments (seg_stride M, elem_stride 1: a = s * M + e); anything else is made contiguous by the caller.
struct Layout {
  sortscan::FastDiv div;  // by S (columns) or M (rows)
  bool columns;
  __device__ __forceinline__ void se(uint32_t a, int64_t& s, int64_t& e) const {
    const uint32_t q = div.div(a);
    if (columns) {
      e = q;
      s = a - q * div.d;
    } else {
      s = q;
      e = a - q * div.d;
    }
  }
};

template <typename scalar_t, typename target_t>
__global__ void build_packed_keys_kernel(const scalar_t* __restrict__ scores, const target_t* __restrict__ target,
                                         int64_t total, Layout lay, int tmode, int64_t pos_label, int64_t ignore_index,
                                         bool has_ignore, uint64_t* __restrict__ keys, int32_t* __restrict__ vals,
                                         int64_t M) {
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < total; a += (int64_t)gridDim.x * blockDim.x) {
    int64_t s, e;
    lay.se(static_cast<uint32_t>(a), s, e);
    const float x = to_f32(scores[a]);
    const int64_t t = static_cast<int64_t>(tmode == kTgtElementwise ? target[a] : target[e]);
    const bool invalid = has_ignore && t == ignore_index;
    const uint64_t sk = static_cast<uint64_t>(desc_key32(x));
    keys[a] = (static_cast<uint64_t>(s) << 33) | (static_cast<uint64_t>(invalid) << 32) | sk;
    vals[a] = static_cast<int32_t>(s * M + e);
  }
}

// packed path keys: [segment | desc-score32 or sentinel] + positive flag byte
template <typename scalar_t, typename target_t, typename K>
__global__ void build_kv8_kernel(const scalar_t* __restrict__ scores, const target_t* __restrict__ target,
                                 int64_t total, Layout lay, int tmode, int64_t pos_label, int64_t ignore_index,
                                 bool has_ignore, K* __restrict__ keys, uint8_t* __restrict__ flags) {
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < total; a += (int64_t)gridDim.x * blockDim.x) {
    int64_t s, e;
    lay.se(static_cast<uint32_t>(a), s, e);
    const int64_t t = static_cast<int64_t>(tmode == kTgtElementwise ? target[a] : target[e]);
    const bool invalid = has_ignore && t == ignore_index;
    const bool pos = !invalid && (tmode == kTgtOneVsRest ? (t == s) : (t == pos_label));
    const uint32_t sk = invalid ? 0xffffffffu : desc_key32(to_f32(scores[a]));
    if constexpr (sizeof(K) == 8) keys[a] = (static_cast<uint64_t>(s) << 32) | sk;
    else keys[a] = sk;
    flags[a] = pos ? 1 : 0;
  }
}

// one segment, 32-bit scores: desc-score32 keys, element id values
template <typename scalar_t>
__global__ void build_score_keys32_kernel(const scalar_t* __restrict__ scores, int64_t total, uint32_t* __restrict__ keys,
                                          int32_t* __restrict__ vals) {
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < total; a += (int64_t)gridDim.x * blockDim.x) {
    keys[a] = desc_key32(to_f32(scores[a]));
    vals[a] = static_cast<int32_t>(a);
  }
}

// fp64 scores, pass 1: desc-score64 keys, flat id values
template <typename scalar_t>
__global__ void build_score_keys_kernel(const scalar_t* __restrict__ scores, int64_t total, Layout lay, int64_t M,
                                        uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < total; a += (int64_t)gridDim.x * blockDim.x) {
    int64_t s, e;
    lay.se(static_cast<uint32_t>(a), s, e);
    keys[a] = desc_key64(static_cast<double>(scores[a]));
    vals[a] = static_cast<int32_t>(s * M + e);
  }
}

// fp64 scores, pass 2: stable (segment, invalid) keys from the sorted flat ids
template <typename target_t>
__global__ void build_segment_keys_kernel(const int32_t* __restrict__ vals, const target_t* __restrict__ target,
                                          int64_t total, sortscan::FastDiv divM, int64_t M, int64_t seg_stride,
                                          int64_t elem_stride, int tmode, int64_t ignore_index, bool has_ignore,
                                          uint32_t* __restrict__ keys) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = vals[i];
    const int64_t s = divM.div(static_cast<uint32_t>(v)), e = v - s * M;
    const int64_t t = static_cast<int64_t>(tmode == kTgtElementwise ? target[s * seg_stride + e * elem_stride] : target[e]);
    const bool invalid = has_ignore && t == ignore_index;
    keys[i] = (static_cast<uint32_t>(s) << 1) | static_cast<uint32_t>(invalid);
  }
}

// ----------------------------------------------------------------------------------------------- tile engine
// One thread owns IT consecutive elements of a tile of NT * IT; grid = (tiles per segment, S).
template <int NT, int IT, class L>
__device__ __forceinline__ void load_tile(const L& ld, int64_t seg_base, int64_t M, int64_t tile_e0,
                                          Elem<typename L::count_t> (&el)[IT + 2]) {
  const int64_t e0 = tile_e0 + static_cast<int64_t>(threadIdx.x) * IT;
  if constexpr (L::kStaged) {
    // coalesced cooperative load of the tile (+1 halo element each side) into LDS, padded 1 per 16 so the
    // thread-contiguous reads below do not all fall into one bank
    using K = typename L::key_type;
    constexpr int T = NT * IT;
    constexpr int P = T + 2 + (T + 2) / 16 + 1;
    __shared__ K sk[P];
    __shared__ uint8_t sf[P];
    for (int j = threadIdx.x; j < T + 2; j += NT) {
      const int64_t e = tile_e0 - 1 + j;
      K k = 0;
      uint8_t f = 0x80;
      if (e >= 0 && e < M) {
        k = ld.keys[seg_base + e];
        f = ld.flags[seg_base + e];
      }
      sk[j + (j >> 4)] = k;
      sf[j + (j >> 4)] = f;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT + 2; ++j) {
      const int l = threadIdx.x * IT + j;
      el[j] = ld.make(sk[l + (l >> 4)], sf[l + (l >> 4)]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < IT + 2; ++j) {
      const int64_t e = e0 - 1 + j;
      if (e >= 0 && e < M) {
        el[j] = ld.load(seg_base + e);
      } else {
        el[j].valid = false;
        el[j].rk = 0;
        el[j].pw = el[j].nw = 0;
      }
    }
  }
}

template <int IT, typename C>
__device__ __forceinline__ RunRec<C> item_rec(const Elem<C> (&el)[IT + 2], int j, int64_t e) {
  const Elem<C>& x = el[j + 1];
  const bool start = x.valid && (e == 0 || !el[j].valid || el[j].rk != x.rk);
  RunRec<C> r;
  r.p = x.pw;
  r.n = x.nw;
  r.sp = C(0);
  r.sn = C(0);
  r.starts = start ? 1 : 0;
  r.has = start ? 1 : 0;
  return r;
}

template <int NT, int IT, class L>
__global__ __launch_bounds__(NT) void run_tile_aggregate_kernel(L ld, int64_t M, int tiles,
                                                                RunRec<typename L::count_t>* __restrict__ agg) {
  using C = typename L::count_t;
  __shared__ RunRec<C> lds[NT / kWave];
  const int64_t s = blockIdx.x / tiles;
  const int t = static_cast<int>(blockIdx.x - s * tiles);
  const int64_t e0 = static_cast<int64_t>(t) * NT * IT + static_cast<int64_t>(threadIdx.x) * IT;
  Elem<C> el[IT + 2];
  load_tile<NT, IT>(ld, s * M, M, static_cast<int64_t>(t) * NT * IT, el);
  RunOp op;
  RunRec<C> acc = run_identity<C>();
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int64_t e = e0 + j;
    if (e < M) acc = op(acc, item_rec<IT>(el, j, e));
  }
  RunRec<C> excl, total;
  sortscan::block_inclusive_scan<NT / kWave>(acc, op, run_identity<C>(), lds, excl, total);
  if (threadIdx.x == 0) agg[s * tiles + t] = total;
}

// Per segment: exclusive prefix of the tile aggregates (written over agg) and the segment total.  Each thread scans
// TPT consecutive tiles sequentially, so one block scan covers NT * TPT tiles (4096 at 256 x 16).
template <int NT, int TPT, typename C>
__global__ __launch_bounds__(NT) void run_tile_scan_kernel(RunRec<C>* __restrict__ agg, int tiles,
                                                           RunRec<C>* __restrict__ seg_total) {
  __shared__ RunRec<C> lds[NT / kWave];
  const int64_t s = blockIdx.x;
  RunOp op;
  RunRec<C> carry = run_identity<C>();
  for (int base = 0; base < tiles; base += NT * TPT) {
    const int t0 = base + threadIdx.x * TPT;
    RunRec<C> acc = run_identity<C>();
    for (int j = 0; j < TPT; ++j)
      if (t0 + j < tiles) acc = op(acc, agg[s * tiles + t0 + j]);
    RunRec<C> excl, total;
    sortscan::block_inclusive_scan<NT / kWave>(acc, op, run_identity<C>(), lds, excl, total);
    RunRec<C> run = op(carry, excl);
    for (int j = 0; j < TPT; ++j) {
      if (t0 + j >= tiles) break;
      const RunRec<C> v = agg[s * tiles + t0 + j];
      agg[s * tiles + t0 + j] = run;
      run = op(run, v);
    }
    carry = op(carry, total);
  }
  if (threadIdx.x == 0) seg_total[s] = carry;
}

constexpr int kEmitCurve = 1;
constexpr int kEmitRanks = 2;

template <int NT, int IT, class L>
__global__ __launch_bounds__(NT) void run_tile_epilogue_kernel(L ld, int64_t M, int tiles,
                                                               const RunRec<typename L::count_t>* __restrict__ prefix,
                                                               Partial* __restrict__ part, int emit,
                                                               double* __restrict__ c_fps, double* __restrict__ c_tps,
                                                               double* __restrict__ c_thr, int32_t* __restrict__ run_of,
                                                               int32_t* __restrict__ run_end) {
  using C = typename L::count_t;
  __shared__ RunRec<C> lds[NT / kWave];
  __shared__ double red[4][NT / kWave];
  const int64_t s = blockIdx.x / tiles;
  const int t = static_cast<int>(blockIdx.x - s * tiles);
  const int64_t e0 = static_cast<int64_t>(t) * NT * IT + static_cast<int64_t>(threadIdx.x) * IT;
  Elem<C> el[IT + 2];
  load_tile<NT, IT>(ld, s * M, M, static_cast<int64_t>(t) * NT * IT, el);
  RunOp op;
  RunRec<C> acc = run_identity<C>();
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int64_t e = e0 + j;
    if (e < M) acc = op(acc, item_rec<IT>(el, j, e));
  }
  RunRec<C> excl, total;
  sortscan::block_inclusive_scan<NT / kWave>(acc, op, run_identity<C>(), lds, excl, total);
  RunRec<C> run = op(prefix[s * tiles + t], excl);
  double area = 0.0, ap = 0.0, cov = 0.0;
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int64_t e = e0 + j;
    if (e >= M) break;
    run = op(run, item_rec<IT>(el, j, e));
    const Elem<C>& x = el[j + 1];
    const Elem<C>& nx = el[j + 2];
    if (!x.valid) continue;
    const int rid = run.starts - 1;
    if (emit & kEmitRanks) run_of[s * M + e] = rid;
    const bool end = (e == M - 1) || !nx.valid || nx.rk != x.rk;
    if (!end) continue;
    const double P = static_cast<double>(run.p), N = static_cast<double>(run.n);
    const double pos_r = static_cast<double>(run.p - run.sp), neg_r = static_cast<double>(run.n - run.sn);
    area += neg_r * (static_cast<double>(run.sp) + 0.5 * pos_r);
    if (P + N > 0.0) ap += pos_r * (P / (P + N));
    if (pos_r > 0.0) cov = fmax(cov, P + N);
    if (emit & kEmitCurve) {
      c_fps[s * M + rid] = N;
      c_tps[s * M + rid] = P;
      c_thr[s * M + rid] = ld.threshold(s * M + e);
    }
    if (emit & kEmitRanks) run_end[s * M + rid] = static_cast<int32_t>(e);
  }
  // deterministic block reduction (fixed tree), one partial per tile
  double v0 = wave_sum(area), v1 = wave_sum(ap), v2 = cov;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v2 = fmax(v2, __shfl_xor(v2, off, kWave));
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) {
    red[0][wave] = v0;
    red[1][wave] = v1;
    red[2][wave] = v2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Partial pt{0.0, 0.0, 0.0, 0.0};
    for (int w = 0; w < NT / kWave; ++w) {
      pt.area += red[0][w];
      pt.ap += red[1][w];
      pt.cov = fmax(pt.cov, red[2][w]);
    }
    part[s * tiles + t] = pt;
  }
}

// stats[s] = {P, N, area, ap, coverage, 0, nruns, 0}
template <typename C>
__global__ __launch_bounds__(256) void run_finalize_kernel(const Partial* __restrict__ part,
                                                           const RunRec<C>* __restrict__ seg_total,
                                                           int tiles, double* __restrict__ stats) {
  __shared__ double red[3][256 / kWave];
  const int64_t s = blockIdx.x;
  double a = 0.0, b = 0.0, c = 0.0;
  for (int t = threadIdx.x; t < tiles; t += blockDim.x) {
    const Partial p = part[s * tiles + t];
    a += p.area;
    b += p.ap;
    c = fmax(c, p.cov);
  }
  a = wave_sum(a);
  b = wave_sum(b);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c = fmax(c, __shfl_xor(c, off, kWave));
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) {
    red[0][wave] = a;
    red[1][wave] = b;
    red[2][wave] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double A = 0.0, B = 0.0, Cv = 0.0;
    for (int w = 0; w < 256 / kWave; ++w) {
      A += red[0][w];
      B += red[1][w];
      Cv = fmax(Cv, red[2][w]);
    }
    const RunRec<C> tot = seg_total[s];
    double* o = stats + s * kStatCols;
    o[0] = static_cast<double>(tot.p);
    o[1] = static_cast<double>(tot.n);
    o[2] = A;
    o[3] = B;
    o[4] = Cv;
    o[5] = 0.0;
    o[6] = static_cast<double>(tot.starts);
    o[7] = 0.0;
  }
}

// average 1-based rank of every element, scattered back to its original flat id (payload path only)
template <class L>
__global__ void avg_rank_scatter_kernel(L ld, int64_t total, sortscan::FastDiv divM, int64_t M,
                                        const int32_t* __restrict__ run_of, const int32_t* __restrict__ run_end,
                                        double* __restrict__ ranks) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = divM.div(static_cast<uint32_t>(i));
    const int r = run_of[i];
    const double hi = run_end[s * M + r];
    const double lo = r == 0 ? 0.0 : run_end[s * M + r - 1] + 1.0;
    ranks[ld.origin(i)] = 0.5 * (lo + hi) + 1.0;
  }
}

template <int NT, int IT, class L>
void run_engine(const L& ld, int64_t S, int64_t M, int emit, const at::Tensor& stats, double* fps, double* tps,
                double* thr, int32_t* run_of, int32_t* run_end, const at::Device& dev, hipStream_t st) {
  constexpr int64_t kTile = static_cast<int64_t>(NT) * IT;
  const int tiles = static_cast<int>((M + kTile - 1) / kTile);
  auto opts = at::TensorOptions().dtype(at::kByte).device(dev);
  using C = typename L::count_t;
  using RR = RunRec<C>;
  auto agg_t = at::empty({S * tiles * static_cast<int64_t>(sizeof(RR))}, opts);
  auto tot_t = at::empty({S * static_cast<int64_t>(sizeof(RR))}, opts);
  auto part_t = at::empty({S * tiles * static_cast<int64_t>(sizeof(Partial))}, opts);
  auto* agg = reinterpret_cast<RR*>(agg_t.data_ptr());
  auto* tot = reinterpret_cast<RR*>(tot_t.data_ptr());
  auto* part = reinterpret_cast<Partial*>(part_t.data_ptr());
  TORCH_CHECK(S * tiles < (1LL << 31), "clf_curve: too many segments / tiles");
  const dim3 grid(static_cast<unsigned>(S * tiles));  // block b -> (segment b / tiles, tile b % tiles)
  hipLaunchKernelGGL((run_tile_aggregate_kernel<NT, IT, L>), grid, dim3(NT), 0, st, ld, M, tiles, agg);
  if (tiles > 256)
    hipLaunchKernelGGL((run_tile_scan_kernel<256, 16, C>), dim3(S), dim3(256), 0, st, agg, tiles, tot);
  else
    hipLaunchKernelGGL((run_tile_scan_kernel<64, 4, C>), dim3(S), dim3(64), 0, st, agg, tiles, tot);
  hipLaunchKernelGGL((run_tile_epilogue_kernel<NT, IT, L>), grid, dim3(NT), 0, st, ld, M, tiles, agg, part, emit, fps,
                     tps, thr, run_of, run_end);
  hipLaunchKernelGGL(run_finalize_kernel<C>, dim3(S), dim3(256), 0, st, part, tot, tiles, stats.data_ptr<double>());
}

template <class L>
void run_engine_auto(const L& ld, int64_t S, int64_t M, int emit, const at::Tensor& stats, double* fps, double* tps,
                     double* thr, int32_t* run_of, int32_t* run_end, const at::Device& dev, hipStream_t st) {
  if (M <= 1024)
    run_engine<64, 16>(ld, S, M, emit, stats, fps, tps, thr, run_of, run_end, dev, st);
  else
    run_engine<256, 16>(ld, S, M, emit, stats, fps, tps, thr, run_of, run_end, dev, st);
}

}  // namespace

// scores: addressed as scores[s * seg_stride + e * elem_stride] for segment s < S, element e < M.
// target: [M] (tmode 0/1) or addressed like scores (tmode 2).  weights: optional fp64 [M].
// emit: bit0 -> compacted curve (fps, tps, thr) per segment at [s * M + run]; bit1 -> average ranks (payload path).
// Returns stats [S, 8] fp64 and, when requested, fps/tps/thr [S, M] fp64 and ranks [S * M] (flat id order).
std::vector<at::Tensor> clf_curve(const at::Tensor& scores, const at::Tensor& target, const c10::optional<at::Tensor>& weights,
                                  int64_t S, int64_t M, int64_t seg_stride, int64_t elem_stride, int64_t tmode,
                                  int64_t pos_label, int64_t ignore_index, bool has_ignore, int64_t emit) {
  TM_CHECK_CUDA(scores);
  TM_SAME_DEVICE(scores, target);
  TORCH_CHECK(S >= 1 && M >= 1, "clf_curve: empty input");
  TORCH_CHECK(S * M < (1LL << 31), "clf_curve: at most 2^31 elements");
  const auto dev = scores.device();
  auto st = stream();
  auto f64 = at::TensorOptions().dtype(at::kDouble).device(dev);
  auto stats = at::empty({S, kStatCols}, f64);
  at::Tensor fps, tps, thr, ranks;
  const bool want_curve = emit & kEmitCurve, want_ranks = emit & kEmitRanks;
  if (want_curve) {
    fps = at::empty({S, M}, f64);
    tps = at::empty({S, M}, f64);
    thr = at::empty({S, M}, f64);
  }
  at::Tensor run_of_t, run_end_t;
  if (want_ranks) {
    ranks = at::empty({S * M}, f64);
    run_of_t = at::empty({S * M}, at::TensorOptions().dtype(at::kInt).device(dev));
    run_end_t = at::empty({S * M}, at::TensorOptions().dtype(at::kInt).device(dev));
  }
  double* fp = want_curve ? fps.data_ptr<double>() : nullptr;
  double* tp = want_curve ? tps.data_ptr<double>() : nullptr;
  double* th = want_curve ? thr.data_ptr<double>() : nullptr;
  int32_t* ro = want_ranks ? run_of_t.data_ptr<int32_t>() : nullptr;
  int32_t* re = want_ranks ? run_end_t.data_ptr<int32_t>() : nullptr;
  const int64_t n = S * M;
  const int grid = grid_cap((n + 255) / 256);
  const bool payload = weights.has_value() || scores.scalar_type() == at::kDouble || want_ranks;
  if (weights.has_value()) {
    TM_SAME_DEVICE(scores, (*weights));
    TORCH_CHECK(weights->scalar_type() == at::kDouble && weights->is_contiguous() && weights->numel() == M &&
                    tmode != kTgtElementwise, "clf_curve: weights must be contiguous fp64 [M] (binary / one-vs-rest)");
  }
  const bool columns = seg_stride == 1 && elem_stride == S;
  const bool rows = elem_stride == 1 && seg_stride == M;
  TORCH_CHECK(columns || rows || (S == 1 && elem_stride == 1) || M == 1,
              "clf_curve: scores must be contiguous column or row segments");
  TORCH_CHECK(tmode != kTgtElementwise || target.strides() == scores.strides(),
              "clf_curve: elementwise targets must share the scores' layout");
  TORCH_CHECK(tmode == kTgtElementwise || target.is_contiguous(), "clf_curve: target must be contiguous");
  const Layout lay{sortscan::FastDiv(static_cast<uint32_t>(columns && S > 1 ? S : M)), columns && S > 1};
  const sortscan::FastDiv divM(static_cast<uint32_t>(M));
  auto i64 = at::TensorOptions().dtype(at::kLong).device(dev);
  auto i32 = at::TensorOptions().dtype(at::kInt).device(dev);
  TM_DISPATCH_TARGET(target.scalar_type(), "clf_curve", [&] {
    const target_t* tg = reinterpret_cast<const target_t*>(target.data_ptr());
    TM_DISPATCH_FLOAT(scores.scalar_type(), "clf_curve", [&] {
      const scalar_t* sc = reinterpret_cast<const scalar_t*>(scores.data_ptr());
      auto k1 = at::empty({n}, i64), k2 = at::empty({n}, i64);
      auto* a = reinterpret_cast<uint64_t*>(k1.data_ptr());
      auto* b = reinterpret_cast<uint64_t*>(k2.data_ptr());
      if (!payload) {
        TORCH_CHECK(S < (1LL << 31), "clf_curve: too many segments for packed keys");
        auto f1 = at::empty({n}, at::TensorOptions().dtype(at::kByte).device(dev));
        auto f2 = at::empty({n}, at::TensorOptions().dtype(at::kByte).device(dev));
        auto* fa = f1.data_ptr<uint8_t>();
        auto* fb = f2.data_ptr<uint8_t>();
        if (S == 1) {
          auto* a32 = reinterpret_cast<uint32_t*>(a);
          auto* b32 = reinterpret_cast<uint32_t*>(b);
          hipLaunchKernelGGL((build_kv8_kernel<scalar_t, target_t, uint32_t>), dim3(grid), dim3(256), 0, st, sc, tg,
                             n, lay, static_cast<int>(tmode), pos_label, ignore_index, has_ignore, a32, fa);
          sortscan::sort_pairs<uint32_t, uint8_t>(a32, b32, fa, fb, n, 0, 32, dev, st);
          run_engine_auto(KV8Loader<uint32_t>{b32, fb}, S, M, static_cast<int>(emit), stats, fp, tp, th, ro, re, dev,
                          st);
        } else {
          hipLaunchKernelGGL((build_kv8_kernel<scalar_t, target_t, uint64_t>), dim3(grid), dim3(256), 0, st, sc, tg,
                             n, lay, static_cast<int>(tmode), pos_label, ignore_index, has_ignore, a, fa);
          sortscan::sort_pairs<uint64_t, uint8_t>(a, b, fa, fb, n, 0, 32 + sortscan::ceil_log2(S), dev, st);
          run_engine_auto(KV8Loader<uint64_t>{b, fb}, S, M, static_cast<int>(emit), stats, fp, tp, th, ro, re, dev,
                          st);
        }
        return;
      }
      auto v1 = at::empty({n}, i32), v2 = at::empty({n}, i32);
      auto* va = v1.data_ptr<int32_t>();
      auto* vb = v2.data_ptr<int32_t>();
      const double* wp = weights.has_value() ? weights->data_ptr<double>() : nullptr;
      auto finish = [&](auto ld) {
        run_engine_auto(ld, S, M, static_cast<int>(emit), stats, fp, tp, th, ro, re, dev, st);
        if (want_ranks)
          hipLaunchKernelGGL((avg_rank_scatter_kernel<decltype(ld)>), dim3(grid), dim3(256), 0, st, ld, n, divM, M,
                             ro, re, ranks.data_ptr<double>());
      };
      if constexpr (!std::is_same<scalar_t, double>::value) {
        if (S == 1 && !has_ignore && !want_curve && !wp) {
          // ranks of one column: 32-bit desc-score keys carrying the element id (4 radix passes)
          auto* a32 = reinterpret_cast<uint32_t*>(a);
          auto* b32 = reinterpret_cast<uint32_t*>(b);
          hipLaunchKernelGGL((build_score_keys32_kernel<scalar_t>), dim3(grid), dim3(256), 0, st, sc, n, a32, va);
          sortscan::sort_pairs<uint32_t, int32_t>(a32, b32, va, vb, n, 0, 32, dev, st);
          if (want_ranks)
            finish(PayloadLoader<scalar_t, target_t, true, false, uint32_t>{b32, vb, sc, tg, wp, divM, M, seg_stride,
                                                                            elem_stride, static_cast<int>(tmode),
                                                                            pos_label, ignore_index, has_ignore});
          else
            finish(PayloadLoader<scalar_t, target_t, true, true, uint32_t>{b32, vb, sc, tg, wp, divM, M, seg_stride,
                                                                           elem_stride, static_cast<int>(tmode),
                                                                           pos_label, ignore_index, has_ignore});
          return;
        }
        // one sort: [segment | invalid | desc-score32] keys carrying the flat id
        TORCH_CHECK(S < (1LL << 30), "clf_curve: too many segments");
        hipLaunchKernelGGL((build_packed_keys_kernel<scalar_t, target_t>), dim3(grid), dim3(256), 0, st, sc, tg, n,
                           lay, static_cast<int>(tmode), pos_label, ignore_index, has_ignore, a, va, M);
        sortscan::sort_pairs<uint64_t, int32_t>(a, b, va, vb, n, 0, 33 + sortscan::ceil_log2(S), dev, st);
        if (want_curve || !want_ranks || wp) {
          finish(PayloadLoader<scalar_t, target_t, true, true>{b, vb, sc, tg, wp, divM, M, seg_stride, elem_stride,
                                                                static_cast<int>(tmode), pos_label, ignore_index,
                                                                has_ignore});
        } else {
          finish(PayloadLoader<scalar_t, target_t, true, false>{b, vb, sc, tg, wp, divM, M, seg_stride, elem_stride,
                                                                 static_cast<int>(tmode), pos_label, ignore_index,
                                                                 has_ignore});
        }
      } else {
        hipLaunchKernelGGL((build_score_keys_kernel<scalar_t>), dim3(grid), dim3(256), 0, st, sc, n, lay, M, a, va);
        sortscan::sort_pairs<uint64_t, int32_t>(a, b, va, vb, n, 0, 64, dev, st);
        const int32_t* sorted_vals = vb;
        if (S > 1 || has_ignore) {
          auto* k32a = reinterpret_cast<uint32_t*>(a);  // reuse k1 as two 32-bit key arrays
          auto* k32b = reinterpret_cast<uint32_t*>(a) + n;
          hipLaunchKernelGGL((build_segment_keys_kernel<target_t>), dim3(grid), dim3(256), 0, st, vb, tg, n, divM, M,
                             seg_stride, elem_stride, static_cast<int>(tmode), ignore_index, has_ignore, k32a);
          sortscan::sort_pairs<uint32_t, int32_t>(k32a, k32b, vb, va, n, 0, 1 + sortscan::ceil_log2(S), dev, st);
          sorted_vals = va;
        }
        finish(PayloadLoader<scalar_t, target_t, false, true>{nullptr, sorted_vals, sc, tg, wp, divM, M, seg_stride,
                                                              elem_stride, static_cast<int>(tmode), pos_label,
                                                              ignore_index, has_ignore});
      }
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {stats, fps, tps, thr, ranks};
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "clf_curve(Tensor scores, Tensor target, Tensor? weights, int S, int M, int seg_stride, int elem_stride, "
      "int tmode, int pos_label, int ignore_index, bool has_ignore, int emit) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("clf_curve", &tm_amd::clf_curve); }
