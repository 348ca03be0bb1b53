// Exact match (subset accuracy) update in two launches (K10 in SURVEY.md §2.5).
//
// Reference (F/classification/exact_match.py:32-128): multiclass -- argmax over dim 1 (a [N, P] label copy), a
// masked fill for ignore_index, `preds == target` ([N, P] bool), `.sum(1) == P`, `.sum()`; multilabel -- a host sync
// to decide whether the scores are probabilities (`_prob_or`), a sigmoid copy, a threshold copy, two masked fills,
// `movedim(1, -1).reshape(-1, L)` (a transposed copy for multi-dim inputs), `== target`, `.sum(1) == L`, `.sum()`.
// Here one pass decides each unit directly from the scores:
//   * multiclass, P == 1: G = 8..64 lanes per sample over the C scores (group argmax, torch.argmax tie / NaN rules;
//     small C packs several samples into a wave);
//   * multiclass, P > 1: one wave per sample, lanes over the P positions (coalesced over the [N, C, P] layout), each
//     lane a sequential argmax over C; a wave vote ANDs the positions;
//   * multilabel: one thread per (sample, position) unit looping over the L labels, judging BOTH readings of float
//     scores (as given / sigmoid in the scores' dtype) and OR-ing a "not a probability" word; the fold keeps the
//     reading the batch calls for (the reference's global `_prob_or` decision) without a host round trip.
// Counts are reduced per block and added with one int64 atomic per block (order independent, deterministic; a
// per-wave atomic on one address serialised the first version at ~70 us per 65536-row batch).  The fold adds the global count and total into the
// metric states in place, or writes the per-sample counts (samplewise), and re-zeroes the workspace.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;

// one int64 atomic per block for a per-thread count pair (every thread of the block must call it)
__device__ __forceinline__ void block_add_counts(long long a, long long b, int64_t* __restrict__ dst_a,
                                                 int64_t* __restrict__ dst_b) {
  __shared__ long long red[2][kBlock / kWave];
  a = wave_sum_ll(a);
  b = wave_sum_ll(b);
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    red[0][w] = a;
    red[1][w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long sa = 0, sb = 0;
    for (int k = 0; k < kBlock / kWave; ++k) {
      sa += red[0][k];
      sb += red[1][k];
    }
    if (sa) atomic_add_i64(dst_a, sa);
    if (sb && dst_b) atomic_add_i64(dst_b, sb);
  }
}

// multiclass, P == 1: preds [N, C] scores, G lanes per row (G = 8 / 16 / 32 / 64 from C: small C packs several rows
// into a wave), 4 loads in flight per lane; ws: i64 [1] (global) or [N] (samplewise)
template <typename scalar_t, typename target_t, int G>
__global__ void __launch_bounds__(kBlock) em_multiclass_row_kernel(const scalar_t* __restrict__ preds,
                                                                   const target_t* __restrict__ target, long long N,
                                                                   int C, long long ignore, bool has_ignore,
                                                                   bool samplewise, int64_t* __restrict__ ws) {
  constexpr int kRows = kBlock / G;
  const int sub = threadIdx.x % G;
  long long local = 0;
  for (long long base = static_cast<long long>(blockIdx.x) * kRows; base < N;
       base += static_cast<long long>(gridDim.x) * kRows) {
    const long long n = base + threadIdx.x / G;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    if (n < N) {
      const scalar_t* r = preds + n * C;
      int c = sub;
      for (; c + 3 * G < C; c += 4 * G) {
        const float v0 = to_f32(r[c]), v1 = to_f32(r[c + G]), v2 = to_f32(r[c + 2 * G]), v3 = to_f32(r[c + 3 * G]);
        if (argmax_better(v0, c, bv, bi)) bv = v0, bi = c;
        if (argmax_better(v1, c + G, bv, bi)) bv = v1, bi = c + G;
        if (argmax_better(v2, c + 2 * G, bv, bi)) bv = v2, bi = c + 2 * G;
        if (argmax_better(v3, c + 3 * G, bv, bi)) bv = v3, bi = c + 3 * G;
      }
      for (; c < C; c += G) {
        const float v = to_f32(r[c]);
        if (argmax_better(v, c, bv, bi)) bv = v, bi = c;
      }
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) {
      const float ov = __shfl_xor(bv, off, kWave);
      const int oi = __shfl_xor(bi, off, kWave);
      if (argmax_better(ov, oi, bv, bi)) bv = ov, bi = oi;
    }
    if (n < N && sub == 0) {
      const long long t = static_cast<long long>(target[n]);
      const bool ok = (has_ignore && t == ignore) || static_cast<long long>(bi) == t;
      if (samplewise)
        ws[n] = ok ? 1 : 0;
      else
        local += ok ? 1 : 0;
    }
  }
  if (!samplewise) block_add_counts(local, 0, ws, nullptr);
}

// multiclass, P == 1, large C with 16-byte aligned rows (C % (16 / sizeof) == 0): one wave per row, 16-byte vector
// loads (8 bf16 / f16 or 4 f32 per lane), up to 4 of them in flight per lane before any compare -- the element-wise
// version issued 2-byte loads and ran at ~1 TB/s
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) em_multiclass_vec_kernel(const scalar_t* __restrict__ preds,
                                                                   const target_t* __restrict__ target, long long N,
                                                                   int C, long long ignore, bool has_ignore,
                                                                   bool samplewise, int64_t* __restrict__ ws) {
  constexpr int kVec = 16 / sizeof(scalar_t);
  const int lane = threadIdx.x & (kWave - 1);
  const int nvec = C / kVec;
  const long long nw = static_cast<long long>(gridDim.x) * (kBlock / kWave);
  long long local = 0;
  auto judge = [&](long long n, float bv, int bi) {
    wave_argmax(bv, bi);
    if (lane == 0) {
      const long long t = static_cast<long long>(target[n]);
      const bool ok = (has_ignore && t == ignore) || static_cast<long long>(bi) == t;
      if (samplewise)
        ws[n] = ok ? 1 : 0;
      else
        local += ok ? 1 : 0;
    }
  };
  auto scan = [&](const u32x4* buf, int v0, float& bv, int& bi) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int v = v0 + k * kWave;
      if (v >= nvec) break;
      const scalar_t* e = reinterpret_cast<const scalar_t*>(&buf[k]);
#pragma unroll
      for (int j = 0; j < kVec; ++j) {
        const float x = to_f32(e[j]);
        const int c = v * kVec + j;
        if (argmax_better(x, c, bv, bi)) bv = x, bi = c;
      }
    }
  };
  auto load = [&](long long n, int v0, u32x4* buf) {
    const u32x4* r = reinterpret_cast<const u32x4*>(preds + n * C);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int v = v0 + k * kWave;
      if (v < nvec) buf[k] = __builtin_nontemporal_load(r + v);
    }
  };
  long long n = (static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  if (nvec <= 4 * kWave) {
    // a whole row fits one 4-vector-per-lane chunk: software-pipelined, the next row's loads are in flight while
    // this row is scanned
    u32x4 cur[4], nxt[4];
    if (n < N) load(n, lane, cur);
    for (; n < N; n += nw) {
      if (n + nw < N) load(n + nw, lane, nxt);
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      scan(cur, lane, bv, bi);
      judge(n, bv, bi);
#pragma unroll
      for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
    }
  } else {
    for (; n < N; n += nw) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int v0 = lane; v0 < nvec; v0 += 4 * kWave) {
        u32x4 buf[4];
        load(n, v0, buf);
        scan(buf, v0, bv, bi);
      }
      judge(n, bv, bi);
    }
  }
  if (!samplewise) block_add_counts(local, 0, ws, nullptr);
}

// multiclass, P > 1: preds [N, C, P] scores; target [N, P]
template <typename scalar_t, typename target_t>
__global__ void __launch_bounds__(kBlock) em_multiclass_pos_kernel(const scalar_t* __restrict__ preds,
                                                                   const target_t* __restrict__ target, long long N,
                                                                   int C, long long P, long long ignore,
                                                                   bool has_ignore, bool samplewise,
                                                                   int64_t* __restrict__ ws) {
  const int lane = threadIdx.x & (kWave - 1);
  const long long nw = static_cast<long long>(gridDim.x) * (kBlock / kWave);
  long long local = 0;
  for (long long n = (static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x) / kWave; n < N; n += nw) {
    int bad = 0;
    for (long long p = lane; p < P; p += kWave) {
      const long long t = static_cast<long long>(target[n * P + p]);
      if (has_ignore && t == ignore) continue;
      const scalar_t* r = preds + n * C * P + p;
      float bv = to_f32(r[0]);
      int bi = 0;
      for (int c = 1; c < C; ++c) {
        const float v = to_f32(r[static_cast<long long>(c) * P]);
        if (argmax_better(v, c, bv, bi)) {
          bv = v;
          bi = c;
        }
      }
      const long long label = bi;
      bad |= label != t;
    }
    const bool ok = !__any(bad);
    if (lane == 0) {
      if (samplewise)
        ws[n] = ok ? 1 : 0;
      else
        local += ok ? 1 : 0;
    }
  }
  if (!samplewise) block_add_counts(local, 0, ws, nullptr);
}

// multilabel: preds / target [N, L, P]; unit u = (n, p); ws: i64 [2] (global: reading A, B) or [2N] (samplewise:
// per-sample counts of correct positions, A then B); notprob: i32 [1]
//
// kLabels (kind 2, multiclass labels [N, L] with P = 1): an ignored position counts as a match (the reference writes
// ignore_index into preds there), float labels compare exactly in the scores' dtype (`preds == target` promotes the
// integer target to it), and there is one reading.
template <typename scalar_t, typename target_t, bool kLabels>
__global__ void __launch_bounds__(kBlock) em_multilabel_kernel(const scalar_t* __restrict__ preds,
                                                               const target_t* __restrict__ target, long long N,
                                                               int L, long long P, float thr, long long ignore,
                                                               bool has_ignore, bool samplewise,
                                                               int64_t* __restrict__ ws, int* __restrict__ notprob) {
  const long long U = N * P;
  long long ca = 0, cb = 0;
  int np = 0;
  for (long long u = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; u < U;
       u += static_cast<long long>(gridDim.x) * kBlock) {
    const long long n = u / P, p = u - n * P;
    const scalar_t* pr = preds + n * L * P + p;
    const target_t* tr = target + n * L * P + p;
    bool oka = true, okb = true;
    for (int l = 0; l < L; ++l) {
      const long long t = static_cast<long long>(tr[static_cast<long long>(l) * P]);
      const scalar_t v = pr[static_cast<long long>(l) * P];
      if constexpr (kLabels) {
        if (has_ignore && t == ignore) continue;
        bool eq;
        if constexpr (std::is_same<scalar_t, double>::value)
          eq = v == static_cast<double>(t);
        else if constexpr (IsFloating<scalar_t>::value)
          eq = to_f32(v) == to_f32(scalar_t(static_cast<float>(t)));
        else
          eq = static_cast<long long>(v) == t;
        oka &= eq;
        okb &= eq;
      } else if constexpr (IsFloating<scalar_t>::value) {
        const float x = to_f32(v);
        np |= !(x >= 0.f && x <= 1.f);  // the reference decides over every score, ignored positions included
        // reference semantics (_multilabel_stat_scores_format): an ignored target becomes -1 while the prediction
        // stays 0/1, so an ignored position never matches and its sample is never an exact match
        if (has_ignore && t == ignore) {
          oka = okb = false;
          continue;
        }
        const float s = round_to<scalar_t>(1.f / (1.f + expf(-x)));
        oka &= static_cast<long long>(x > thr) == t;
        okb &= static_cast<long long>(s > thr) == t;
      } else {
        if (has_ignore && t == ignore) {
          oka = okb = false;
          continue;
        }
        const bool eq = static_cast<long long>(v) == t;
        oka &= eq;
        okb &= eq;
      }
    }
    if (samplewise) {
      if (oka) atomic_add_i64(ws + n, 1);
      if (!kLabels && okb) atomic_add_i64(ws + N + n, 1);
    } else {
      ca += oka;
      cb += okb;
    }
  }
  if (!kLabels && __any(np) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(notprob, 1);
  if (!samplewise) block_add_counts(ca, cb, ws, ws + 1);
}

// global: correct += (notprob ? ws[1] : ws[0]); total += total_add.  samplewise: out[n] = ws[(notprob ? N : 0) + n].
// Re-zeroes ws (two_readings: 2 slots / 2N) and notprob.
__global__ void em_fold_kernel(int64_t* __restrict__ ws, long long N, bool samplewise, bool two_readings,
                               int* __restrict__ notprob, int64_t* __restrict__ correct, int64_t* __restrict__ total,
                               long long total_add, int64_t* __restrict__ out) {
  const bool use_b = two_readings && *notprob != 0;
  if (samplewise) {
    for (long long n = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; n < N;
         n += static_cast<long long>(gridDim.x) * blockDim.x) {
      out[n] = use_b ? ws[N + n] : ws[n];
      ws[n] = 0;
      if (two_readings) ws[N + n] = 0;
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *correct += use_b ? ws[1] : ws[0];
    *total += total_add;
    ws[0] = 0;
    ws[1] = 0;
    *notprob = 0;
  }
}

__global__ void em_reset_notprob_kernel(int* notprob) { *notprob = 0; }

}  // namespace

// kind 0 multiclass (preds [N, C, P] scores, has_c; target [N, P]); kind 1 multilabel (preds / target [N, L, P];
// C = L); kind 2 multiclass labels of any dtype (preds / target [N, L], C = L positions, P = 1).  ws: i64 zeroed, [max(2, 2N)]; notprob: i32 [1] zero.  Global: correct / total
// i64 [1] states updated in place (total += N for multiclass, N * P for multilabel).  Samplewise: out i64 [N] receives
// the per-sample counts (0/1 multiclass, correct positions multilabel).
void exact_match_update(const at::Tensor& preds, const at::Tensor& target, int64_t kind, int64_t C, int64_t P,
                        bool has_c, double threshold, int64_t ignore_index, bool has_ignore, bool samplewise,
                        at::Tensor ws, at::Tensor notprob, at::Tensor correct, at::Tensor total, at::Tensor out) {
  TM_CHECK_CUDA(preds);
  for (const at::Tensor* t :
       std::initializer_list<const at::Tensor*>{&target, &ws, &notprob, &correct, &total, &out})
    TM_SAME_DEVICE(preds, (*t));
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(kind == 0 || kind == 1 || kind == 2, "exact_match_update: bad kind");
  TORCH_CHECK((kind == 0) == has_c, "exact_match_update: only multiclass scores (kind 0) carry a class dimension");
  TORCH_CHECK(kind != 2 || P == 1, "exact_match_update: multiclass labels are one unit per sample (P = 1)");
  TORCH_CHECK(C >= 1 && P >= 1, "exact_match_update: C and P must be positive");
  const long long N = P > 0 ? target.numel() / (kind == 0 ? P : C * P) : 0;
  TORCH_CHECK(target.numel() == N * (kind == 0 ? P : C * P), "exact_match_update: target shape");
  TORCH_CHECK(preds.numel() == N * C * P, "exact_match_update: preds shape");
  TORCH_CHECK(ws.scalar_type() == at::kLong && ws.is_contiguous() && ws.numel() >= std::max<long long>(2, 2 * N),
              "exact_match_update: ws");
  TORCH_CHECK(notprob.scalar_type() == at::kInt && notprob.numel() == 1, "exact_match_update: notprob");
  TORCH_CHECK(correct.scalar_type() == at::kLong && correct.numel() == 1 && total.scalar_type() == at::kLong &&
                  total.numel() == 1, "exact_match_update: states");
  TORCH_CHECK(!samplewise || (out.scalar_type() == at::kLong && out.numel() == N && out.is_contiguous()),
              "exact_match_update: out");
  auto s = stream();
  int64_t* w = ws.data_ptr<int64_t>();
  if (N > 0) {
    TM_DISPATCH_TARGET(target.scalar_type(), "exact_match_update", [&] {
      TM_DISPATCH_PREDS(preds.scalar_type(), "exact_match_update", [&] {
        const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
        const target_t* t = reinterpret_cast<const target_t*>(target.data_ptr());
        const long long ig = static_cast<long long>(ignore_index);
        float thr = static_cast<float>(threshold);  // the threshold as ATen compares it against 16-bit scores
        if constexpr (std::is_same<scalar_t, c10::BFloat16>::value) thr = static_cast<float>(c10::BFloat16(thr));
        if constexpr (std::is_same<scalar_t, c10::Half>::value) thr = static_cast<float>(c10::Half(thr));
        constexpr int kVec = 16 / sizeof(scalar_t);
        const bool vec_ok = IsFloating<scalar_t>::value && C >= 64 * kVec && C % kVec == 0 &&
                            reinterpret_cast<uintptr_t>(preds.data_ptr()) % 16 == 0;
        if (kind == 0 && P == 1 && vec_ok) {
          hipLaunchKernelGGL((em_multiclass_vec_kernel<scalar_t, target_t>),
                             dim3(grid_cap((N + (kBlock / kWave) - 1) / (kBlock / kWave), 2048)), dim3(kBlock), 0, s,
                             p, t, N, static_cast<int>(C), ig, has_ignore, samplewise, w);
        } else if (kind == 0 && P == 1) {
          auto row = [&](auto g) {
            constexpr int G = decltype(g)::value;
            hipLaunchKernelGGL((em_multiclass_row_kernel<scalar_t, target_t, G>),
                               dim3(grid_cap((N + kBlock / G - 1) / (kBlock / G), 1024)), dim3(kBlock), 0, s, p, t, N,
                               static_cast<int>(C), ig, has_ignore, samplewise, w);
          };
          if (C <= 8)
            row(std::integral_constant<int, 8>{});
          else if (C <= 16)
            row(std::integral_constant<int, 16>{});
          else if (C <= 32)
            row(std::integral_constant<int, 32>{});
          else
            row(std::integral_constant<int, 64>{});
        } else if (kind == 0) {
          hipLaunchKernelGGL((em_multiclass_pos_kernel<scalar_t, target_t>),
                             dim3(grid_cap((N + (kBlock / kWave) - 1) / (kBlock / kWave), 2048)), dim3(kBlock), 0,
                             s, p, t, N, static_cast<int>(C), static_cast<long long>(P), ig, has_ignore,
                             samplewise, w);
        } else if (kind == 1) {
          hipLaunchKernelGGL((em_multilabel_kernel<scalar_t, target_t, false>),
                             dim3(grid_cap((N * P + kBlock - 1) / kBlock, 2048)), dim3(kBlock), 0, s, p, t, N,
                             static_cast<int>(C), static_cast<long long>(P), thr, ig,
                             has_ignore, samplewise, w, notprob.data_ptr<int>());
        } else {
          hipLaunchKernelGGL((em_multilabel_kernel<scalar_t, target_t, true>),
                             dim3(grid_cap((N + kBlock - 1) / kBlock, 2048)), dim3(kBlock), 0, s, p, t, N,
                             static_cast<int>(C), 1LL, thr, ig, has_ignore, samplewise, w,
                             notprob.data_ptr<int>());
        }
      });
    });
  }
  const bool two = kind == 1;
  const long long total_add = kind == 1 ? N * P : N;
  if (samplewise) {
    if (N > 0)
      hipLaunchKernelGGL(em_fold_kernel, dim3(grid_cap((N + 255) / 256, 1024)), dim3(256), 0, s, w, N, true, two,
                         notprob.data_ptr<int>(), correct.data_ptr<int64_t>(), total.data_ptr<int64_t>(), total_add,
                         out.data_ptr<int64_t>());
    if (two) hipLaunchKernelGGL(em_reset_notprob_kernel, dim3(1), dim3(1), 0, s, notprob.data_ptr<int>());
  } else {
    hipLaunchKernelGGL(em_fold_kernel, dim3(1), dim3(64), 0, s, w, N, false, two, notprob.data_ptr<int>(),
                       correct.data_ptr<int64_t>(), total.data_ptr<int64_t>(), total_add, nullptr);
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "exact_match_update(Tensor preds, Tensor target, int kind, int C, int P, bool has_c, float threshold, "
      "int ignore_index, bool has_ignore, bool samplewise, Tensor(a!) ws, Tensor(b!) notprob, Tensor(c!) correct, "
      "Tensor(d!) total, Tensor(e!) out) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("exact_match_update", &exact_match_update); }

}  // namespace tm_amd
