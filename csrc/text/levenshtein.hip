// Batched Levenshtein edit distance on integer token ids (K28 in SURVEY.md): WER / CER / MER / WIL / WIP and the
// beam-limited (tercom / sacrebleu style) EditDistance.
//
// The reference runs an O(P * R) pure-Python DP per sentence pair (F/text/helper.py:329-350, and the beam-limited
// `_LevenshteinEditDistance` at F/text/helper.py:44-295).  Here one 64-lane wave owns one pair and sweeps the DP row
// by row with the previous / current rows in LDS.  Inside a row the vertical and diagonal moves are independent per
// column, and the horizontal (insertion) chain is a prefix minimum:
//     cur[j] = min_{k <= j} ( t[k] + (j - k) * ins ),   t[j] = min(prev[j - 1] + sub(j), prev[j] + del)
//            = j * ins + prefix_min_k( t[k] - k * ins )
// so each 64-column chunk is one wave-wide min-scan (6 DPP/shuffle steps) plus a running carry across chunks.
// The optional tercom beam (cells outside [pseudo_diag - w, pseudo_diag + w) stay +inf) is applied as a column mask,
// which reproduces the reference's (possibly non-optimal) beamed distance bit-exactly.
//
// The same op has a multithreaded host implementation (CPU dispatch key) so CPU-resident metrics avoid the Python
// DP as well.
#include "common/tm_common.h"

#include <ATen/Parallel.h>

#include <cmath>
#include <vector>

namespace tm_amd {
namespace {

constexpr int kInf = 1 << 28;
constexpr int kBeam = 25;  // tercom beam width (F/text/helper.py:21)
constexpr int kWavesPerBlock = 4;

struct Beam {
  double ratio;
  int width;
};

__host__ __device__ inline Beam make_beam(int plen, int rlen) {
  Beam b;
  b.ratio = plen > 0 ? static_cast<double>(rlen) / static_cast<double>(plen) : 1.0;
  b.width = (b.ratio / 2 > kBeam) ? static_cast<int>(ceil(b.ratio / 2 + kBeam)) : kBeam;
  return b;
}

__host__ __device__ inline void beam_range(const Beam& b, int i, int plen, int rlen, int& lo, int& hi) {
  const int diag = static_cast<int>(floor(static_cast<double>(i) * b.ratio));
  lo = diag - b.width > 0 ? diag - b.width : 0;
  hi = (i == plen) ? rlen + 1 : (rlen + 1 < diag + b.width ? rlen + 1 : diag + b.width);
}

__device__ __forceinline__ int wave_prefix_min(int v, int lane) {
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int o = __shfl_up(v, off, kWave);
    if (lane >= off) v = min(v, o);
  }
  return v;
}

// one wave per pair; LDS holds two rows of (max_r + 1) ints per wave
__global__ void __launch_bounds__(kWave* kWavesPerBlock)
    levenshtein_kernel(const int* __restrict__ pred, const int64_t* __restrict__ poff, const int* __restrict__ ref,
                       const int64_t* __restrict__ roff, int npairs, int row_stride, int ins, int del, int sub,
                       int use_beam, int64_t* __restrict__ out) {
  extern __shared__ int lds[];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  const int pair = blockIdx.x * kWavesPerBlock + wave;
  if (pair >= npairs) return;  // whole wave exits together; no block-level barriers below
  int* prev = lds + wave * 2 * row_stride;
  int* cur = prev + row_stride;
  const int* p = pred + poff[pair];
  const int* r = ref + roff[pair];
  const int plen = static_cast<int>(poff[pair + 1] - poff[pair]);
  const int rlen = static_cast<int>(roff[pair + 1] - roff[pair]);

  for (int j = lane; j <= rlen; j += kWave) prev[j] = j * ins;
  const Beam bm = make_beam(plen, rlen);
  for (int i = 1; i <= plen; ++i) {
    int lo = 0, hi = rlen + 1;
    if (use_beam) beam_range(bm, i, plen, rlen, lo, hi);
    const int tok = p[i - 1];
    int carry = kInf;  // prefix min of (t[k] - k * ins) over previous chunks
    for (int j0 = 0; j0 <= rlen; j0 += kWave) {
      const int j = j0 + lane;
      int t = kInf;
      if (j <= rlen && j >= lo && j < hi) {
        const int up = prev[j];
        t = up >= kInf ? kInf : up + del;
        if (j > 0) {
          const int dg = prev[j - 1];
          if (dg < kInf) t = min(t, dg + (r[j - 1] == tok ? 0 : sub));
        }
      }
      const int u = t >= kInf ? kInf : t - j * ins;
      int pm = min(wave_prefix_min(u, lane), carry);
      carry = __shfl(pm, kWave - 1, kWave);
      if (j <= rlen) {
        int v = pm >= kInf ? kInf : pm + j * ins;
        if (j < lo || j >= hi || v > kInf) v = kInf;
        cur[j] = v;
      }
    }
    __builtin_amdgcn_wave_barrier();
    int* tmp = prev;
    prev = cur;
    cur = tmp;
  }
  if (lane == 0) out[pair] = prev[rlen];
}

int64_t host_one(const int* p, int plen, const int* r, int rlen, int ins, int del, int sub, bool use_beam,
                 std::vector<int>& prev, std::vector<int>& cur) {
  prev.resize(rlen + 1);
  cur.resize(rlen + 1);
  for (int j = 0; j <= rlen; ++j) prev[j] = j * ins;
  const Beam bm = make_beam(plen, rlen);
  for (int i = 1; i <= plen; ++i) {
    int lo = 0, hi = rlen + 1;
    if (use_beam) beam_range(bm, i, plen, rlen, lo, hi);
    std::fill(cur.begin(), cur.end(), kInf);
    const int tok = p[i - 1];
    for (int j = lo; j < hi; ++j) {
      int v = prev[j] >= kInf ? kInf : prev[j] + del;
      if (j > 0) {
        if (prev[j - 1] < kInf) v = std::min(v, prev[j - 1] + (r[j - 1] == tok ? 0 : sub));
        if (cur[j - 1] < kInf) v = std::min(v, cur[j - 1] + ins);
      }
      cur[j] = v;
    }
    std::swap(prev, cur);
  }
  return prev[rlen];
}

void check_inputs(const at::Tensor& pred, const at::Tensor& poff, const at::Tensor& ref, const at::Tensor& roff,
                  const at::Tensor& out) {
  TORCH_CHECK(pred.scalar_type() == at::kInt && ref.scalar_type() == at::kInt, "levenshtein: token ids must be int32");
  TORCH_CHECK(poff.scalar_type() == at::kLong && roff.scalar_type() == at::kLong, "levenshtein: offsets must be int64");
  TORCH_CHECK(out.scalar_type() == at::kLong, "levenshtein: out must be int64");
  TM_CHECK_CONTIG(pred);
  TM_CHECK_CONTIG(ref);
  TM_CHECK_CONTIG(poff);
  TM_CHECK_CONTIG(roff);
  TM_CHECK_CONTIG(out);
  TORCH_CHECK(poff.numel() == roff.numel() && out.numel() == poff.numel() - 1, "levenshtein: offset/out size mismatch");
}

}  // namespace

// dist[b] = Levenshtein(pred[poff[b]:poff[b+1]] -> ref[roff[b]:roff[b+1]]) with the given operation costs;
// `max_ref_len` is the host-known max reference length (sizes the LDS rows).
void levenshtein_cuda(const at::Tensor& pred, const at::Tensor& poff, const at::Tensor& ref, const at::Tensor& roff,
                      at::Tensor out, int64_t ins, int64_t del, int64_t sub, bool use_beam, int64_t max_ref_len) {
  check_inputs(pred, poff, ref, roff, out);
  TM_CHECK_CUDA(pred);
  const int npairs = static_cast<int>(out.numel());
  if (npairs == 0) return;
  const int stride = static_cast<int>(max_ref_len) + 1;
  const size_t lds = static_cast<size_t>(kWavesPerBlock) * 2 * stride * sizeof(int);
  TORCH_CHECK(lds <= 160 * 1024, "levenshtein: reference too long for the LDS kernel (", max_ref_len, " tokens)");
  if (lds > 64 * 1024)
    TORCH_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&levenshtein_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) == hipSuccess,
                "levenshtein: cannot raise LDS limit");
  const int blocks = (npairs + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(levenshtein_kernel, dim3(blocks), dim3(kWave * kWavesPerBlock), lds, stream(),
                     pred.data_ptr<int>(), poff.data_ptr<int64_t>(), ref.data_ptr<int>(), roff.data_ptr<int64_t>(),
                     npairs, stride, static_cast<int>(ins), static_cast<int>(del), static_cast<int>(sub),
                     use_beam ? 1 : 0, out.data_ptr<int64_t>());
}

void levenshtein_cpu(const at::Tensor& pred, const at::Tensor& poff, const at::Tensor& ref, const at::Tensor& roff,
                     at::Tensor out, int64_t ins, int64_t del, int64_t sub, bool use_beam, int64_t /*max_ref_len*/) {
  check_inputs(pred, poff, ref, roff, out);
  const int npairs = static_cast<int>(out.numel());
  const int* p = pred.data_ptr<int>();
  const int* r = ref.data_ptr<int>();
  const int64_t* po = poff.data_ptr<int64_t>();
  const int64_t* ro = roff.data_ptr<int64_t>();
  int64_t* o = out.data_ptr<int64_t>();
  at::parallel_for(0, npairs, 16, [&](int64_t b0, int64_t b1) {
    std::vector<int> prev, cur;
    for (int64_t b = b0; b < b1; ++b)
      o[b] = host_one(p + po[b], static_cast<int>(po[b + 1] - po[b]), r + ro[b], static_cast<int>(ro[b + 1] - ro[b]),
                      static_cast<int>(ins), static_cast<int>(del), static_cast<int>(sub), use_beam, prev, cur);
  });
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "levenshtein(Tensor pred, Tensor poff, Tensor ref, Tensor roff, Tensor(a!) out, int ins, int dele, int sub, "
      "bool use_beam, int max_ref_len) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("levenshtein", &levenshtein_cuda); }
TORCH_LIBRARY_IMPL(tm_amd, CPU, m) { m.impl("levenshtein", &levenshtein_cpu); }

}  // namespace tm_amd
