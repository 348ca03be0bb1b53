// Extended edit distance (RWTH EED) DP for a batch of (hypothesis, reference) code-point sequences, host side.
// Exact sequential double-precision recurrence of the reference (F/text/eed.py:41-85: CDER initialisation, deletion
// chain, jump to alpha + row minimum after reference blanks, coverage penalty from first-argmin visit counts),
// parallel over pairs with at::parallel_for.  Registered for the CPU dispatch key: text inputs are host strings.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdint>
#include <limits>
#include <vector>

namespace tm_amd {
namespace {

double eed_one(const int* h, int n, const int* r, int m, double alpha, double rho, double del, double ins,
               std::vector<double>& row, std::vector<double>& nxt, std::vector<long>& visits) {
  row.assign(n + 1, 1.0);
  row[0] = 0.0;
  nxt.assign(n + 1, 0.0);
  visits.assign(n + 1, -1);
  for (int w = 0; w < m; ++w) {
    const int rc = r[w];
    nxt[0] = row[0] + 1.0;
    for (int i = 1; i <= n; ++i) {
      double v = nxt[i - 1] + del;
      const double s = row[i - 1] + (h[i - 1] != rc ? 1.0 : 0.0);
      if (s < v) v = s;
      const double t = row[i] + ins;
      if (t < v) v = t;
      nxt[i] = v;
    }
    int k = 0;
    for (int i = 1; i <= n; ++i)
      if (nxt[i] < nxt[k]) k = i;
    visits[k] += 1;
    if (rc == ' ') {
      const double jump = alpha + nxt[k];
      for (int i = 0; i <= n; ++i) nxt[i] = std::min(nxt[i], jump);
    }
    std::swap(row, nxt);
  }
  double cov = 0.0;
  for (long v : visits) cov += v >= 0 ? static_cast<double>(v) : 1.0;
  cov *= rho;
  const double score = (row[n] + cov) / (static_cast<double>(m) + cov);
  return score < 1.0 ? score : 1.0;
}

at::Tensor eed_scores(const at::Tensor& hyp, const at::Tensor& hoff, const at::Tensor& ref, const at::Tensor& roff,
                      double alpha, double rho, double del, double ins) {
  TORCH_CHECK(!hyp.is_cuda(), "eed_scores is a host op");
  TORCH_CHECK(hyp.scalar_type() == at::kInt && ref.scalar_type() == at::kInt, "eed_scores: int32 code points");
  TORCH_CHECK(hoff.scalar_type() == at::kLong && roff.scalar_type() == at::kLong, "eed_scores: int64 offsets");
  TORCH_CHECK(hoff.numel() == roff.numel(), "eed_scores: offset size mismatch");
  const auto hc = hyp.contiguous(), rc = ref.contiguous(), ho = hoff.contiguous(), ro = roff.contiguous();
  const int64_t npairs = ho.numel() - 1;
  auto out = at::empty({npairs}, hyp.options().dtype(at::kDouble));
  const int* h = hc.data_ptr<int>();
  const int* r = rc.data_ptr<int>();
  const int64_t* hp = ho.data_ptr<int64_t>();
  const int64_t* rp = ro.data_ptr<int64_t>();
  double* o = out.data_ptr<double>();
  at::parallel_for(0, npairs, 4, [&](int64_t b0, int64_t b1) {
    std::vector<double> row, nxt;
    std::vector<long> visits;
    for (int64_t b = b0; b < b1; ++b)
      o[b] = eed_one(h + hp[b], static_cast<int>(hp[b + 1] - hp[b]), r + rp[b], static_cast<int>(rp[b + 1] - rp[b]),
                     alpha, rho, del, ins, row, nxt, visits);
  });
  return out;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("eed_scores(Tensor hyp, Tensor hoff, Tensor ref, Tensor roff, float alpha, float rho, float dele, "
        "float ins) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CPU, m) { m.impl("eed_scores", &eed_scores); }

}  // namespace tm_amd
