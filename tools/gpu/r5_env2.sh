#!/bin/bash
# Round 5: kernarg preload (compiler) x kernarg placement (runtime) on the standalone region, and which part of the
# Python-side setup before the first region makes its host launches slow.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for b in region_mb region_mb_pre; do
  for i in 1 2; do
    timeout -k 10 60 tools/mb/$b $b >> gpurun_out/r5_region_mb2.jsonl 2>&1 || exit 1
    HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 tools/mb/$b ${b}_hostkarg >> gpurun_out/r5_region_mb2.jsonl 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r5_region_mb2.jsonl"):
    d = json.loads(l)
    print(d["case"], "steady", d["steady_us_per_launch"], *[d[f"rep{r}"] for r in range(4)], "launch", d["launch1"][:6])
PY
for c in onering onering_nocr onering_conly onering_ronly onering onering_nocr onering_conly onering_ronly; do
  timeout -k 10 120 python3 benchmarks/first_region_probe.py $c >> gpurun_out/r5_first_region2.jsonl 2>gpurun_out/r5_fr2.err || { tail -5 gpurun_out/r5_fr2.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r5_first_region2.jsonl"):
    d = json.loads(l)
    print(d["case"], d["rep0"], d["rep1"], "host0", d["per_update0"][:8])
PY
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py tests/test_gemm_big_gpu.py tests/test_macro_curves.py tests/test_corr_merge.py -m gpu > gpurun_out/r5_h16_tests.log 2>&1 || { tail -40 gpurun_out/r5_h16_tests.log; exit 1; }
tail -2 gpurun_out/r5_h16_tests.log
timeout -k 10 300 python3 benchmarks/bench_gemm16.py > gpurun_out/r5_bench_gemm16.jsonl 2>&1 || { tail -5 gpurun_out/r5_bench_gemm16.jsonl; exit 1; }
cut -c1-400 gpurun_out/r5_bench_gemm16.jsonl
