#!/bin/bash
# GPU step: FID Newton-Schulz compute -- tests, bench, kernel profile
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_image_generative.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2k_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_fid.py > gpurun_out/r2k_fid.jsonl 2>&1 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2k_prof -o p --output-format csv -- python3 $R/benchmarks/bench_fid.py > $R/gpurun_out/r2k_prof.log 2>&1)
