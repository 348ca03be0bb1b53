#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 300 python -u benchmarks/bench_misc_kernels.py > gpurun_out/misc.jsonl 2>&1 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/misc_prof -o p --output-format csv -- python3 $R/benchmarks/bench_misc_kernels.py > $R/gpurun_out/misc_prof.log 2>&1)
