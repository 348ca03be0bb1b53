#!/bin/bash
# misc kernel bench (incl. top-k) + kernel stats for the topk rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_misc_kernels.py > gpurun_out/r2r_misc.jsonl 2> gpurun_out/r2r_misc.err
rc=$?; cat gpurun_out/r2r_misc.jsonl; exit $rc
