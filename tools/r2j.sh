#!/bin/bash
# GPU step: RLE tests + mAP segm bench (512 x 100 masks @ 640x480) + kernel profile
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_rle.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2j_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_map_segm.py > gpurun_out/r2j_segm.jsonl 2>&1 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2j_prof -o p --output-format csv -- python3 $R/benchmarks/bench_map_segm.py --images 128 > $R/gpurun_out/r2j_prof.log 2>&1)
