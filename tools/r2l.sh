#!/bin/bash
# GPU step: read_flag probe + host compute costs + validation tests + headline bench
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 120 python -u benchmarks/flag_read_probe.py > gpurun_out/flag_probe.json 2>&1 &&
timeout -k 10 200 python -u benchmarks/host_update_profile.py > gpurun_out/host_prof.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2l_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2l_bench20.json 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 500 --warmup 20 > gpurun_out/r2l_bench500.json 2>&1
