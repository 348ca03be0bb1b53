#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_detection.py tests/test_panoptic_gpu.py tests/test_reference_doctests.py -k "map or mean_ap or MeanAverage or detection or iou" > gpurun_out/r3_s26_tests.log 2>&1 || { tail -40 gpurun_out/r3_s26_tests.log; exit 1; }
tail -3 gpurun_out/r3_s26_tests.log
timeout -k 10 300 python -u benchmarks/map_compute_phases.py > gpurun_out/r3_s26_map_phases.json 2>&1 || { tail -30 gpurun_out/r3_s26_map_phases.json; exit 1; }
cat gpurun_out/r3_s26_map_phases.json
