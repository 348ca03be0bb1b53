#!/bin/bash
# One mAP compute() on the device timeline: rocprofv3 kernel + HIP runtime trace of map_compute_timing.py's runs,
# then tools/gpu/compute_window.py between two coco_summary_kernel dispatches.
#   bash tools/gpu/map_window.sh <name>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-mapw}
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/gpurun_out/${N}_tr -o p --output-format csv -- python3 $R/benchmarks/map_compute_timing.py > $R/gpurun_out/${N}_tr.log 2>&1 || { tail -20 $R/gpurun_out/${N}_tr.log; exit 1; }
cd $R && python3 tools/gpu/compute_window.py gpurun_out/${N}_tr --end coco_summary_kernel --nth 3 > gpurun_out/${N}_window.txt
tail -16 gpurun_out/${N}_window.txt
rm -rf gpurun_out/${N}_tr
