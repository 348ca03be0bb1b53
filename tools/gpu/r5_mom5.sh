#!/bin/bash
# moments_small_kernel ablation (measurement only): where do the ~8 us of a 1024-pair launch go
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for c in config5; do for a in 0 1 2 7; do
cd /tmp && TM_AMD_MOMENTS_HANDOFF=0 TM_AMD_MOMENTS_ABLATE=$a timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m5 -o p -- python3 $R/benchmarks/moments_probe.py --n 1024 --cases $c > $R/gpurun_out/m5.log 2>&1 || { tail -5 $R/gpurun_out/m5.log; exit 1; }
cd $R && echo "case=$c ablate=$a" >> gpurun_out/r5m5_kstats.txt && python3 tools/gpu/kstats.py gpurun_out/m5 moments launch >> gpurun_out/r5m5_kstats.txt; rm -rf gpurun_out/m5
done; done
cat gpurun_out/r5m5_kstats.txt
