#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5m7.txt
: > $O
for n in 8192 32768 65536; do for r in 512 256 1024; do
cd /tmp && TM_AMD_MOMENTS_ROWS=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m7 -o p -- python3 $R/benchmarks/moments_probe.py --n $n --cases config5 > $R/gpurun_out/m7.log 2>&1 || { tail -5 $R/gpurun_out/m7.log; exit 1; }
cd $R && echo "n=$n rows=$r $(python3 tools/gpu/kstats.py gpurun_out/m7 moments | cut -c60-)" >> $O; rm -rf gpurun_out/m7
done; done
cat $O
