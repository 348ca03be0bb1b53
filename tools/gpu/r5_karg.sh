#!/bin/bash
# kernel-argument placement: kernel durations with HIP_FORCE_DEV_KERNARG unset / 0 / 1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_karg.txt
for v in unset 0 1; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  cd /tmp && TM_AMD_MOMENTS_HANDOFF=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/k1 -o p -- python3 $R/benchmarks/moments_probe.py --n 1024 --cases config5 > $R/gpurun_out/k1.log 2>&1 || { tail -5 $R/gpurun_out/k1.log; exit 1; }
  cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/k2 -o p -- python3 $R/bench.py --steps 200 --warmup 5 --no-baseline > $R/gpurun_out/k2.log 2>&1 || { tail -5 $R/gpurun_out/k2.log; exit 1; }
  cd $R && echo "HIP_FORCE_DEV_KERNARG=$v" >> $O && python3 tools/gpu/kstats.py gpurun_out/k1 moments >> $O && python3 tools/gpu/kstats.py gpurun_out/k2 ord16 >> $O && tail -1 gpurun_out/k2.log | cut -c1-120 >> $O; rm -rf gpurun_out/k1 gpurun_out/k2
done
cat $O
