#!/bin/bash
# Full GPU suite + smoke + separate rocprof kernel traces of our headline path and of the emulated baseline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_full_gpu_suite.log 2>&1
rc=$?
tail -15 gpurun_out/r3_full_gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ours -o ours -- python3 $R/bench.py --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/r3_prof_ours.log 2>&1 || { tail -20 $R/gpurun_out/r3_prof_ours.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_base -o base -- python3 $R/benchmarks/reference_headline.py > $R/gpurun_out/r3_prof_base.log 2>&1 || { tail -20 $R/gpurun_out/r3_prof_base.log; exit 1; }
cd $R
cp $(find gpurun_out/prof_ours -name "*kernel_stats.csv" | head -1) gpurun_out/r3_headline_ours_kernel_stats.csv
cp $(find gpurun_out/prof_base -name "*kernel_stats.csv" | head -1) gpurun_out/r3_headline_baseline_kernel_stats.csv
rm -rf gpurun_out/prof_ours gpurun_out/prof_base
cut -d, -f1-4 gpurun_out/r3_headline_ours_kernel_stats.csv | head -8
