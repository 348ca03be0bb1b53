#!/bin/bash
# CLIP math kernels, cat-state arena, retrieval / wrapper changes on the GPU; then the full GPU suite and smoke; then
# rocprof kernel stats of the retrieval PR-curve + CLIP kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_multimodal.py tests/test_state_arena.py tests/test_retrieval_kernel.py tests/test_wrappers.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s36_targeted.log 2>&1 || { tail -30 gpurun_out/r3_s36_targeted.log; exit 1; }
tail -1 gpurun_out/r3_s36_targeted.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_full_gpu_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r3_full_gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
timeout -k 10 300 python benchmarks/bench_retrieval_clip.py > gpurun_out/r3_bench_retrieval_clip.jsonl 2>&1 || { tail -20 gpurun_out/r3_bench_retrieval_clip.jsonl; exit 1; }
cat gpurun_out/r3_bench_retrieval_clip.jsonl | grep -v amdgpu.ids
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rc -o rc -- python3 $R/benchmarks/bench_retrieval_clip.py --ours-only > $R/gpurun_out/r3_prof_rc.log 2>&1 || { tail -20 $R/gpurun_out/r3_prof_rc.log; exit 1; }
cd $R
cp $(find gpurun_out/prof_rc -name "*kernel_stats.csv" | head -1) gpurun_out/r3_retrieval_clip_kernel_stats.csv
rm -rf gpurun_out/prof_rc
cut -d, -f1-4 gpurun_out/r3_retrieval_clip_kernel_stats.csv | cut -c1-150 | head -12
