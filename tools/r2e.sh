set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_graphed_compute_gpu.py tests/test_kernels_gpu.py tests/test_classification_extras.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2e_tests.log 2>&1; rc=$?; tail -30 gpurun_out/r2e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/graphed_compute_breakdown.py 2>&1 | grep -v amdgpu.ids || exit 1
for a in "--sync-every-step --graph"; do
  timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 $a 2>&1 | grep -v amdgpu.ids || exit 1
done
