set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_graphed_compute_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2c_tests.log 2>&1; rc=$?; tail -30 gpurun_out/r2c_tests.log; [ $rc -eq 0 ] || exit $rc
for a in "--sync-every-step" "--sync-every-step --graph" "--graph"; do
  timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 $a 2>&1 | grep -v amdgpu.ids || exit 1
done
