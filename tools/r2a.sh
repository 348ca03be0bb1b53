set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_gpu_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r2_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1 && tail -3 gpurun_out/r2_bench.log
