set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dgemm_gpu.py tests/test_pairwise_precision_gpu.py tests/test_determinism_gpu.py > gpurun_out/dgv_tests.log 2>&1 || { tail -30 gpurun_out/dgv_tests.log; exit 1; }
tail -2 gpurun_out/dgv_tests.log
for v in ${DGV_VARIANTS:-0 8 64 4}; do TM_AMD_DGEMM_VARIANT=$v timeout -k 10 200 python benchmarks/bench_dgemm.py 2>&1 | grep '^{' >> gpurun_out/dgv_bench.jsonl || exit 1; done
cat gpurun_out/dgv_bench.jsonl | cut -c1-130
