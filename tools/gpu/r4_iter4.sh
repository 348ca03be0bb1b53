#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_native_forward_gpu.py tests/test_fused_compute_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i4_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i4_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_forward.py 2>gpurun_out/r4i4_forward.err > gpurun_out/r4i4_bench_forward.jsonl || { tail -20 gpurun_out/r4i4_forward.err; exit 1; }
cut -c1-260 gpurun_out/r4i4_bench_forward.jsonl
for tile in 2 0 1 4; do
  TM_AMD_FEWBINS_TILE=$tile timeout -k 10 120 python benchmarks/bench_fewbins.py >> gpurun_out/r4i4_fewbins.jsonl 2>gpurun_out/r4i4_fewbins.err || { tail -20 gpurun_out/r4i4_fewbins.err; exit 1; }
done
grep '"C": 10' gpurun_out/r4i4_fewbins.jsonl | tr -d '{}"' 
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fb -o p -- python3 $R/benchmarks/bench_fewbins.py > $R/gpurun_out/r4i4_pmc.log 2>&1 || { tail -20 $R/gpurun_out/r4i4_pmc.log; exit 1; }
cd $R && find gpurun_out/pmc_fb -name "*.csv" | head -5
