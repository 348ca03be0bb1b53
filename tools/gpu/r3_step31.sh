#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_s31_pmc -o gemm -- python3 $GRAFT_REPO_ROOT/benchmarks/gemm_pmc_driver.py 4096 4096 2048 > $GRAFT_REPO_ROOT/gpurun_out/r3_s31.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_s31.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r3_s31_pmc -name "*.csv" | head
