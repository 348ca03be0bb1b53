#!/bin/bash
# Two PMC passes over a benchmarks/*_pmc_driver.py (DRIVER=..., default the fp64 GEMM one), one pass per run.
#   bash tools/gpu/dgemm_pmc.sh <name>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-dpmc}
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/${N}_p$i -o p --output-format csv -- python3 $R/benchmarks/${DRIVER:-dgemm_pmc_driver.py} $ARGS > $R/gpurun_out/${N}_p$i.log 2>&1 || { tail -20 $R/gpurun_out/${N}_p$i.log; exit 1; }
  cd $R && f=$(find gpurun_out/${N}_p$i -name "*counter_collection.csv" | head -1) && cp $f gpurun_out/${N}_p$i.csv && rm -rf gpurun_out/${N}_p$i
done
python3 tools/gpu/pmc_summary.py gpurun_out/${N}_p1.csv gpurun_out/${N}_p2.csv
