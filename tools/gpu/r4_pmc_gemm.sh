#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmcg$i -o p -- python3 $R/benchmarks/gemm_one.py > $R/gpurun_out/r4pmcg$i.log 2>&1 || { tail -5 $R/gpurun_out/r4pmcg$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ("pmcg1", "pmcg2"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        k = "ours" if "gemm_nt_big" in r["Kernel_Name"] else ("vendor" if "Cijk" in r["Kernel_Name"] else None)
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
    for k in agg:
        print(d, k, {c: f"{v / n[k][c]:.4g}" for c, v in sorted(agg[k].items())})
PY
python3 tools/gpu/trace_summary.py gpurun_out/pmcg1 | cut -c1-140
rm -rf gpurun_out/pmcg1 gpurun_out/pmcg2
