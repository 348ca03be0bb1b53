#!/bin/bash
# Round 5: counters of the 16-bit GEMM (ours vs hipBLASLt) at 8192 x 8192 x 512 bf16, one pass per counter set.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmch$i -o p -- python3 $R/benchmarks/gemm16_one.py > $R/gpurun_out/r5pmch$i.log 2>&1 || { tail -5 $R/gpurun_out/r5pmch$i.log; exit 1; }
done
cd $R && python3 - <<'PY' > gpurun_out/r5_pmc_gemm16.txt
import csv, glob, collections
for d in ("pmch1", "pmch2", "pmch3"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        k = "ours" if "gemm_nt_h16" in r["Kernel_Name"] else ("vendor" if ("Cijk" in r["Kernel_Name"] or "gemm" in r["Kernel_Name"].lower()) else None)
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
    for k in agg:
        print(d, k, {c: f"{v / n[k][c]:.4g}" for c, v in sorted(agg[k].items())})
PY
cat gpurun_out/r5_pmc_gemm16.txt
python3 tools/gpu/trace_summary.py gpurun_out/pmch1 | cut -c1-160 | head -12
rm -rf gpurun_out/pmch1 gpurun_out/pmch2 gpurun_out/pmch3
