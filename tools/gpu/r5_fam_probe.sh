#!/bin/bash
# family_rows_g_kernel: ablations (kernel trace per setting) + counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp
for ab in 0 1 2 4 8 15; do
  TM_AMD_FAMILY_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fp_$ab -o p -- python3 $R/benchmarks/family_probe.py > $R/gpurun_out/fp_$ab.log 2>&1 || { tail -5 $R/gpurun_out/fp_$ab.log; exit 1; }
  echo "ablate=$ab $(grep step_us $R/gpurun_out/fp_$ab.log) $(grep -h family_rows $(find $R/gpurun_out/fp_$ab -name '*kernel_stats.csv') | cut -d, -f2-4)"
  rm -rf $R/gpurun_out/fp_$ab
done
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/fpm$i -o p -- python3 $R/benchmarks/family_probe.py > $R/gpurun_out/fpm$i.log 2>&1 || { tail -5 $R/gpurun_out/fpm$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ("fpm1", "fpm2"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        for k in ("family_rows_g", "family_fold", "moments_small"):
            if k in name:
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
    for k in agg:
        print(d, k, {c: f"{v / n[k][c]:.4g}" for c, v in sorted(agg[k].items())})
PY
rm -rf gpurun_out/fpm1 gpurun_out/fpm2
