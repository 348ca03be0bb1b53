#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $R/gpurun_out/pmc1 -o p -- python3 $R/benchmarks/fewbins_one.py > $R/gpurun_out/r4pmc1.log 2>&1 || { tail -5 $R/gpurun_out/r4pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmc2 -o p -- python3 $R/benchmarks/fewbins_one.py > $R/gpurun_out/r4pmc2.log 2>&1 || { tail -5 $R/gpurun_out/r4pmc2.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ("pmc1", "pmc2"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(float); n = collections.Counter(); dur = []
    for r in csv.DictReader(open(f)):
        if "fewbins_tile" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(d, {k: round(v / n[k]) for k, v in agg.items()})
PY
python3 tools/gpu/trace_summary.py gpurun_out/pmc1 --match fewbins | cut -c1-140
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
