#!/bin/bash
# moments_small_kernel counters at 1024 pairs, full vs fully ablated (measurement only)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp
for a in 0 7; do
  TM_AMD_MOMENTS_HANDOFF=0 TM_AMD_MOMENTS_ABLATE=$a timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/gpurun_out/mom$a -o p -- python3 $R/benchmarks/moments_probe.py --n 1024 --cases config5 > $R/gpurun_out/mom$a.log 2>&1 || { tail -5 $R/gpurun_out/mom$a.log; exit 1; }
  TM_AMD_MOMENTS_HANDOFF=0 TM_AMD_MOMENTS_ABLATE=$a timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_SMEM --kernel-trace --output-format csv -d $R/gpurun_out/mob$a -o p -- python3 $R/benchmarks/moments_probe.py --n 1024 --cases config5 > $R/gpurun_out/mob$a.log 2>&1 || { tail -5 $R/gpurun_out/mob$a.log; exit 1; }
done
cd $R && python3 - <<'PY' | tee gpurun_out/r5m6_counters.txt
import csv, glob, collections
for d in ("mom0", "mob0", "mom7", "mob7"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "moments_small" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(d, {c: f"{v / n[c]:.4g}" for c, v in sorted(agg.items())})
PY
rm -rf gpurun_out/mom? gpurun_out/mob?
