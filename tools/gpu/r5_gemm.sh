#!/bin/bash
# Round 5: 16-bit GEMM ring variant -- correctness, A/B bench against the 2-stage kernel and hipBLASLt, counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
TM_AMD_GEMM16_RING=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py -m gpu > gpurun_out/r5g_tests.log 2>&1 || { tail -30 gpurun_out/r5g_tests.log; exit 1; }
tail -1 gpurun_out/r5g_tests.log
timeout -k 10 200 python3 benchmarks/bench_gemm16.py > gpurun_out/r5g_bench_ring0.jsonl 2>&1 || { tail -5 gpurun_out/r5g_bench_ring0.jsonl; exit 1; }
TM_AMD_GEMM16_RING=1 timeout -k 10 200 python3 benchmarks/bench_gemm16.py > gpurun_out/r5g_bench_ring1.jsonl 2>&1 || { tail -5 gpurun_out/r5g_bench_ring1.jsonl; exit 1; }
grep shape gpurun_out/r5g_bench_ring0.jsonl | cut -c1-200
grep shape gpurun_out/r5g_bench_ring1.jsonl | cut -c1-200
cd /tmp
i=0
for ring in 0 1; do
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  TM_AMD_GEMM16_RING=$ring timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmch$i -o p -- python3 $R/benchmarks/gemm16_one.py > $R/gpurun_out/r5pmch$i.log 2>&1 || { tail -5 $R/gpurun_out/r5pmch$i.log; exit 1; }
done
done
cd $R && python3 - <<'PY' > gpurun_out/r5_pmc_gemm16.txt
import csv, glob, collections
for d in ("pmch1", "pmch2", "pmch3", "pmch4"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = "ours_ring" if "h16_ring" in name else ("ours" if "gemm_nt_h16" in name else ("vendor" if ("Cijk" in name or "gemm" in name.lower()) else None))
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
    for k in agg:
        print(d, k, {c: f"{v / n[k][c]:.4g}" for c, v in sorted(agg[k].items())})
PY
cat gpurun_out/r5_pmc_gemm16.txt
python3 tools/gpu/trace_summary.py gpurun_out/pmch1 | cut -c1-160 | head -8
python3 tools/gpu/trace_summary.py gpurun_out/pmch3 | cut -c1-160 | head -8
rm -rf gpurun_out/pmch1 gpurun_out/pmch2 gpurun_out/pmch3 gpurun_out/pmch4
