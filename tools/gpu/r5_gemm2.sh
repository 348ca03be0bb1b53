#!/bin/bash
# 16-bit GEMM with the transposed-accumulator vector-store epilogue: tests (both main loops), bench, counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py tests/test_pairwise.py tests/test_pairwise_precision_gpu.py -m gpu > gpurun_out/r5g2_tests.log 2>&1 || { tail -30 gpurun_out/r5g2_tests.log; exit 1; }
tail -1 gpurun_out/r5g2_tests.log
TM_AMD_GEMM16_RING=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py -m gpu > gpurun_out/r5g2_tests_ring.log 2>&1 || { tail -30 gpurun_out/r5g2_tests_ring.log; exit 1; }
tail -1 gpurun_out/r5g2_tests_ring.log
timeout -k 10 200 python3 benchmarks/bench_gemm16.py > gpurun_out/r5g2_bench.jsonl 2>&1 || { tail -5 gpurun_out/r5g2_bench.jsonl; exit 1; }
grep shape gpurun_out/r5g2_bench.jsonl | cut -c1-420
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmch$i -o p -- python3 $R/benchmarks/gemm16_one.py > $R/gpurun_out/r5pmch$i.log 2>&1 || { tail -5 $R/gpurun_out/r5pmch$i.log; exit 1; }
done
cd $R && python3 - <<'PY' > gpurun_out/r5_pmc_gemm16_t.txt
import csv, glob, collections
for d in ("pmch1", "pmch2"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = "ours" if "gemm_nt_h16" in name else ("vendor" if "Cijk" in name else None)
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
    for k in agg:
        print(d, k, {c: f"{v / n[k][c]:.4g}" for c, v in sorted(agg[k].items())})
PY
cat gpurun_out/r5_pmc_gemm16_t.txt
python3 tools/gpu/kstats.py gpurun_out/pmch1 gemm Cijk
rm -rf gpurun_out/pmch1 gpurun_out/pmch2
