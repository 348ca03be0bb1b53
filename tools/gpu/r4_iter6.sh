#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
T="tests/test_stream_kernels_gpu.py tests/test_kernel_boundaries_gpu.py tests/test_kernels_gpu.py tests/test_classification_stats.py tests/test_native_forward_gpu.py"
timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i6_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i6_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
for r in 8 4 2; do
  cd /tmp && TM_AMD_FEWBINS_R=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fb$r -o p -- python3 $R/benchmarks/bench_fewbins.py > $R/gpurun_out/r4i6_fb$r.log 2>&1 || { tail -20 $R/gpurun_out/r4i6_fb$r.log; exit 1; }
  cd $R && python3 - "$r" <<'PY'
import csv, glob, sys, collections
r = sys.argv[1]
f = glob.glob(f"gpurun_out/prof_fb{r}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = collections.defaultdict(list)
for x in rows:
    n = x["Kernel_Name"]
    if "fewbins" in n or "finalize" in n:
        by[(n.split("<")[0][-30:], x["Grid_Size"])].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000)
for k, v in sorted(by.items()):
    v.sort()
    print("R", r, k, "n", len(v), "median_us", round(v[len(v) // 2], 2))
PY
  rm -rf gpurun_out/prof_fb$r
done
timeout -k 10 200 python benchmarks/collection_phases.py --profile gpurun_out/r4i6_collection_profile.txt > gpurun_out/r4i6_collection_phases.json 2>gpurun_out/r4i6_phases.err || { tail -20 gpurun_out/r4i6_phases.err; exit 1; }
cat gpurun_out/r4i6_collection_phases.json
head -45 gpurun_out/r4i6_collection_profile.txt | tail -36 | cut -c1-160
