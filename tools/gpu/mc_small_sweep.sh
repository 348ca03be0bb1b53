set -o pipefail
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "TM_AMD_FEWBINS_FUSED=0 TM_AMD_MC_STATS_DIRECT=0" "TM_AMD_FEWBINS_GROUP=0" "TM_AMD_FEWBINS_GROUP=2" "TM_AMD_FEWBINS_GROUP=4" "TM_AMD_FEWBINS_GROUP=8" "TM_AMD_FEWBINS_GROUP=16" "TM_AMD_FEWBINS_GROUP=4 TM_AMD_FEWBINS_TILE=2" "TM_AMD_FEWBINS_GROUP=4 TM_AMD_FEWBINS_TILE=4" "TM_AMD_FEWBINS_FUSED=0 TM_AMD_MC_STATS_DIRECT=0"; do
  ( export $v && timeout -k 10 120 python3 -u benchmarks/bench_mc_small.py >> gpurun_out/mcs2_bench.jsonl 2>> gpurun_out/mcs2_bench.err ) || { echo "variant $v failed"; tail -20 gpurun_out/mcs2_bench.err; exit 1; }
done
cat gpurun_out/mcs2_bench.jsonl
bash tools/gpu/kstat_sweep.sh mcs2 benchmarks/bench_mc_small.py fewbins "TM_AMD_FEWBINS_FUSED=0 TM_AMD_MC_STATS_DIRECT=0" "TM_AMD_FEWBINS_GROUP=0" "TM_AMD_FEWBINS_GROUP=4" "TM_AMD_FEWBINS_GROUP=8"
