set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_h -o p --output-format csv -- python3 $R/benchmarks/update_graph_kernels.py > $R/gpurun_out/prof_h.log 2>&1) || { tail -20 gpurun_out/prof_h.log; exit 1; }
f=$(find gpurun_out/prof_h -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/r2h_kernel_trace.csv
rm -rf gpurun_out/prof_h
echo ok
