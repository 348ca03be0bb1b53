#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for v in 1 0 1 0; do
  TORCHMETRICS_AMD_FUSED_SCALARS=$v timeout -k 10 200 python benchmarks/collection_host_breakdown.py > gpurun_out/r4i18_bd$v.json 2>gpurun_out/r4i18_bd.err || { tail -20 gpurun_out/r4i18_bd.err; exit 1; }
  echo "scalars=$v $(cat gpurun_out/r4i18_bd$v.json)"
done
