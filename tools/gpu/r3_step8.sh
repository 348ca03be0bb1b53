#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mb/confmat_ring_mb > gpurun_out/r3_confmat_ring_mb2.jsonl 2>&1 || { tail -20 gpurun_out/r3_confmat_ring_mb2.jsonl; exit 1; }
cat gpurun_out/r3_confmat_ring_mb2.jsonl
