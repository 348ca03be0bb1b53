#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mb/confmat_ring_mb | tee gpurun_out/r3_confmat_ring_mb.jsonl
