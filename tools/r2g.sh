set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python benchmarks/collection_step_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
