#!/bin/bash
# Run the given GPU test files in ONE pytest process with a per-test timeout; log under gpurun_out/.
#   bash tools/gpu/tests.sh <log-name> <pytest args...>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
NAME=$1; shift
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/$NAME.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/$NAME.log | tail -30
tail -5 gpurun_out/$NAME.log
exit $rc
