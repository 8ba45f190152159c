#!/bin/bash
# Run GPU test files one pytest process at a time, each bounded; log under gpurun_out/.
# usage: tools/gpu_tests.sh LOGNAME test_file [test_file ...]   (extra pytest args via PYARGS)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LOG=gpurun_out/$1
shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${PYARGS:-} "$@" > "$LOG" 2>&1
rc=$?
tail -5 "$LOG"
exit $rc
