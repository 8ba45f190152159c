#!/bin/bash
# send side: build tests on the tree, then A/B of library builds (tools/bin/libws_*.so)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build.py \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for cfg in c4 c4 c2 c64; do
  timeout -k 10 300 python -u tools/ab_build.py $cfg "$@" >> gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
done
cat gpurun_out/${T}_ab.txt
