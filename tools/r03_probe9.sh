#!/bin/bash
# Round-3 probe 9: TLS through the batcher + all batcher tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p9
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_batcher_tls.py tests/test_gpu_batcher.py tests/test_batcher_transitions.py tests/test_gpu_known_answers.py > $OUT/pytest.log 2>&1
rc=$?
tail -40 $OUT/pytest.log | grep -E "passed|failed|Error|assert|^E " | head -30
exit $rc
