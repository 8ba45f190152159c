#!/bin/bash
# after the stream-scratch fixes: the batcher suites first (fresh process, the closing run's
# crash), then the stream suites
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -X faulthandler -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_batcher_group.py tests/test_batcher_transitions.py tests/test_gpu_batcher.py tests/test_gpu_batcher_tls.py \
  > gpurun_out/${T}_batcher.log 2>&1 || { tail -30 gpurun_out/${T}_batcher.log; exit 1; }
tail -1 gpurun_out/${T}_batcher.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_streams_full.py tests/test_gpu_engine.py tests/test_gpu_stamps.py \
  > gpurun_out/${T}_streams.log 2>&1 || { tail -30 gpurun_out/${T}_streams.log; exit 1; }
tail -1 gpurun_out/${T}_streams.log
