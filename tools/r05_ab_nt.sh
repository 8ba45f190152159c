#!/bin/bash
# same-process A/B of the C4 / C2 stream decodes: streaming stores for the walk's frame records
# and k_stream_desc's descriptors (UVHTTP_WS_STREAM_NT=1, engine B) against write-back stores
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
{
AB_ENV_B=UVHTTP_WS_STREAM_NT=1 timeout -k 10 300 python -u tools/ab_lib.py tree tree c4:streams c2:streams || exit 1
AB_ENV_B=UVHTTP_WS_STREAM_NT=1 timeout -k 10 300 python -u tools/ab_lib.py tree tree c4:streams || exit 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab.txt
UVHTTP_WS_STREAM_NT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
