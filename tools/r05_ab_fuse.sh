#!/bin/bash
# same-process A/B of the C4 stream decode: the walk, scan and k_stream_desc apart (default)
# against k_swalk_fused (UVHTTP_WS_WALK_FUSE=1, blocks in blockIdx order); k_swalk_fused with
# block tickets against without; first-step speculation against none (UVWS_WALK_SPEC_FIRST_OFF
# build: tools/build_variant.sh specfirstoff -DUVWS_WALK_SPEC_FIRST_OFF).
# profiles/r05fy_streams_fused_ab.txt ran this with the fused walk as the default (its
# first line: A fused, B apart)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_streams_full.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
{
AB_ENV_B=UVHTTP_WS_WALK_FUSE=1,UVHTTP_WS_PLAN_TICKET=0 timeout -k 10 300 python -u tools/ab_lib.py tree tree c4:streams || exit 1
UVHTTP_WS_WALK_FUSE=1 UVHTTP_WS_PLAN_TICKET=0 AB_ENV_B=UVHTTP_WS_PLAN_TICKET=1 timeout -k 10 300 python -u tools/ab_lib.py tree tree c4:streams || exit 1
timeout -k 10 300 python -u tools/ab_lib.py tree tools/bin/libws_specfirstoff.so c4:streams || exit 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab.txt
