#!/bin/bash
# same-process A/B of the C4 stream decode: the walk's own payload pass at kU = 4 / 8 / 16 loads per
# lane, against the payload kernel (UVHTTP_WS_WALK_UNMASK=0)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
{
timeout -k 10 300 python -u tools/ab_lib.py tree tools/bin/libws_ku8.so c4:streams || exit 1
timeout -k 10 300 python -u tools/ab_lib.py tree tools/bin/libws_pipe4.so c4:streams || exit 1
timeout -k 10 300 python -u tools/ab_lib.py tree tools/bin/libws_pipe8.so c4:streams || exit 1
AB_ENV_B=UVHTTP_WS_WALK_UNMASK=0 timeout -k 10 300 python -u tools/ab_lib.py tree tree c4:streams || exit 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab.txt
