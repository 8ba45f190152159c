#!/bin/bash
# same-process A/B: the speculative compact pass reading 8-byte-aligned payload windows as two
# 8-byte LDS reads (-DUVWS_SPEC_B64) against the tree, C4 compact with and without descriptors
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_lib.py tree tools/bin/libws_specb64.so c4:compact_nd c4:compact c4:compact_nd 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab.txt
