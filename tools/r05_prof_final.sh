#!/bin/bash
# round-5 closing rocprofv3 evidence: kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes for the
# headline (C3 in place) and the stream decode (C4, C2)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r05j}
for pair in c3:inplace c4:streams c2:streams; do
  TAG=$TAG timeout -k 10 900 tools/profile.sh ${pair%%:*} ${pair##*:} > gpurun_out/${TAG}_${pair/:/_}_prof.txt 2>&1 || { tail -20 gpurun_out/${TAG}_${pair/:/_}_prof.txt; exit 1; }
  tail -3 gpurun_out/${TAG}_${pair/:/_}_prof.txt
done
