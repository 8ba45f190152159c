#!/bin/bash
# A/B of two builds on bench.py lines that ab_lib.py cannot drive (streams mode): on the GPU box
# (a scratch copy of the tree) swap the in-tree library between OLD and the tree's own build,
# twice, interleaved; then the stream tests on the tree's build.
#   usage (GPU box): OLD=tools/bin/libws_old.so tools/ab_streams_swap.sh [cfg:mode ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OLD=${OLD:?OLD=path to the baseline library}
PAIRS=${*:-c3:streams c2:streams c4:streams}
LIB=uvhttp_amd/lib/libuvhttp_ws_amd.so
cp $LIB /tmp/new.so
for r in 1 2; do
  cp "$OLD" $LIB
  tools/r04_bench_quick.sh r04_swap_old$r.jsonl $PAIRS > gpurun_out/r04_swap_old$r.txt 2>&1 || exit 1
  cp /tmp/new.so $LIB
  tools/r04_bench_quick.sh r04_swap_new$r.jsonl $PAIRS > gpurun_out/r04_swap_new$r.txt 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_streams_full.py > gpurun_out/r04_swap_tests.txt 2>&1
