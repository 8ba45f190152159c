#!/bin/bash
# Round evidence on one GPU box: full GPU suite + smoke + default bench (round_end.sh), the
# all-mode matrix, rocprofv3 stats + PMC traffic of the headline kernel, TLS open benches.
# Every GPU step is time-limited; the first failure ends the script.  usage: TAG=r02g tools/evidence.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
export TAG
tools/round_end.sh
tools/bench_matrix.sh
tools/profile.sh c3 inplace
tools/profile.sh c4 inplace
for c in aes chacha; do
  timeout -k 10 300 python tools/bench_tls.py --cipher $c --steps 10 --warmup 2 \
    > gpurun_out/bench_tls_${c}_$TAG.json 2> gpurun_out/bench_tls_${c}_$TAG.err
  cat gpurun_out/bench_tls_${c}_$TAG.json
done
