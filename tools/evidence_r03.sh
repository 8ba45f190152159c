#!/bin/bash
# Round-3 final evidence on one GPU box (every GPU step time-limited; the first failure ends it):
# full GPU suite + smoke + default bench (round_end.sh), the all-mode matrix, rocprofv3 stats +
# PMC traffic for C3/C4/C2 in place, TLS open benches and the TLS -> WebSocket chain, the
# live-shape e2e with the box's PCIe ceiling.   usage: TAG=r03f tools/evidence_r03.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03f}
export TAG
tools/round_end.sh
tools/bench_matrix.sh
tools/profile.sh c3 inplace
tools/profile.sh c4 inplace
tools/profile.sh c2 inplace
for c in aes chacha; do
  timeout -k 10 300 python tools/bench_tls.py --cipher $c --steps 10 --warmup 2 \
    > gpurun_out/bench_tls_${c}_$TAG.json 2> gpurun_out/bench_tls_${c}_$TAG.err
  cat gpurun_out/bench_tls_${c}_$TAG.json
done
: > gpurun_out/tls_chain_$TAG.jsonl
for args in "--plen 16384 --records 4" "--plen 1024 --records 64" "--plen 16384 --records 4 --cipher chacha" "--plen 1024 --records 64 --cipher chacha"; do
  timeout -k 10 200 python tools/bench_tls.py --chain --conns 16384 $args --steps 10 >> gpurun_out/tls_chain_$TAG.jsonl 2>> gpurun_out/tls_chain_$TAG.err
done
cat gpurun_out/tls_chain_$TAG.jsonl
timeout -k 10 900 python bench.py --config c2 --e2e --no-cpu-baseline --no-c5-base > gpurun_out/bench_e2e_$TAG.json 2> gpurun_out/bench_e2e_$TAG.err
cat gpurun_out/bench_e2e_$TAG.json
