#!/bin/bash
# Round-3 final evidence, part 3: TLS open benches, the TLS -> WebSocket chain (after the AES
# table change), bench.py --e2e (batch pipeline + live-shape batcher + the box's PCIe ceiling)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03f}
for c in aes chacha; do
  timeout -k 10 300 python tools/bench_tls.py --cipher $c --steps 10 --warmup 2 \
    > gpurun_out/bench_tls_${c}_$TAG.json 2> gpurun_out/bench_tls_${c}_$TAG.err || { echo "tls $c failed"; exit 1; }
  cut -c1-300 gpurun_out/bench_tls_${c}_$TAG.json
done
: > gpurun_out/tls_chain_$TAG.jsonl
for args in "--plen 16384 --records 4" "--plen 1024 --records 64" "--plen 16384 --records 4 --cipher chacha" "--plen 1024 --records 64 --cipher chacha"; do
  timeout -k 10 200 python tools/bench_tls.py --chain --conns 16384 $args --steps 10 >> gpurun_out/tls_chain_$TAG.jsonl 2>> gpurun_out/tls_chain_$TAG.err || { echo "chain failed"; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/tls_chain_$TAG.jsonl'):
    d=json.loads(l); print('chain', d['config']['workload'][:60], d['value'], d['ms_per_step'])"
timeout -k 10 900 python bench.py --config c2 --e2e --no-cpu-baseline --no-c5-base > gpurun_out/bench_e2e_$TAG.json 2> gpurun_out/bench_e2e_$TAG.err || { echo "e2e failed"; tail -5 gpurun_out/bench_e2e_$TAG.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/bench_e2e_$TAG.json'))
print('e2e_pcie', json.dumps(d.get('e2e_pcie'))[:300])
for k,v in d['e2e_live'].items(): print('e2e_live', k, json.dumps(v)[:300])"
