#!/bin/bash
# Extra round evidence: the streams row of the matrix, the end-to-end (PCIe-inclusive) rates,
# TLS record-size sweep.  usage: TAG=r02g tools/evidence_extra.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
export TAG
MODES=streams tools/bench_matrix.sh
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c5-base --e2e \
  > gpurun_out/bench_e2e_$TAG.json 2> gpurun_out/bench_e2e_$TAG.err
cat gpurun_out/bench_e2e_$TAG.json
: > gpurun_out/tls_sizes_$TAG.jsonl
for c in aes chacha; do
  for spec in "64 256" "16 1024" "4 4096"; do
    set -- $spec
    timeout -k 10 300 python tools/bench_tls.py --cipher $c --records $1 --plen $2 --steps 5 --warmup 2 \
      --no-cpu-baseline >> gpurun_out/tls_sizes_$TAG.jsonl 2>> gpurun_out/tls_sizes_$TAG.err
  done
done
python3 -c "
import json,sys
for l in open('gpurun_out/tls_sizes_$TAG.jsonl'):
    d=json.loads(l); print(d['config']['workload'], d['value'], d['kernel']['plaintext_gbs'])"
