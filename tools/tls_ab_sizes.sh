#!/bin/bash
# TLS crypto A/B over record sizes: tools/bench_tls.py against each build in tools/bin, one
# process each.  usage: CIPHER=chacha SIZES="64:256 16:1024 4:4096 2:8192" tools/tls_ab_sizes.sh
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${SIZES:-64:256 16:1024 4:4096 2:8192}; do
  recs=${spec%%:*}; plen=${spec##*:}
  for lib in tools/bin/libws_*.so; do
    timeout -k 10 200 python tools/bench_tls.py --lib "$lib" --cipher ${CIPHER:-chacha} --records $recs --plen $plen \
      --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abs.json 2> gpurun_out/abs.err || { echo "fail $lib"; tail -5 gpurun_out/abs.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abs.json')); print('$plen', sys.argv[1], d['value'], d['kernel']['plaintext_gbs'])" $(basename $lib .so)
  done
done
