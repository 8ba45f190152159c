#!/bin/bash
# packed AES-GCM kernel A/B (T-table copies, waves per workgroup, tree tables from global):
# TLS 1.3 AES-128-GCM records of 256 B / 1 KiB / 4 KiB / 16 KiB, one process per build
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03p17
for spec in 64:256 16:1024 4:4096; do
  recs=${spec%%:*}; plen=${spec##*:}
  for lib in tools/bin/libws_*.so; do
    n=$(basename $lib .so)
    timeout -k 10 200 python tools/bench_tls.py --lib "$lib" --cipher aes --records $recs --plen $plen --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r03p17/$n.$plen.json 2> gpurun_out/r03p17/$n.$plen.err || { echo "fail $n $plen"; tail -5 gpurun_out/r03p17/$n.$plen.err; exit 1; }
    python3 -c "
import json
a=json.load(open('gpurun_out/r03p17/$n.$plen.json'))
print('$plen', '$n', a['value'], a['kernel']['avg_us'], a['kernel']['plaintext_gbs'])"
  done
done
