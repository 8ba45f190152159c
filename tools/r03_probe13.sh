#!/bin/bash
# AES-GCM kernel A/B (waves per workgroup, T-table copies, red8 table, waves_per_eu):
# 16 KiB and 256-B TLS 1.3 AES-128-GCM records, one process per build in tools/bin.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03p13
for lib in tools/bin/libws_*.so; do
  n=$(basename $lib .so)
  timeout -k 10 200 python tools/bench_tls.py --lib "$lib" --cipher aes --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r03p13/$n.16k.json 2> gpurun_out/r03p13/$n.16k.err || { echo "fail $n"; tail -5 gpurun_out/r03p13/$n.16k.err; exit 1; }
  timeout -k 10 200 python tools/bench_tls.py --lib "$lib" --cipher aes --records 64 --plen 256 --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r03p13/$n.256.json 2> gpurun_out/r03p13/$n.256.err || { echo "fail256 $n"; tail -5 gpurun_out/r03p13/$n.256.err; exit 1; }
  python3 -c "
import json,sys
a=json.load(open('gpurun_out/r03p13/$n.16k.json')); b=json.load(open('gpurun_out/r03p13/$n.256.json'))
print('$n', '16k', a['value'], a['kernel']['avg_us'], a['kernel']['plaintext_gbs'], '256', b['value'], b['kernel']['avg_us'], b['kernel']['plaintext_gbs'])"
done
