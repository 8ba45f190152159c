#!/bin/bash
# TLS crypto-kernel A/B: bench_tls.py against each variant build in tools/bin (one process each).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in tools/bin/libws_*.so; do
  timeout -k 10 200 python tools/bench_tls.py --lib "$lib" --steps 10 --warmup 2 --no-cpu-baseline ${TLS_ARGS:-} \
    > gpurun_out/ab_$(basename $lib .so).json 2> gpurun_out/ab_$(basename $lib .so).err || { echo "fail $lib"; tail -5 gpurun_out/ab_$(basename $lib .so).err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['lib'], d['value'], d['kernel']['avg_us'], d['kernel']['plaintext_gbs'])" gpurun_out/ab_$(basename $lib .so).json
done
