#!/bin/bash
# TLS AES-GCM after the LDS work: GPU TLS tests, record-size sweep (in-tree library), kernel
# trace of the 256-B case
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p20
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_tls.py tests/test_gpu_tls_ws_chain.py tests/test_gpu_batcher_tls.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for spec in aes:64:256 aes:16:1024 aes:4:4096 aes:4:16384 chacha:64:256; do
  IFS=: read c recs plen <<< "$spec"
  timeout -k 10 200 python tools/bench_tls.py --cipher $c --records $recs --plen $plen --steps 10 --warmup 2 --no-cpu-baseline \
    > $O/$c.$plen.json 2> $O/$c.$plen.err || { echo "fail $c $plen"; tail -5 $O/$c.$plen.err; exit 1; }
  python3 -c "
import json
a=json.load(open('$O/$c.$plen.json'))
print('$c', '$plen', a['value'], a['kernel']['avg_us'], a['kernel']['plaintext_gbs'])"
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof256 -o run -- python3 tools/bench_tls.py --cipher aes --records 64 --plen 256 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof256.out 2>&1 || { echo "prof failed"; tail -5 $O/prof256.out; exit 1; }
find $O/prof256 -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -20
