#!/bin/bash
# AES-GCM A/B round 2 (T-table copies x waves per workgroup, round-key stride, red8) at 16 KiB
# and 256-B records, then SQ LDS counters for the old and the new layout (16 KiB and 256 B).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03p15
for lib in tools/bin/libws_*.so; do
  n=$(basename $lib .so)
  timeout -k 10 200 python tools/bench_tls.py --lib "$lib" --cipher aes --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r03p15/$n.16k.json 2> gpurun_out/r03p15/$n.16k.err || { echo "fail $n"; tail -5 gpurun_out/r03p15/$n.16k.err; exit 1; }
  timeout -k 10 200 python tools/bench_tls.py --lib "$lib" --cipher aes --records 64 --plen 256 --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r03p15/$n.256.json 2> gpurun_out/r03p15/$n.256.err || { echo "fail256 $n"; tail -5 gpurun_out/r03p15/$n.256.err; exit 1; }
  python3 -c "
import json,sys
a=json.load(open('gpurun_out/r03p15/$n.16k.json')); b=json.load(open('gpurun_out/r03p15/$n.256.json'))
print('$n', '16k', a['value'], a['kernel']['avg_us'], a['kernel']['plaintext_gbs'], '256', b['value'], b['kernel']['avg_us'], b['kernel']['plaintext_gbs'])"
done
export SQ_COUNTERS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES"
for n in old base c64w16; do
  TAG=r03p15_${n}_16k tools/pmc_sq.sh python3 $PWD/tools/bench_tls.py --lib $PWD/tools/bin/libws_$n.so --cipher aes --steps 3 --warmup 1 --no-cpu-baseline > /dev/null || exit 1
  TAG=r03p15_${n}_256 tools/pmc_sq.sh python3 $PWD/tools/bench_tls.py --lib $PWD/tools/bin/libws_$n.so --cipher aes --records 64 --plen 256 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null || exit 1
done
grep -h "k_tls_open" gpurun_out/pmc_sq_r03p15_*/summary.txt
