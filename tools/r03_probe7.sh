#!/bin/bash
# Round-3 probe 7: 1024-thread k_plan on records (parity + C4 A/B) and the TLS -> WS chain.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p7
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_engine.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for w in 1 0 1 0; do
  UVHTTP_WS_PLAN_WIDE=$w timeout -k 10 200 python bench.py --config c4 --steps 200 --warmup 10 --no-cpu-baseline \
    --no-c5-base --no-ceiling > $OUT/bench_c4_wide$w.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench_c4_wide$w.json'));r=d['roofline'];print('c4 wide=$w', d['value'], d['ms_per_step'], r['avg_kernel_us'])"
done
timeout -k 10 300 python -u tools/fused_sweep.py 120,250,500,1000,2000,3000,4000 > $OUT/fused_sweep.txt 2>&1 || { cat $OUT/fused_sweep.txt; exit 1; }
cat $OUT/fused_sweep.txt
for args in "--plen 16384 --records 4" "--plen 1024 --records 64" "--plen 16384 --records 4 --cipher chacha" "--plen 1024 --records 64 --cipher chacha"; do
  timeout -k 10 200 python tools/bench_tls.py --chain --conns 16384 $args --steps 10 > $OUT/tls_chain.tmp 2>>$OUT/tls.err || { tail -5 $OUT/tls.err; exit 1; }
  cat $OUT/tls_chain.tmp >> $OUT/tls_chain.jsonl
  python3 -c "import json;d=json.loads(open('$OUT/tls_chain.tmp').read());print('chain $args', d['value'], d['ms_per_step'], d['kernel']['avg_us'])"
done
