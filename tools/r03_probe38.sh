#!/bin/bash
# Round-3 probe 38: k_unmask_stride mask in 32-bit tile-relative arithmetic (no f64 division per
# vector): fused parity, then in-process A/B against the previous build (tools/bin/libws_HEAD.so)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p38
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_known_answers.py tests/test_gpu_batcher.py tests/test_batcher_transitions.py tests/test_gpu_batcher_tls.py tests/test_c1_echo.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/ab_lib.py tools/bin/libws_HEAD.so tree c4:inplace c4:inplace > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
for k in 1 2; do
  timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --no-c5-base > $OUT/b.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('c4', d['value'], d['ms_per_step'], r['avg_kernel_us'], r['copy_ceiling']['avg_us'])"
done
for a in 0 1; do
  timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async $a | tee -a $OUT/e2e.jsonl || exit 1
done
timeout -k 10 120 tools/bin/pcie_probe 256 2 | tee $OUT/pcie.jsonl
