#!/bin/bash
# single-pass fused stride path: parity tests, frame-size sweep (single / records / plan-first),
# C4 and C2 bench
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p24
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_known_answers.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/fused_sweep.py 250,1000,3000 3 > $O/sweep.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep.txt; exit 1; }
cat $O/sweep.txt
for cfg in c4 c2; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-c5-base > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo "bench $cfg failed"; tail -5 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['avg_kernel_us'], d['roofline']['kernel'])"
done
