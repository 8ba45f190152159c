#!/bin/bash
# Every (config, mode) pair of bench.py on one GPU, one JSON line each (no CPU baseline).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bench_matrix_${TAG:-r01}.jsonl
: > "$OUT"
for cfg in c3 c2 c4; do
  for mm in ${MODES:-inplace inplace:nd compact compact:nd streams build build_masked}; do
    IFS=: read mode nd <<< "$mm"
    timeout -k 10 300 python bench.py --config $cfg --mode $mode ${nd:+--no-desc} --steps ${STEPS:-100} --warmup 10 \
      --no-cpu-baseline >> "$OUT" 2>> gpurun_out/bench_matrix.err || { echo "fail $cfg $mode"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    r = d["roofline"]
    print(f'{d["config"]["workload"][:3]} {d["config"]["mode"]:21s} {d["value"]:9.1f} GiB/s  '
          f'{d["ms_per_step"]:8.3f} ms/step  kernel {r["avg_kernel_us"]:8.1f} us  '
          f'{r["achieved"]:7.1f} GB/s ({100*r["frac"]:.1f}%)')
PY
