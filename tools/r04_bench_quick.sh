#!/bin/bash
# Quick bench lines for a list of cfg:mode pairs (no CPU baseline), one JSON line each.
# usage: tools/r04_bench_quick.sh OUT cfg:mode [cfg:mode ...]   (extra bench args via BARGS)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
shift
mkdir -p gpurun_out
: > "$OUT"
for pair in "$@"; do
  cfg=${pair%%:*}; mode=${pair##*:}
  timeout -k 10 300 python bench.py --config "$cfg" --mode "$mode" --steps ${STEPS:-100} --warmup 10 \
    --no-cpu-baseline --no-c5-base ${BARGS:-} >> "$OUT" 2>> "$OUT.err" || { echo "fail $pair"; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    r = d["roofline"]
    tl = d.get("device_timeline") or {}
    print(f'{d["config"]["workload"][:3]} {d["config"]["mode"]:8s} {d["value"]:8.1f} GiB/s '
          f'{d["ms_per_step"]*1e3:8.1f} us/step  {r["kernel"]} {r["avg_kernel_us"]} us '
          f'(events {r["event_kernel_us"]}) {100*(r["frac"] or 0):.1f}%  chain {tl.get("chain_us")} '
          f'between {tl.get("gap_between_calls_us")}/{tl.get("gap_between_calls_max_us")} gaps {tl.get("gaps_us")}')
PY
