#!/bin/bash
# Round-3 probe 33: is C4 compact's slower k_plan (87 vs 61 us, DESIGN §5 open question) the
# Infinity Cache state?  k_plan time in compact and in place (k_plan-first path: FUSED=0), with
# the wire reused every step and with 4 rotating copies (each step's wire cold).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p33
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  cd /tmp
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run \
    -- python3 "$ROOT/bench.py" --config c4 --steps 40 --warmup 8 --no-cpu-baseline --no-c5-base --no-ceiling $ARGS \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "$tag failed"; return 1; }
  cd "$ROOT"
  python3 - "$OUT/$tag" "$OUT/$tag.json" "$tag" <<'PY'
import csv, glob, sys, json
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
d = json.load(open(sys.argv[2]))
ks = {r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0][-20:]: float(r["AverageNs"]) / 1e3
      for r in csv.DictReader(open(f))}
print(sys.argv[3], d["value"], d["ms_per_step"], " ".join(f"{k}={v:.1f}" for k, v in ks.items() if not k.startswith("__") and "gen" not in k and "elementwise" not in k))
PY
}
ARGS="--mode compact" run compact_warm X=1 || exit 1
ARGS="--mode compact --rotate 4" run compact_cold X=1 || exit 1
ARGS="--mode inplace" run inplace_planfirst_warm UVHTTP_WS_FUSED=0 || exit 1
ARGS="--mode inplace --rotate 4" run inplace_planfirst_cold UVHTTP_WS_FUSED=0 || exit 1
ARGS="--mode inplace" run inplace_fused_warm X=1 || exit 1
ARGS="--mode inplace --rotate 4" run inplace_fused_cold X=1 || exit 1
