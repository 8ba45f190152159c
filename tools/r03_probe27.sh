#!/bin/bash
# Round-3 probe 27: which kernel makes some C2 stream-decode runs slow?
# 6 standalone runs under a kernel trace, per-run step time + per-kernel medians, then the wave
# walk (UVHTTP_WS_WALK=wave) and C2 in place as controls.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p27
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # tag, env..., then bench args
  local tag=$1; shift
  cd /tmp
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run \
    -- python3 "$ROOT/bench.py" --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-c5-base --no-ceiling \
    $MODEARGS > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "$tag failed"; return 1; }
  cd "$ROOT"
  python3 - "$OUT/$tag" "$OUT/$tag.json" "$tag" <<'PY'
import csv, glob, sys, collections, json
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
d = json.load(open(sys.argv[2]))
dur = collections.defaultdict(list); gap = []
prev = None
for r in rows[-500:]:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0][-18:]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[n].append((e - s) / 1e3)
    if prev is not None: gap.append((s - prev) / 1e3)
    prev = e
med = lambda v: sorted(v)[len(v) // 2]
print(sys.argv[3], d["value"], d["ms_per_step"], "host", d.get("host_issue_us_per_step"),
      " ".join(f"{k}={med(v):.1f}/{max(v):.1f}" for k, v in dur.items()),
      f"gap_med={med(gap):.2f} gap_sum={sum(gap):.0f}us")
PY
}
for k in 1 2 3 4 5 6; do MODEARGS="--mode streams" run s$k X=1 || exit 1; done
for k in 1 2 3; do MODEARGS="--mode streams" run w$k UVHTTP_WS_WALK=wave || exit 1; done
for k in 1 2; do MODEARGS="--mode inplace" run i$k X=1 || exit 1; done
for k in 1 2 3 4; do
  timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/plain$k.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/plain$k.json'));print('plain', d['value'], d['ms_per_step'])"
done
