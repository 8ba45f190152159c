#!/bin/bash
# Round-3 probe 1: k_plan counters on C4 in place (kernel-trace stats, FETCH/WRITE, two SQ
# passes) and the C2 stream-decode host/launch gap (4 repeated runs + a runtime trace).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p1
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$ROOT/bench.py --config c4 --mode inplace --no-cpu-baseline --no-c5-base"
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1 || true
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 $B --steps 20 --warmup 5 > "$OUT/c4_trace.json" 2> "$OUT/c4_trace.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 $B --steps 3 --warmup 1 > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 $B --steps 3 --warmup 1 > /dev/null 2> "$OUT/write.err"
cd "$ROOT"
TAG=r03p1_sq1 SQ_COUNTERS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
  tools/pmc_sq.sh python3 $B --steps 3 --warmup 1
TAG=r03p1_sq2 SQ_COUNTERS="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" \
  tools/pmc_sq.sh python3 $B --steps 3 --warmup 1 || echo "sq2 failed"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
for kind in ("fetch", "write"):
    fs = glob.glob(sys.argv[1] + f"/{kind}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
        agg[k].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(kind, k, "per launch KiB median", sorted(v)[len(v) // 2], "n", len(v))
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f'{n[:50]:50s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.2f} us')
PY
# C2 streams, repeated (the launch-gap observation), then one runtime trace
for k in 1 2 3 4; do
  timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 \
    --no-cpu-baseline >> "$OUT/c2_streams_repeat.jsonl"
done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/c2s_trace" -o run \
  -- python3 "$ROOT/bench.py" --config c2 --mode streams --steps 30 --warmup 5 --no-cpu-baseline \
  > "$OUT/c2s_trace.json" 2> "$OUT/c2s_trace.err"
echo done
