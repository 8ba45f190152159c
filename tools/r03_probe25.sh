#!/bin/bash
# Round-3 probe 25 (re-run after a container reset lost r03p1/r03p4's raw output):
#  1. C4 in place (fused stride path): kernel trace + two SQ counter passes + FETCH/WRITE per
#     kernel, k_plan included
#  2. the stream-decode launch gap: C2 streams 4x standalone, the full
#     all-mode matrix, and one kernel + HIP runtime trace of C2 streams
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p25
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$ROOT/bench.py --config c4 --mode inplace --no-cpu-baseline --no-c5-base --no-ceiling"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4trace" -o run \
  -- python3 $B --steps 20 --warmup 5 > "$OUT/c4_trace.json" 2> "$OUT/c4_trace.err" || { echo "c4 trace failed"; exit 1; }
cd "$ROOT"
TAG=r03p25_sq1 SQ_COUNTERS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
  tools/pmc_sq.sh python3 $B --steps 3 --warmup 1 || { echo "sq1 failed"; exit 1; }
TAG=r03p25_sq2 SQ_COUNTERS="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
  tools/pmc_sq.sh python3 $B --steps 3 --warmup 1 || { echo "sq2 failed"; exit 1; }
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 $B --steps 3 --warmup 1 > /dev/null 2> "$OUT/fetch.err" || { echo "fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 $B --steps 3 --warmup 1 > /dev/null 2> "$OUT/write.err" || { echo "write failed"; exit 1; }
cd "$ROOT"
python3 - "$OUT" > "$OUT/c4_kernels.txt" <<'PY'
import csv, glob, sys, collections
for kind in ("fetch", "write"):
    fs = glob.glob(sys.argv[1] + f"/{kind}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
        agg[k].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(kind, k, "per launch KiB median", sorted(v)[len(v) // 2], "n", len(v))
f = glob.glob(sys.argv[1] + "/c4trace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f'{n[:50]:50s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.2f} us')
PY
cat "$OUT/c4_kernels.txt"
for k in 1 2 3 4; do
  timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 \
    --no-cpu-baseline --no-c5-base --no-ceiling >> "$OUT/c2_streams_repeat.jsonl" 2>> "$OUT/c2s.err" || { echo "c2 streams failed"; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/c2_streams_repeat.jsonl'):
    d = json.loads(l); print('c2 streams', d['value'], d['ms_per_step'], d['host_issue_us_per_step'])"
TAG=r03p25 STEPS=100 timeout -k 10 900 tools/bench_matrix.sh > "$OUT/matrix.txt" 2>&1 || { echo "matrix failed"; tail -5 "$OUT/matrix.txt"; exit 1; }
cp gpurun_out/bench_matrix_r03p25.jsonl "$OUT/"
cat "$OUT/matrix.txt"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/c2s_trace" -o run \
  -- python3 "$ROOT/bench.py" --config c2 --mode streams --steps 30 --warmup 5 --no-cpu-baseline --no-c5-base --no-ceiling \
  > "$OUT/c2s_trace.json" 2> "$OUT/c2s_trace.err" || { echo "c2s trace failed"; exit 1; }
echo done
