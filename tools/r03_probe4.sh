#!/bin/bash
# Round-3 probe 4: where the fused C4 step goes (kernel trace + k_plan counters on records).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p4
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$ROOT/bench.py --config c4 --mode inplace --no-cpu-baseline --no-c5-base --no-ceiling"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 $B --steps 20 --warmup 5 > "$OUT/c4_trace.json" 2> "$OUT/c4_trace.err" || exit 1
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/trace/*kernel_trace.csv")[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
prev = None; gaps = collections.defaultdict(list); dur = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:34]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[n].append((e - s) / 1e3)
    if prev: gaps[(prev[0], n)].append((s - prev[1]) / 1e3)
    prev = (n, e)
for k, v in dur.items():
    v.sort(); print(f"{k:36s} n={len(v):3d} median {v[len(v)//2]:8.2f} us")
for k, v in gaps.items():
    if len(v) > 3:
        v.sort(); print("gap", k, f"median {v[len(v)//2]:.2f} us")
PY
TAG=r03p4_sq1 SQ_COUNTERS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
  tools/pmc_sq.sh python3 $B --steps 3 --warmup 1 || exit 1
TAG=r03p4_sq2 SQ_COUNTERS="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
  tools/pmc_sq.sh python3 $B --steps 3 --warmup 1 || exit 1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 $B --steps 3 --warmup 1 > /dev/null 2> "$OUT/fetch.err" || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 $B --steps 3 --warmup 1 > /dev/null 2> "$OUT/write.err" || exit 1
cd "$ROOT"
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
PY
for fpt in 4 8 16; do
  UVHTTP_WS_PLAN_FPT=$fpt timeout -k 10 100 python3 bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/c4_fpt$fpt.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c4_fpt$fpt.json'));print('fpt $fpt', d['value'], d['ms_per_step'])"
done
UVHTTP_WS_PLAN_TICKET=0 timeout -k 10 100 python3 bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/c4_noticket.json || exit 1
python3 -c "import json;d=json.load(open('$OUT/c4_noticket.json'));print('noticket', d['value'], d['ms_per_step'])"
