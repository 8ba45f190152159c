#!/bin/bash
# One SQ counter pass (8 slots) over a command's kernels; per-kernel sums of each counter
# -> gpurun_out/pmc_sq_$TAG/summary.txt.   usage: TAG=x tools/pmc_sq.sh python3 tools/bench_tls.py ...
# (counters: wave / instruction / issue-cycle accounting, MI355X_MICROARCH.md § rocprofv3 PMC)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${TAG:-sq}
OUT=$ROOT/gpurun_out/pmc_sq_$TAG
mkdir -p "$OUT"
CTR=${SQ_COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"}
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d "$OUT/raw" -o run -- "$@" > "$OUT/cmd.out" 2> "$OUT/cmd.err"
cd "$ROOT"
python3 - "$OUT" <<'PY' | tee "$OUT/summary.txt"
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/raw/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, c in agg.items():
    n = len(disp[k])
    print(k, f"dispatches={n}", " ".join(f"{a}={v / n:.4g}" for a, v in sorted(c.items())))
PY
