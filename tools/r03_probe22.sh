#!/bin/bash
# k_plan block-size / frames-per-lane A/B on the header path (C2, C3 in place): rocprofv3 kernel
# stats per variant (k_plan average) and the bench rate; parity tests under the 64-thread plan.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p22
mkdir -p $O
UVHTTP_WS_PLAN_NT=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_known_answers.py > $O/pytest_nt64.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_nt64.log; exit 1; }
tail -1 $O/pytest_nt64.log
export TMPDIR=/tmp
for cfg in c2 c3; do
  for v in "base" "UVHTTP_WS_PLAN_NT=64" "UVHTTP_WS_PLAN_NT=128" "UVHTTP_WS_PLAN_FPT=2" "UVHTTP_WS_PLAN_FPT=4"; do
    tag=$cfg.$(echo $v | tr '=' '_')
    if [ "$v" = base ]; then ENVV=""; else ENVV="$v"; fi
    env $ENVV timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 $PWD/bench.py --config $cfg --no-cpu-baseline --no-c5-base --no-ceiling --steps 40 > $O/$tag.json 2> $O/$tag.err || { echo "fail $tag"; tail -3 $O/$tag.err; exit 1; }
    python3 - $O/$tag <<'PY'
import csv, glob, json, sys
d = sys.argv[1]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
ks = {r["Name"].split("(")[0].split("::")[-1][:28]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(f))}
b = json.loads(open(d + ".json").read().strip().splitlines()[-1])
print(d.split("/")[-1], b["value"], b["ms_per_step"], {k: round(v, 1) for k, v in ks.items() if "plan" in k or "unmask" in k})
PY
  done
done
