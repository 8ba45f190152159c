#!/bin/bash
# non-temporal header loads in the wave walk (UVHTTP_WS_WALK_NT_LOAD=1): same-process A/B,
# bench lines with the device timeline, and the PMC traffic with the switch on
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
{
AB_ENV_B=UVHTTP_WS_WALK_NT_LOAD=1 timeout -k 10 300 python -u tools/ab_lib.py tree tree c4:streams || exit 1
AB_ENV_B=UVHTTP_WS_WALK_NT_LOAD=1 timeout -k 10 300 python -u tools/ab_lib.py tree tree c4:streams || exit 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab.txt
: > gpurun_out/${T}_bench.jsonl
for nt in 1 0 1 0; do
  UVHTTP_WS_WALK_NT_LOAD=$nt timeout -k 10 300 python -u bench.py --config c4 --mode streams --steps 200 --warmup 20 \
    --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
done
python3 - gpurun_out/${T}_bench.jsonl <<'PY'
import json, sys
for i, line in enumerate(open(sys.argv[1])):
    d = json.loads(line)
    t = d.get("device_timeline") or {}
    print("nt" if i % 2 == 0 else "wb", d["value"], d["ms_per_step"], t.get("kernels_us"))
PY
UVHTTP_WS_WALK_NT_LOAD=1 TAG=$T MNAME=streams_ntload timeout -k 10 900 tools/profile.sh c4 streams > gpurun_out/${T}_prof.txt 2>&1 || { tail -20 gpurun_out/${T}_prof.txt; exit 1; }
tail -1 gpurun_out/${T}_prof.txt | cut -c1-700
