#!/bin/bash
# pipeline depth vs upload look-ahead (UVHTTP_WS_PIPE_AHEAD) and copy engine (HSA_ENABLE_SDMA)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 120 python3 tools/pipeline_trace.py $D 2048 1 2>/dev/null | sed "s/}$/, \"env\": \"$*\"}/" >> gpurun_out/${T}_pipe.jsonl || exit 1; }
for D in 3 4 8; do D=$D run X=0; D=$D run UVHTTP_WS_PIPE_AHEAD=2; D=$D run UVHTTP_WS_PIPE_AHEAD=1; done
D=4 run HSA_ENABLE_SDMA=0; D=3 run HSA_ENABLE_SDMA=0
python3 -c "
import json
for l in open('gpurun_out/${T}_pipe.jsonl'):
    d=json.loads(l); print(d['depth'], d['env'], d['value'])"
