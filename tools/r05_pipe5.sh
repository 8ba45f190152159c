#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 120 python3 tools/pipeline_trace.py $D 2048 1 2>/dev/null | sed "s/}$/, \"env\": \"$*\"}/" >> gpurun_out/${T}_pipe.jsonl || exit 1; }
for D in 3 4 8; do D=$D run UVHTTP_WS_PIPE_IN_FLIGHT=0; D=$D run UVHTTP_WS_PIPE_IN_FLIGHT=3; D=$D run UVHTTP_WS_PIPE_IN_FLIGHT=2; done
python3 -c "
import json
for l in open('gpurun_out/${T}_pipe.jsonl'):
    d=json.loads(l); print(d['depth'], d['env'], d['value'])"
