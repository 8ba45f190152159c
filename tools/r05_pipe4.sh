#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
for D in 3 4 8; do for F in 256 512 1024 4096; do
  timeout -k 10 120 python3 tools/pipeline_trace.py $D $F 1 2>/dev/null >> gpurun_out/${T}_pipe.jsonl || exit 1
done; done
python3 -c "
import json
for l in open('gpurun_out/${T}_pipe.jsonl'):
    d=json.loads(l); print(d['depth'], d['slot_frames'], round(d['slot_frames']*65550/2**20), 'MiB/slot', d['value'])"
