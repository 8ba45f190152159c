#!/bin/bash
# Round-3 probe 47: async batcher staging capacity 1.0 vs 1.4 rounds (pinned loop, AVX2 copies)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p47
mkdir -p $OUT
timeout -k 10 60 tools/bin/pcie_probe 256 1 | tee $OUT/pcie.jsonl
for r in 1 2; do
  for cfg in "1 1.0" "1 1.4" "0 1.0"; do
    set -- $cfg
    timeout -k 10 120 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async $1 --pin 1 --cap $2 > $OUT/e.json 2>/dev/null || exit 1
    cat $OUT/e.json >> $OUT/e2e.jsonl
    python3 -c "import json;d=json.load(open('$OUT/e.json'));print('async=$1 cap=$2', d['value'], d['ms_per_flush'], d['device_flushes'], d['per_flush_ms']['copy'], d['blocked_ms_per_flush'], d['max_blocked_ms'], 'host', d['host_flushes'], 'fallback', d['fallback_flushes'], 'cap', d['capacity_flushes'], 'err', d['device_errors'])"
  done
done
