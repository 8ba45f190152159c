#!/bin/bash
# Cold-HBM refresh on the final tree: --rotate 4 (four wire copies, > 256 MB Infinity Cache)
# against the warm run, in place, C4 / C2 / C3, interleaved, two rounds each.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p55
mkdir -p $O
: > $O/rotate.jsonl
for rep in 1 2; do
  for cfg in c4 c2 c3; do
    for rot in 1 4; do
      timeout -k 10 300 python bench.py --config $cfg --rotate $rot --no-cpu-baseline --no-c5-base --steps 50 > $O/b.json 2> $O/b.err || { echo "bench $cfg rot $rot failed"; tail -5 $O/b.err; exit 1; }
      python -c "import json,sys; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); d['rotate']=$rot; d['rep']=$rep; print(json.dumps(d))" >> $O/rotate.jsonl
      tail -1 $O/rotate.jsonl | cut -c1-160
    done
  done
done
