#!/bin/bash
# Round-4 evidence on one GPU box, in two parts (each fits one gpurun call); every GPU step is
# time-limited and the first failure ends it.
#   PART=a: full GPU suite + smoke + default bench (round_end.sh), the all-mode matrix
#   PART=b: rocprofv3 stats + PMC traffic (C3 / C4 / C2 in place, C4 compact), two SQ counter
#           passes on C4 in place and compact, TLS open benches, the live-shape e2e
# usage: PART=a TAG=r04f tools/evidence_r04.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04f}
export TAG
if [ "${PART:-a}" = a ]; then
  tools/round_end.sh
  tools/bench_matrix.sh
  exit 0
fi
tools/profile.sh c3 inplace
tools/profile.sh c4 inplace
tools/profile.sh c2 inplace
tools/profile.sh c4 compact
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
SQ2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS"
for mode in inplace compact; do
  SQ_COUNTERS="$SQ1" TAG=${TAG}_c4_${mode}_sq1 tools/pmc_sq.sh python3 "$PWD/bench.py" --config c4 --mode $mode \
    --steps 3 --warmup 1 --no-cpu-baseline --no-c5-base --no-ceiling --no-stamps
  SQ_COUNTERS="$SQ2" TAG=${TAG}_c4_${mode}_sq2 tools/pmc_sq.sh python3 "$PWD/bench.py" --config c4 --mode $mode \
    --steps 3 --warmup 1 --no-cpu-baseline --no-c5-base --no-ceiling --no-stamps
done
for c in aes chacha; do
  timeout -k 10 300 python tools/bench_tls.py --cipher $c --steps 10 --warmup 2 \
    > gpurun_out/bench_tls_${c}_$TAG.json 2> gpurun_out/bench_tls_${c}_$TAG.err
done
timeout -k 10 600 python bench.py --e2e --steps 5 --warmup 2 --no-cpu-baseline --no-c5-base \
  > gpurun_out/bench_e2e_$TAG.json 2> gpurun_out/bench_e2e_$TAG.err
