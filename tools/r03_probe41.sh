#!/bin/bash
# Round-3 probe 41: C4 k_plan in compact vs in place (k_plan-first, FUSED=0): SQ counters +
# FETCH/WRITE per kernel, to see what the 91 vs 63 us is (not the cache: r03p33)
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
for mode in compact inplace; do
  B="$ROOT/bench.py --config c4 --mode $mode --no-cpu-baseline --no-c5-base --no-ceiling --steps 3 --warmup 1"
  UVHTTP_WS_FUSED=0 TAG=r03p41_${mode}_sq1 SQ_COUNTERS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
    tools/pmc_sq.sh python3 $B > /dev/null || exit 1
  UVHTTP_WS_FUSED=0 TAG=r03p41_${mode}_sq2 SQ_COUNTERS="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
    tools/pmc_sq.sh python3 $B > /dev/null || exit 1
  grep k_plan gpurun_out/pmc_sq_r03p41_${mode}_sq1/summary.txt gpurun_out/pmc_sq_r03p41_${mode}_sq2/summary.txt
done
