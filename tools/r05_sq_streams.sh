#!/bin/bash
# SQ counters (two passes) for the C4 stream decode's kernels: how the walk's waves spend cycles
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CMD="python3 $PWD/bench.py --config c4 --mode streams --steps 3 --warmup 1 --no-cpu-baseline --no-c5-base --no-ceiling"
TAG=r05sq_c4_streams_1 tools/pmc_sq.sh $CMD > /dev/null || exit 1
SQ_COUNTERS="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
  TAG=r05sq_c4_streams_2 tools/pmc_sq.sh $CMD > /dev/null || exit 1
cat gpurun_out/pmc_sq_r05sq_c4_streams_1/summary.txt gpurun_out/pmc_sq_r05sq_c4_streams_2/summary.txt
