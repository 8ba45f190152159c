#!/bin/bash
# PMC evidence, round 5: HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and two SQ counter passes
# for the C4 send side (kb_emit_frames) and the C4 summary-only decodes (in place, compact)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05}
export TAG=$T
SQ2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
for spec in "c4 build build" "c4 inplace inplace_summary_only --no-desc" "c4 compact compact_summary_only --no-desc"; do
  read c m name xa <<< "$spec"
  XARGS="${xa:-}" MNAME=$name tools/profile.sh $c $m || { echo "profile $spec failed"; exit 1; }
  B="python3 $(pwd)/bench.py --config $c --mode $m ${xa:-} --steps 3 --warmup 1 --no-cpu-baseline --no-c5-base --no-ceiling"
  TAG=${T}_${c}_${name}_sq1 tools/pmc_sq.sh $B > /dev/null || { echo "sq1 $spec failed"; exit 1; }
  TAG=${T}_${c}_${name}_sq2 SQ_COUNTERS="$SQ2" tools/pmc_sq.sh $B > /dev/null || { echo "sq2 $spec failed"; exit 1; }
done
ls gpurun_out/evidence/
for f in gpurun_out/evidence/traffic_c4_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', d.get('traffic_over_alg'), d.get('step_traffic_over_alg'), d.get('per_kernel_hbm_bytes'))"; done
grep -h "kb_emit\|k_sum\|k_unmask_stride" gpurun_out/pmc_sq_${T}_*/summary.txt
