#!/bin/bash
# round-5 A/B runs (tools/ab_lib.py); usage: tools/r05_ab.sh TAG "LIB_A LIB_B PAIRS [ENV]" ...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  read -r A B P E <<< "$spec"
  echo "== $A vs $B $P ${E:-}" >> gpurun_out/${T}_ab.txt
  env ${E:-} timeout -k 10 300 python -u tools/ab_lib.py $A $B ${P//,/ } >> gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
done
cat gpurun_out/${T}_ab.txt
