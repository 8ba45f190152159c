#!/bin/bash
# Round-3 evidence run: full GPU suite, smoke, default bench, payload-kernel traffic (C3 / C4 /
# C2 in place), --rotate 4 for C2 / C4, SQ LDS counters of the shipped TLS AES kernels.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p21
mkdir -p $O
PYARGS="-m gpu" tools/gpu_tests.sh r03p21/full_pytest.log tests/ || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
for cfg in c4 c3 c2; do
  TAG=r03 tools/profile.sh $cfg inplace > $O/profile_$cfg.log 2>&1 || { echo "profile $cfg failed"; tail -5 $O/profile_$cfg.log; exit 1; }
  tail -1 $O/profile_$cfg.log
done
for cfg in c4 c2; do
  timeout -k 10 300 python bench.py --config $cfg --rotate 4 --no-cpu-baseline --no-c5-base --steps 50 > $O/bench_${cfg}_rot4.json 2> $O/bench_${cfg}_rot4.err || { echo "rotate $cfg failed"; exit 1; }
  cat $O/bench_${cfg}_rot4.json
done
export SQ_COUNTERS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES"
TAG=r03p21_final_16k tools/pmc_sq.sh python3 $PWD/tools/bench_tls.py --cipher aes --steps 3 --warmup 1 --no-cpu-baseline > /dev/null || exit 1
TAG=r03p21_final_256 tools/pmc_sq.sh python3 $PWD/tools/bench_tls.py --cipher aes --records 64 --plen 256 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null || exit 1
grep -h "k_tls_open" gpurun_out/pmc_sq_r03p21_final_*/summary.txt
