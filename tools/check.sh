#!/bin/bash
# The GPU-box driver: every check and measurement of the rounds, as named steps.  Logs and lines
# land under gpurun_out/${TAG}_*; what is cited gets copied into profiles/ (named per round).
#
#   TAG=r06z tools/check.sh STEP [STEP ...]        ("all" = tests smoke bench matrix)
#
#   tests      the whole pytest -m gpu suite (one process, every test bounded)
#   suite      a test subset: SUITE="tests/test_gpu_x.py tests/test_gpu_y.py"
#   smoke      __graft_entry__.smoke()
#   bench      the default bench.py line (C3 in place, with the CPU baseline)
#   matrix     tools/bench_matrix.sh (every config x mode)
#   lines      one bench line per LINES entry cfg:mode[:nd] (nd = --no-desc), no CPU baseline,
#              printed with the device timeline (BARGS: more bench args, e.g. "--steps 100")
#   c5x2       the 2-rank C5 line on one GPU (--oversubscribe: the N>1 path and its stamp merge)
#   ab         tools/ab_lib.py: library A against B (AB_A / AB_B, default the tree's testhooks build)
#              on ABCFG cfg:mode pairs; AB_ENV_B=K=V or AB_STAMPS=1 switch engine B
#   prof       tools/profile.sh per PROFS cfg:mode (rocprofv3 stats, FETCH_SIZE / WRITE_SIZE passes,
#              HBM bytes per launch -> gpurun_out/evidence/); XARGS / MNAME pass through
#   sq         tools/pmc_sq.sh: SQ counter passes over PROFS (SQ_COUNTERS picks the set)
#   abbuild    tools/ab_build.py: the send side against AB_B (AB_MASKED=0 and 1)
#   walkcmp    C4 streams: the speculative decode, the wave walk, the lane walk
#   e2e        live-shape harness (tests/c/_build/batcher_e2e) per read model, after a PCIe warm-up
#   pipe       tools/pipeline_trace.py per pipeline depth and in-flight bound
#   stamps     tools/stamp_probe.py (device stamps against HIP events, idle / warm-up rows)
#
# Every GPU step runs under its own timeout and the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-chk}
O=gpurun_out/${TAG}
STEPS=" ${*:-all} "
has() { [[ "$STEPS" == *" $1 "* || ( "$STEPS" == *" all "* && " tests smoke bench matrix " == *" $1 "* ) ]]; }
TH=uvhttp_amd/lib/libuvhttp_ws_amd_testhooks.so
line() {  # one bench JSON line, summarised
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t = d.get('device_timeline') or {}
r = d.get('roofline') or {}
print(sys.argv[2], d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'frac', r.get('frac'), r.get('kernel'),
      'kernels', t.get('kernels_us'), 'gaps', t.get('gaps_us'))" "$1" "$2"
}
if has tests; then
  PYARGS="-m gpu" tools/gpu_tests.sh ${TAG}_pytest_gpu.log tests/
fi
if has suite; then
  tools/gpu_tests.sh ${TAG}_pytest_suite.log ${SUITE:?SUITE=test files}
fi
if has smoke; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${O}_smoke.log 2>&1
  tail -1 ${O}_smoke.log
fi
if has bench; then
  timeout -k 10 600 python -u bench.py > ${O}_bench.json 2> ${O}_bench.err
  cut -c1-600 ${O}_bench.json
fi
if has matrix; then
  TAG=$TAG timeout -k 10 1200 tools/bench_matrix.sh
fi
if has lines; then
  for cm in ${LINES:-c4:inplace c4:compact c4:streams}; do
    IFS=: read c m nd <<< "$cm"
    f=${O}_bench_${c}_${m}${nd:+_nd}.json
    timeout -k 10 300 python -u bench.py --config $c --mode $m ${nd:+--no-desc} --no-cpu-baseline \
      ${BARGS:---steps 20 --warmup 5} > $f 2>> ${O}_bench.err
    line $f "$cm"
  done
fi
if has c5x2; then
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --config c5 --steps 2 --warmup 1 --oversubscribe \
    > ${O}_c5x2.json 2> ${O}_c5x2.err
  cut -c1-600 ${O}_c5x2.json
fi
if has ab; then
  timeout -k 10 600 python -u tools/ab_lib.py ${AB_A:-$TH} ${AB_B:-$TH} ${ABCFG:-c4:inplace} > ${O}_ab.txt 2>&1
  cat ${O}_ab.txt
fi
if has prof; then
  for cm in ${PROFS:-c3:inplace c4:inplace c4:compact c4:streams}; do
    TAG=$TAG tools/profile.sh ${cm%%:*} ${cm##*:}
  done
fi
if has sq; then
  for cm in ${PROFS:-c4:inplace}; do
    B="python3 $(pwd)/bench.py --config ${cm%%:*} --mode ${cm##*:} ${XARGS:-} --steps 3 --warmup 1 --no-cpu-baseline --no-c5-base --no-ceiling"
    TAG=${TAG}_${cm%%:*}_${cm##*:} tools/pmc_sq.sh $B > /dev/null
  done
  cat gpurun_out/pmc_sq_${TAG}_*/summary.txt
fi
if has abbuild; then
  tools/gpu_tests.sh ${TAG}_pytest_build.log tests/test_gpu_build.py
  for m in 0 1; do
    AB_MASKED=$m timeout -k 10 300 python -u tools/ab_build.py c4 tree ${AB_B:?AB_B=library} > ${O}_ab_build_$m.txt 2>&1
    cat ${O}_ab_build_$m.txt
  done
fi
if has walkcmp; then
  for v in "UVHTTP_WS_STREAM_SPEC=1" "UVHTTP_WS_STREAM_SPEC=0" "UVHTTP_WS_STREAM_SPEC=0 UVHTTP_WS_WALK=lane"; do
    env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --config c4 --mode streams --no-cpu-baseline \
      > ${O}_walkcmp.json 2>> ${O}_bench.err
    line ${O}_walkcmp.json "[$v]"
  done
fi
if has e2e; then
  E=tests/c/_build/batcher_e2e
  A="--conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async 1 --cap 0.5 --pin 1"
  for w in 1 2 3 4; do timeout -k 10 120 $E $A > /dev/null; done
  for m in submit kcopy zc; do timeout -k 10 120 $E $A --reads $m >> ${O}_e2e.jsonl; done
  cat ${O}_e2e.jsonl
fi
if has pipe; then
  for D in 3 4 8; do
    for f in 0 2 3; do
      UVHTTP_WS_PIPE_IN_FLIGHT=$f timeout -k 10 120 python3 tools/pipeline_trace.py $D 2048 1 \
        | sed "s/}$/, \"in_flight\": $f}/" >> ${O}_pipe.jsonl
    done
  done
  cat ${O}_pipe.jsonl
fi
if has stamps; then
  timeout -k 10 300 python -u tools/stamp_probe.py ${STAMP_CFGS:-c3 c2} > ${O}_stamp_probe.txt 2>&1
  cat ${O}_stamp_probe.txt
fi
