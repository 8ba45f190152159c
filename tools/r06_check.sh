#!/bin/bash
# Round-6 GPU check: full pytest -m gpu, smoke(), default bench, then the 2-rank C5 line on one GPU
# (the N>1 roofline the round-5 verdict found broken).  Logs under gpurun_out/r06_$TAG*.
# usage: TAG=a tools/r06_check.sh [tests|smoke|bench|c5x2|all ...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-a}
O=gpurun_out/r06${TAG}
STEPS=${*:-all}
has() { [[ " $STEPS " == *" all "* || " $STEPS " == *" $1 "* ]]; }
if has tests; then
  PYARGS="-m gpu" tools/gpu_tests.sh r06${TAG}_pytest_gpu.log tests/
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${O}_smoke.log 2>&1
  tail -1 ${O}_smoke.log
fi
if has bench; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > ${O}_bench.json 2> ${O}_bench.err
  cat ${O}_bench.json
fi
if has c5x2; then
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --config c5 --steps 2 --warmup 1 --oversubscribe \
    > ${O}_c5x2.json 2> ${O}_c5x2.err
  cat ${O}_c5x2.json
fi
if has deliver; then
  tools/gpu_tests.sh r06${TAG}_pytest_deliver.log tests/test_gpu_deliver_messages.py tests/test_gpu_summary_compact.py \
    tests/test_gpu_spec_compact.py tests/test_gpu_parity.py
fi
if has abstamps; then
  AB_STAMPS=1 timeout -k 10 300 python tools/ab_lib.py tree tree c3:inplace c2:inplace > ${O}_ab_stamps.txt 2>&1
  cat ${O}_ab_stamps.txt
fi
if has emit; then
  tools/gpu_tests.sh r06${TAG}_pytest_emit.log tests/test_gpu_desc_emit.py tests/test_gpu_spec_compact.py tests/test_gpu_summary_compact.py tests/test_gpu_deliver_messages.py tests/test_gpu_fused.py tests/test_gpu_stamps.py \
    tests/test_gpu_engine.py tests/test_gpu_parity.py tests/test_gpu_summary_only.py
fi
if has c4; then
  for m in inplace compact; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config c4 --mode $m --no-cpu-baseline \
      > ${O}_bench_c4_$m.json 2>> ${O}_bench.err
    python -c "import json,sys; d=json.load(open('${O}_bench_c4_$m.json')); t=d.get('device_timeline') or {}; print('$m', d['value'], d['ms_per_step'], t.get('kernels_us'), t.get('gaps_us'))"
  done
fi
if has abemit; then
  TH=uvhttp_amd/lib/libuvhttp_ws_amd_testhooks.so
  for B in ${ABEMIT:-0}; do
    AB_ENV_B=UVHTTP_WS_DESC_EMIT=$B timeout -k 10 300 python tools/ab_lib.py $TH $TH ${ABCFG:-c4:inplace f2k:inplace} > ${O}_ab_emit_$B.txt 2>&1
    cat ${O}_ab_emit_$B.txt
  done
fi
if has abfused; then
  TH=uvhttp_amd/lib/libuvhttp_ws_amd_testhooks.so
  AB_ENV_B=UVHTTP_WS_FUSED_MAX=${FMAX:-8192} timeout -k 10 300 python tools/ab_lib.py $TH $TH c2:inplace c2:inplace_nd \
    c2:compact c2:compact_nd > ${O}_ab_fused_max.txt 2>&1
  cat ${O}_ab_fused_max.txt
fi
if has sspec; then
  tools/gpu_tests.sh r06${TAG}_pytest_sspec.log tests/test_gpu_stream_spec.py tests/test_gpu_streams_full.py \
    tests/test_gpu_streams.py tests/test_gpu_batcher.py
fi
if has c4s; then
  for c in c4 c2 c3; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config $c --mode streams --no-cpu-baseline \
      > ${O}_bench_${c}_streams.json 2>> ${O}_bench.err
    python -c "import json,sys; d=json.load(open('${O}_bench_${c}_streams.json')); t=d.get('device_timeline') or {}; print('$c streams', d['value'], d['ms_per_step'], t.get('kernels_us'), t.get('gaps_us'))"
  done
fi
if has build; then
  tools/gpu_tests.sh r06${TAG}_pytest_build.log tests/test_gpu_build.py
  for m in 0 1; do
    AB_MASKED=$m timeout -k 10 300 python tools/ab_build.py c4 tree tools/bin/libws_zeroall.so > ${O}_ab_build_$m.txt 2>&1
    cat ${O}_ab_build_$m.txt
  done
fi
if has walkcmp; then
  for v in "" "UVHTTP_WS_STREAM_SPEC=0" "UVHTTP_WS_STREAM_SPEC=0 UVHTTP_WS_WALK=lane"; do
    env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config c4 --mode streams --no-cpu-baseline \
      > ${O}_walkcmp.json 2>> ${O}_bench.err
    python -c "import json,sys; d=json.load(open('${O}_walkcmp.json')); t=d.get('device_timeline') or {}; print('[$v]', d['value'], d['ms_per_step'], t.get('kernels_us'))"
  done
fi
if has prof; then
  for cm in ${PROFS:-c3:inplace c4:inplace c4:compact c4:streams}; do
    TAG=r06${TAG} tools/profile.sh ${cm%%:*} ${cm##*:}
  done
fi
