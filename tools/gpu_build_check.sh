#!/bin/bash
# Build-path check on one GPU: parity tests, then every config x client/server frames, and
# the small-frame emit shapes (UVHTTP_WS_BUILD_SMALL) on C4.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_build.py > gpurun_out/t_build.log 2>&1 || { tail -30 gpurun_out/t_build.log; exit 1; }
tail -2 gpurun_out/t_build.log
one() {
timeout -k 10 200 python bench.py --config $1 --mode $2 --steps 50 --warmup 5 --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'][:3], d['config']['mode'], '${UVHTTP_WS_BUILD_SMALL:-}', d['value'], r['avg_kernel_us'], r['achieved'], r['frac'])"
}
for c in c3 c2 c4; do for m in build build_masked; do one $c $m; done; done
for k in 1 2 3; do UVHTTP_WS_BUILD_SMALL=$k one c4 build; done
