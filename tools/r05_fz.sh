set -uo pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_stamps.py tests/test_gpu_engine.py tests/test_gpu_streams_full.py > gpurun_out/r05fz_tests.log 2>&1 || { tail -30 gpurun_out/r05fz_tests.log; exit 1; }
tail -1 gpurun_out/r05fz_tests.log
bash tools/r05_ab_fuse.sh r05fz2 > /dev/null || exit 1
cat gpurun_out/r05fz2_ab.txt
for c in c4; do timeout -k 10 300 python -u bench.py --config $c --mode streams --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/r05fz_bench.jsonl || exit 1; done
