set -o pipefail
cp uvhttp_amd/lib/libuvhttp_ws_amd.so /tmp/new.so
cp tools/bin/libws_base.so uvhttp_amd/lib/libuvhttp_ws_amd.so
tools/r04_bench_quick.sh r04_streams_old.jsonl c3:streams c2:streams c4:streams > gpurun_out/r04_streams_old.txt 2>&1
cp /tmp/new.so uvhttp_amd/lib/libuvhttp_ws_amd.so
tools/r04_bench_quick.sh r04_streams_new.jsonl c3:streams c2:streams c4:streams > gpurun_out/r04_streams_new.txt 2>&1
cp tools/bin/libws_base.so uvhttp_amd/lib/libuvhttp_ws_amd.so
tools/r04_bench_quick.sh r04_streams_old2.jsonl c3:streams > gpurun_out/r04_streams_old2.txt 2>&1
cp /tmp/new.so uvhttp_amd/lib/libuvhttp_ws_amd.so
tools/r04_bench_quick.sh r04_streams_new2.jsonl c3:streams > gpurun_out/r04_streams_new2.txt 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_streams_full.py > gpurun_out/r04_streams_tests.txt 2>&1
