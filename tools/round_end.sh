#!/bin/bash
# Round-end check on the GPU box: full pytest -m gpu, smoke(), default bench; logs under gpurun_out/.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYARGS="-m gpu" tools/gpu_tests.sh full_pytest.log tests/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
cat gpurun_out/bench_default.json
