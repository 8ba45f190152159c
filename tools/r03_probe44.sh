#!/bin/bash
# Round-3 probe 44: host copy rate and live-shape e2e by NUMA node of the loop thread (taskset),
# with the GPU's NUMA node from sysfs
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p44
mkdir -p $OUT
for f in /sys/class/drm/card*/device/numa_node; do echo "$f $(cat $f)"; done 2>/dev/null | tee $OUT/gpu_numa.txt
grep -h "numa_node\|simd_count" /sys/class/kfd/kfd/topology/nodes/*/properties 2>/dev/null | paste - - | head -4
N0=$(lscpu | grep "NUMA node0 CPU" | awk '{print $NF}' | cut -d, -f1)
N1=$(lscpu | grep "NUMA node1 CPU" | awk '{print $NF}' | cut -d, -f1)
echo "node0 $N0 node1 $N1"
for node in 0 1; do
  C=$([ $node = 0 ] && echo $N0 || echo $N1)
  timeout -k 10 120 taskset -c $C tools/bin/copy_probe 1 | head -2 | sed "s/^/node$node /" | tee -a $OUT/copy.txt
  for a in 1 0; do
    timeout -k 10 120 taskset -c $C tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async $a > $OUT/e2e_n${node}_a$a.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$OUT/e2e_n${node}_a$a.json'));print('node$node async=$a', d['value'], d['ms_per_flush'], d['device_flushes'], d['per_flush_ms']['copy'], d['blocked_ms_per_flush'])" | tee -a $OUT/e2e.txt
  done
done
