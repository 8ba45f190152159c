#!/usr/bin/env python3
"""One host-memory pipeline run (uvhttp_ws_gpu_pipeline_*) at a given depth after a warm-up of
the same pipeline shape, for a rocprofv3 kernel + memory-copy trace (depth 4
ran at 24-27 GiB/s against 44 at depth 3).
usage: python tools/pipeline_trace.py DEPTH [SLOT_FRAMES] [WARM_RUNS]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import uvhttp_amd as U  # noqa: E402


def main():
    depth = int(sys.argv[1])
    sf = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    n, plen = 65536, 65536
    stride = U.gen_frame_stride(plen)
    for _ in range(warm):  # PCIe warm-up (the link's power state ramps with traffic)
        bench.e2e_rate(n, plen, stride, 0, 0, depth=3, slot_frames=sf)
    r = bench.e2e_rate(n, plen, stride, 0, 0, depth=depth, slot_frames=sf)
    r["depth"] = depth
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
