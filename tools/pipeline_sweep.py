#!/usr/bin/env python3
"""Host-memory pipeline (uvhttp_ws_gpu_pipeline_*) over slot depth x slot size, after the PCIe
warm-up bench.py --e2e uses: C3 frames (64 KiB), one JSON line per shape.
usage: python tools/pipeline_sweep.py [depths, e.g. 4,3] [slot frames, e.g. 1024,2048]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import uvhttp_amd as U  # noqa: E402


def main():
    warm = bench.e2e_warmup(0)
    print(json.dumps({"warmup_runs": warm}), flush=True)
    n, plen = 65536, 65536
    stride = U.gen_frame_stride(plen)
    depths = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [3, 4]
    sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [512, 1024, 2048, 4096]
    for depth in depths:
        for sf in sizes:
            for rep in range(2):
                r = bench.e2e_rate(n, plen, stride, 0, 0, depth=depth, slot_frames=sf)
                r["rep"] = rep
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
