#!/usr/bin/env python3
"""End-to-end (host memory -> H2D -> decode -> D2H) rate of the pipeline for several slot
counts / sizes (C3 frames).  PCIe-bound; DESIGN.md records the best."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

n, plen = 65536, 65536
stride = 10 + 4 + plen
for depth, sf in [(3, 1024), (4, 1024), (4, 256), (6, 512), (8, 256), (3, 4096)]:
    r = bench.e2e_rate(n, plen, stride, 64 << 20, 0, depth=depth, slot_frames=sf)
    print(depth, sf, r["value"], "GiB/s", flush=True)
