#!/usr/bin/env python3
"""Interleaved A/B of send-side framing (uvhttp_ws_gpu_build_frames) across builds of the
library in ONE process: python tools/ab_build.py CFG LIB [LIB ...]   (CFG: c2 | c3 | c4)
Prints, per build, the median kb_emit time (engine timing) and whole-call time."""
import os
import statistics
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402

CFG = {"c2": (65536, 4096), "c3": (65536, 65536), "c4": (1048576, 256),
       "c1k": (262144, 1024), "c2k": (131072, 2048), "c64": (4194304, 64),
       # mixed sizes (payloads 100-412 bytes, seeded): the frame-grouped kernel's LDS-window path
       "mix": (1048576, 256)}


def main():
    n, plen = CFG[sys.argv[1]]
    libs = sys.argv[2:]
    engs = [U.GpuEngine(0, library=U.load_library(p if p != "tree" else U.LIB_PATH)) for p in libs]
    # uvhttp_ws_build_desc_t (include/uvhttp_ws_amd.h), server frames as bench.py --mode build
    fr = np.zeros(n, dtype=[("po", "<u8"), ("pl", "<u8"), ("key", "<u4"), ("op", "u1"),
                            ("fin", "u1"), ("mask", "u1"), ("r0", "u1"), ("r1", "<u8")])
    fr["po"] = np.arange(n, dtype=np.uint64) * plen
    fr["pl"] = plen
    if sys.argv[1] == "mix":
        fr["pl"] = np.random.default_rng(7).integers(100, 413, n, dtype=np.uint64)
    src_len = n * plen + 64
    if os.environ.get("AB_ALIGN"):  # experiment: payload sources at the output's 16-byte phase
        hm = (2 if plen < 126 else 4 if plen < 65536 else 10) + (4 if os.environ.get("AB_MASKED") == "1" else 0)
        st = np.arange(n, dtype=np.uint64) * np.uint64(plen + hm)
        fr["po"] = np.arange(n, dtype=np.uint64) * np.uint64(plen + 16) + (st + np.uint64(hm)) % np.uint64(16)
        src_len = n * (plen + 16) + 64
    fr["key"] = np.arange(n, dtype=np.uint32) * 2654435761
    fr["op"], fr["fin"] = 2, 1
    fr["mask"] = int(os.environ.get("AB_MASKED", "0"))
    dev = "cuda"
    d = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
    src = torch.randint(0, 256, (src_len,), dtype=torch.uint8, device=dev)
    outs = [torch.zeros(n * (plen + 14) + 64, dtype=torch.uint8, device=dev) for _ in engs]
    offs = [torch.zeros(n + 1, dtype=torch.int64, device=dev) for _ in engs]
    st = torch.cuda.current_stream()
    K, R = 20, 7
    step = [[] for _ in engs]
    kern = [[] for _ in engs]
    for r in range(R):
        for k, e in enumerate(engs):
            for _ in range(3):
                e.build_frames(src, d, n, outs[k], out_off=offs[k], stream=st)
            e.set_timing(True)
            e.kernel_time()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(K):
                e.build_frames(src, d, n, outs[k], out_off=offs[k], stream=st)
            b.record(st)
            b.synchronize()
            e.set_timing(False)
            ms, cnt = e.kernel_time()
            if r:
                step[k].append(a.elapsed_time(b) / K)
                kern[k].append(ms / max(cnt, 1))
    ref = outs[0]
    for k, p in enumerate(libs):
        same = bool(torch.equal(outs[k], ref)) and bool(torch.equal(offs[k], offs[0]))
        print(f"{sys.argv[1]} {os.path.basename(p):24s} step {statistics.median(step[k]) * 1e3:8.1f} us  "
              f"kb_emit {statistics.median(kern[k]) * 1e3:8.1f} us  same_as_first={same}", flush=True)


if __name__ == "__main__":
    main()
