#!/usr/bin/env python3
"""Interleaved A/B of payload-kernel tile shapes (engine.set_tile) on one device, per config.
Reports the median payload-kernel time and achieved algorithmic GB/s for each shape."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402

SHAPES = [(64, 1), (64, 2), (64, 4), (128, 1), (128, 2), (256, 1), (256, 2), (256, 4)]
CFG = {"c2": (65536, 4096, False), "c3": (65536, 65536, False), "c4": (1048576, 256, True)}


def main():
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c3", "c2", "c4"]
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["inplace", "compact"]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    eng = U.GpuEngine(0)
    st = torch.cuda.current_stream()
    for c in cfgs:
        n, plen, frag = CFG[c]
        stride = U.gen_frame_stride(plen)
        wl = stride * n
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        eng.gen_frames(wire, n, plen, 7, opcode0=2, fragmented=frag)
        desc, summ = eng.alloc_outputs(n)
        arena = torch.empty(n * plen + 64, dtype=torch.uint8, device="cuda")
        msgs = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        mm = 256 << 20
        alg = n * (stride + plen)
        for mode in modes:
            res = {s: [] for s in SHAPES}
            for r in range(rounds):
                for s in SHAPES:
                    eng.set_tile(*s)
                    eng.set_timing(r > 0)
                    for _ in range(3):
                        if mode == "inplace":
                            eng.decode_inplace(wire, n, stride=stride, max_message_size=mm,
                                               wire_len=wl, desc=desc, summary=summ, stream=st)
                        else:
                            eng.decode_compact(wire, n, arena, stride=stride, max_message_size=mm,
                                               wire_len=wl, desc=desc, msgs=msgs, summary=summ,
                                               stream=st)
                    eng.set_timing(False)
                    ms, k = eng.kernel_time()
                    if k:
                        res[s].append(ms / k)
            torch.cuda.synchronize()
            sm = eng.read_summary(summ)
            assert sm["n_delivered"] == n and sm["status"] == 0, sm
            for s in SHAPES:
                med = statistics.median(res[s])
                print(f"{c} {mode:8s} block {s[0]:4d} vpt {s[1]}  {med * 1e3:9.1f} us  "
                      f"{alg / (med * 1e-3) / 1e9:7.1f} GB/s  min {alg / (min(res[s]) * 1e-3) / 1e9:7.1f}",
                      flush=True)
        del wire, arena, msgs, desc, summ
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
