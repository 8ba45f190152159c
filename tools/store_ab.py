#!/usr/bin/env python3
"""Interleaved A/B of the payload store policy (UVHTTP_WS_STORE_POLICY 0 = global nt store,
18 = buffer store sc1|nt) on the real in-place kernel, per config, one process."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402

CFG = {"c2": (65536, 4096, False), "c3": (65536, 65536, False), "c4": (1048576, 256, True)}


def main():
    engines = {}
    for pol in ("0", "18"):
        os.environ["UVHTTP_WS_STORE_POLICY"] = pol
        engines[pol] = U.GpuEngine(0)
    st = torch.cuda.current_stream()
    for c in sys.argv[1].split(",") if len(sys.argv) > 1 else ["c3", "c2", "c4"]:
        n, plen, frag = CFG[c]
        stride = U.gen_frame_stride(plen)
        wl = stride * n
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        engines["0"].gen_frames(wire, n, plen, 3, opcode0=2, fragmented=frag)
        alg = n * (stride + plen)
        res = {p: [] for p in engines}
        outs = {p: engines[p].alloc_outputs(n) for p in engines}
        for r in range(9):
            for p, e in engines.items():
                e.set_timing(r > 0)
                for _ in range(5):
                    e.decode_inplace(wire, n, stride=stride, max_message_size=256 << 20,
                                     wire_len=wl, desc=outs[p][0], summary=outs[p][1], stream=st)
                e.set_timing(False)
                ms, k = e.kernel_time()
                if k:
                    res[p].append(ms / k)
        for p in engines:
            med = statistics.median(res[p])
            print(f"{c} store_policy {p:>2s}: {med * 1e3:9.1f} us  {alg / (med * 1e-3) / 1e9:7.1f} GB/s",
                  flush=True)
        del wire
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
