#!/usr/bin/env python3
"""Fused stride path vs k_plan-first path (UVHTTP_WS_FUSED=0), interleaved in one process,
over frame sizes: the whole in-place decode step (torch events around K steps) per size.
Sets the automatic choice in run_decode (kFusedMaxAvg); FUSED_TILES=BxV,... adds fused
engines with those payload tiles (UVHTTP_WS_FUSED_TILE).

  python tools/fused_sweep.py [plen,plen,...] [rounds]
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402


def engine(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return U.GpuEngine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    plens = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
        [50, 120, 250, 500, 1000, 2000, 4000, 8000, 16000]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    K = 20
    engs = {"fused": engine({"UVHTTP_WS_FUSED": "1", "UVHTTP_WS_FUSED_MAX": "1099511627776"})}
    # FUSED_TILES=256x4,512x4: the fused path with those payload tiles too (UVHTTP_WS_FUSED_TILE)
    for t in filter(None, os.environ.get("FUSED_TILES", "").split(",")):
        engs["fused_" + t] = engine({"UVHTTP_WS_FUSED": "1", "UVHTTP_WS_FUSED_MAX": "1099511627776",
                                     "UVHTTP_WS_FUSED_TILE": t})
    engs["plan_first"] = engine({"UVHTTP_WS_FUSED": "0"})
    st = torch.cuda.current_stream()
    for plen in plens:
        stride = U.gen_frame_stride(plen)
        n = min(1 << 22, (280 << 20) // stride)
        wl = stride * n
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        engs["fused"].gen_frames(wire, n, plen, 7, opcode0=2, fragmented=plen <= 256)
        res = {k: [] for k in engs}
        outs = {k: e.alloc_outputs(n) for k, e in engs.items()}
        for e in engs.values():
            e.reserve(n, wl, 0)
        for r in range(rounds + 1):
            for k, e in engs.items():
                desc, summ = outs[k]
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(K):
                    e.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ,
                                     max_message_size=1 << 30, stream=st)
                b.record(st)
                b.synchronize()
                if r:
                    res[k].append(a.elapsed_time(b) * 1e3 / K)
        for k, e in engs.items():
            s = e.read_summary(outs[k][1])
            assert s["n_delivered"] == n, (k, s)
        med = {k: statistics.median(v) for k, v in res.items()}
        gib = n * plen / 2 ** 30
        print(f"plen {plen:6d} stride {stride:6d} n {n:8d}  " + "  ".join(
            f"{k} {med[k]:8.1f} us ({gib / med[k] * 1e6:7.1f} GiB/s)" for k in engs), flush=True)


if __name__ == "__main__":
    main()
