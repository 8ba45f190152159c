#!/usr/bin/env python3
"""k_plan per-block phase timeline (experiment build with -DUVWS_PLAN_PHASES).

  tools/build_variant.sh phases -DUVWS_PLAN_PHASES
  python tools/plan_phases.py tools/bin/libws_phases.so cfg:mode[:fused0] ...

For one decode call per case (after warm-up) prints, per k_plan block, when it started (after its
ticket), finished pass 1 (header / record loads + parse), the block scan, the look-back and pass 2
(state machine + descriptor stores), and its last wave's end — as percentiles over blocks, relative
to the earliest block start — plus the call's kernel-level device stamps."""
import ctypes as C
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402

CFG = {"c2": (65536, 4096, False), "c3": (65536, 65536, False), "c4": (1048576, 256, True)}


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1)))]


def main():
    L = U.load_library(sys.argv[1])
    L.uvhttp_ws_gpu_engine_debug_phases.restype = C.c_int
    L.uvhttp_ws_gpu_engine_debug_phases.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
    khz = 100000.0
    for case in sys.argv[2:]:
        parts = case.split(":")
        cfg, mode = parts[0], parts[1]
        if len(parts) > 2 and parts[2] == "fused0":
            os.environ["UVHTTP_WS_FUSED"] = "0"
        else:
            os.environ.pop("UVHTTP_WS_FUSED", None)
        n, plen, frag = CFG[cfg]
        e = U.GpuEngine(0, library=L)
        stride = U.gen_frame_stride(plen)
        wl = stride * n
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        e.gen_frames(wire, n, plen, 7, opcode0=2, fragmented=frag)
        desc, summ = e.alloc_outputs(n)
        arena = torch.empty(n * plen + 64, dtype=torch.uint8, device="cuda")
        msgs = torch.empty(n * 32, dtype=torch.uint8, device="cuda")

        def run():
            if mode == "inplace":
                e.decode_inplace(wire, n, stride=stride, max_message_size=256 << 20, wire_len=wl,
                                 desc=desc, summary=summ)
            else:
                e.decode_compact(wire, n, arena, stride=stride, max_message_size=256 << 20,
                                 wire_len=wl, desc=desc, msgs=msgs, summary=summ)
        e.set_stamps(True)
        for rep in range(4):
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            e.read_stamps()
            buf = np.zeros(8 * 8192, np.uint64)
            L.uvhttp_ws_gpu_engine_debug_phases(e.h, buf.ctypes.data, 8192)
            run()
            torch.cuda.synchronize()
            ks = e.read_stamps()
            buf[:] = 0
            L.uvhttp_ws_gpu_engine_debug_phases(e.h, buf.ctypes.data, 8192)
            ph = buf.reshape(8192, 8)
            used = ph[:, 0] > 0
            ph = ph[used].astype(np.int64)
            if not len(ph):
                print(case, "no k_plan blocks stamped")
                continue
            t0 = ph[:, 0].min()
            us = lambda x: x * 1e3 / khz  # noqa: E731  ticks -> us
            starts = us(ph[:, 0] - t0)
            p1 = us(ph[:, 1] - ph[:, 0])
            scan = us(ph[:, 2] - ph[:, 1])
            lb = us(ph[:, 3] - ph[:, 2])
            p2 = us(ph[:, 4] - ph[:, 3])
            tail = us(ph[:, 5] - ph[:, 4])
            end = us(ph[:, 5] - t0)
            f = lambda v: f"{pct(v, .1):6.1f}/{pct(v, .5):6.1f}/{pct(v, .9):6.1f}/{max(v):6.1f}"  # noqa: E731
            print(f"{case} rep{rep}: {len(ph)} blocks, kernel span {max(end):.1f} us  (p10/p50/p90/max)")
            print(f"   start skew {f(starts)}  pass1 {f(p1)}  scan {f(scan)}  lookback {f(lb)}  "
                  f"pass2 {f(p2)}  tail {f(tail)}  end {f(end)}")
            cus = len(set(int(x) for x in ph[:, 7]))
            print(f"   distinct CU ids {cus}")
            if ks:
                b0 = min(k[2] for k in ks)
                print("   kernels: " + "  ".join(f"{k[1]} {(k[2]-b0)/1e3:.1f}-{(k[3]-b0)/1e3:.1f}" for k in ks))
        e.close()
        del wire, arena, msgs, desc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
