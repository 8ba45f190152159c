#!/usr/bin/env python3
"""Interleaved A/B of two builds of libuvhttp_ws_amd.so in ONE process on one device.

  python tools/ab_lib.py LIB_A LIB_B cfg:mode [cfg:mode ...]     (mode: inplace | inplace_nd | compact | compact_nd | streams)

LIB_B may be "tree" for the in-tree build.  AB_STAMPS=1 turns engine B's device stamps on;
AB_ENV_B="K=V,..." sets environment switches for engine B only.  Each round runs K decode steps with engine A,
then K with engine B, on the same device buffers; reports the median whole-step time
(torch events around the K steps) and the median payload-kernel time (engine timing)."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402

CFG = {"c2": (65536, 4096, False), "c3": (65536, 65536, False), "c4": (1048576, 256, True),
       # (extra frame sizes for shape rules: same 256 MiB of payload)
       "f2k": (131072, 2048, False), "f8k": (32768, 8192, False), "f16k": (16384, 16384, False),
       "f24k": (10922, 24576, False), "f32k": (8192, 32768, False)}


def main():
    libs = [U.load_library(p if p != "tree" else U.LIB_PATH) for p in sys.argv[1:3]]
    names = [os.path.basename(p) for p in sys.argv[1:3]]
    rounds, K = 7, 20
    st = torch.cuda.current_stream()
    for pair in sys.argv[3:]:
        cfg, mode = pair.split(":")
        n, plen, frag = CFG[cfg]
        engs = [U.GpuEngine(0, library=libs[0])]
        # AB_ENV_B="K=V[,K=V]": environment switches for engine B only (read at engine creation)
        env_b = dict(kv.split("=", 1) for kv in os.environ.get("AB_ENV_B", "").split(",") if kv)
        old = {k: os.environ.get(k) for k in env_b}
        os.environ.update(env_b)
        try:
            engs.append(U.GpuEngine(0, library=libs[1]))
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        if os.environ.get("AB_STAMPS"):  # B with device stamps on (A off): their runtime cost
            engs[1].set_stamps(True)
        stride = U.gen_frame_stride(plen)
        wl = stride * n
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        engs[0].gen_frames(wire, n, plen, 7, opcode0=2, fragmented=frag)
        mm = 256 << 20
        sdev = None
        if mode == "streams":  # bench.py's layout: 4096 connections when fragmented, else one per frame
            import numpy as np
            conns = 4096 if frag else n
            per = n // conns
            sa = np.zeros(conns, dtype=U.STREAM_DT)
            sa["begin"] = np.arange(conns, dtype=np.uint64) * per * stride
            sa["len"] = per * stride
            sa["recv_buffer_size"] = max(65536, per * stride)
            sa["max_frame_size"], sa["max_message_size"], sa["is_server"] = 16 << 20, mm, 1
            if frag:
                sa["pending_bytes"][1:] = 1
                sa["pending_opcode"] = 2
            sdev = torch.from_numpy(sa.view(np.uint8).copy()).to("cuda")
            sres = [torch.empty(conns * U.STREAM_RESULT_BYTES, dtype=torch.uint8, device="cuda") for _ in engs]
        outs = []
        for e in engs:
            desc, summ = e.alloc_outputs(n)
            arena = torch.empty(n * plen + 64, dtype=torch.uint8, device="cuda") if mode.startswith("compact") else None
            msgs = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
            outs.append((desc, summ, arena, msgs))

        def run(k):
            e = engs[k]
            desc, summ, arena, msgs = outs[k]
            if mode == "streams":
                e.decode_streams(wire, sdev, conns, n, desc=desc, results=sres[k], wire_len=wl, stream=st)
            elif mode in ("inplace", "inplace_nd"):
                e.decode_inplace(wire, n, stride=stride, max_message_size=mm, wire_len=wl,
                                 desc=desc, summary=summ, stream=st, no_desc=mode == "inplace_nd")
            else:
                e.decode_compact(wire, n, arena, stride=stride, max_message_size=mm,
                                 wire_len=wl, desc=desc, msgs=msgs, summary=summ, stream=st,
                                 no_desc=mode == "compact_nd")

        step = [[], []]
        kern = [[], []]
        for r in range(rounds):
            for k in (0, 1):
                for _ in range(3):
                    run(k)
                engs[k].set_timing(True)
                engs[k].kernel_time()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(K):
                    run(k)
                b.record(st)
                b.synchronize()
                engs[k].set_timing(False)
                ms, cnt = engs[k].kernel_time()
                if r:
                    step[k].append(a.elapsed_time(b) / K)
                    kern[k].append(ms / max(cnt, 1))
        for k in (0, 1):
            if os.environ.get("AB_NOCHECK"):  # experiment builds may decode wrongly
                continue
            if mode == "streams":
                rs = engs[k].read_stream_results(sres[k], conns)
                assert all(x.status == 0 for x in rs) and sum(x.n_delivered for x in rs) == n, names[k]
            else:
                s = engs[k].read_summary(outs[k][1])
                assert s["n_delivered"] == n and s["status"] == 0, (names[k], s)
        ms = [statistics.median(x) for x in step]
        ks = [statistics.median(x) for x in kern]
        print(f"{cfg} {mode:8s} step A {ms[0]*1e3:9.1f} us  B {ms[1]*1e3:9.1f} us  "
              f"({(ms[0]/ms[1]-1)*100:+.1f}% B faster) | payload A {ks[0]*1e3:8.1f} B {ks[1]*1e3:8.1f} us "
              f"| other A {(ms[0]-ks[0])*1e3:6.1f} B {(ms[1]-ks[1])*1e3:6.1f} us", flush=True)
        for e in engs:
            e.close()
        del wire, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
