#!/usr/bin/env python3
"""Time the in-place decode of C2/C3/C4 under several engine environments in ONE process.

  python tools/stride_probe.py c4 c2 -- KEY=VAL,KEY=VAL  KEY=VAL ...

Each environment (comma-separated KEY=VAL list, read when its engine is created; the key LIB
names a library build, e.g. one from tools/build_variant.sh) gets an engine; rounds interleave
the engines on the same device buffers.  Reports the median
whole-step time (torch events around K steps) and the median time of the engine-timed kernel.
No result checks: experiment settings (e.g. UVHTTP_WS_MAX_POLLS=0) may decode wrongly."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402

CFG = {"c2": (65536, 4096, False), "c3": (65536, 65536, False), "c4": (1048576, 256, True)}


def engine(env):
    env = dict(env)
    lib = env.pop("LIB", None)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        if lib:
            return U.GpuEngine(0, library=U.load_library(os.path.join(REPO, lib)))
        return U.GpuEngine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    i = sys.argv.index("--")
    cfgs, envs = sys.argv[1:i], sys.argv[i + 1:]
    envs = [dict(kv.split("=", 1) for kv in e.split(",") if kv) for e in envs]
    rounds, K = 5, 20
    st = torch.cuda.current_stream()
    for cfg in cfgs:
        n, plen, frag = CFG[cfg]
        stride = U.gen_frame_stride(plen)
        wl = stride * n
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        engs = [engine(e) for e in envs]
        engs[0].gen_frames(wire, n, plen, 7, opcode0=2, fragmented=frag)
        outs = [e.alloc_outputs(n) for e in engs]
        step = [[] for _ in engs]
        kern = [[] for _ in engs]
        for r in range(rounds):
            for k, e in enumerate(engs):
                desc, summ = outs[k]

                def run():
                    e.decode_inplace(wire, n, stride=stride, max_message_size=256 << 20,
                                     wire_len=wl, desc=desc, summary=summ, stream=st)
                for _ in range(3):
                    run()
                e.set_timing(True)
                e.kernel_time()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(K):
                    run()
                b.record(st)
                b.synchronize()
                e.set_timing(False)
                ms, cnt = e.kernel_time()
                if r:
                    step[k].append(a.elapsed_time(b) / K)
                    kern[k].append(ms / max(cnt, 1))
        for k, e in enumerate(engs):
            s = e.read_summary(outs[k][1])
            print(f"{cfg} {sys.argv[i + 1 + k]:50s} step {statistics.median(step[k]) * 1e3:8.1f} us"
                  f"  kernel {statistics.median(kern[k]) * 1e3:8.1f} us  delivered {s['n_delivered']}",
                  flush=True)
            try:
                e.sync()
            except U.GpuError:
                pass
            e.close()
        del wire, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
