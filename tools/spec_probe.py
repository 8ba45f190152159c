#!/usr/bin/env python3
"""Which path the stream decode takes on the equal-frame fuzzer's shapes
(tests/test_gpu_fuzz.py::test_hypothesis_equal_frame_streams_vs_oracle): each case decoded with
device stamps on — "walk" among a call's kernels means the speculative decode gave the call to
the walk (plan refusal, or a break in the pass / state machine), none means k_sspec_* decoded
it — and checked against the oracle as the fuzzer does.

  python tools/spec_probe.py
"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402
import test_gpu_streams as TS  # noqa: E402
from test_gpu_fuzz import _spec_case  # noqa: E402

BASE = {"plen": 200, "n": 30, "pattern": "frag", "op": 2, "break_at": None, "break_kind": "len",
        "tail": 0, "pending": False, "mm": 0, "reads": [0]}
VARIANTS = [
    {}, {"pattern": "whole"}, {"pattern": "mixed"}, {"pattern": "open_end"}, {"pending": True},
    {"tail": 9}, {"reads": [1000]}, {"plen": 65536, "n": 5}, {"plen": 58},
    {"break_at": 0}, {"break_at": 15}, {"break_at": 29}, {"break_at": 15, "break_kind": "ping"},
    {"break_at": 15, "break_kind": "rsv"}, {"break_at": 15, "break_kind": "unmasked"},
    {"break_at": 15, "break_kind": "cont", "pattern": "whole"}, {"break_at": 15, "break_kind": "start"},
    {"mm": 3000},
]


def main():
    import ctypes as C

    @U.CONTEXT_RESOLVER
    def resolver(conn):  # (test_gpu_streams' hooks fixture)
        return 0x77

    @U.CONTROL_SINK
    def sink(ctx, conn, op, p, n):
        TS.SINK.setdefault(conn, []).append(("pong" if op == 0xA else "close_echo",
                                             C.string_at(p, n) if n else b""))

    U.lib().uvhttp_ws_amd_set_control_hooks(resolver, sink)
    eng = U.GpuEngine(0)
    for i, v in enumerate(VARIANTS):
        rng = random.Random(1000 + i)
        conns = [dict(BASE, **v) for _ in range(6)]
        cases = [c for c in (_spec_case(U, rng, c) for c in conns) if c]
        eng.set_stamps(True)
        eng.read_stamps()
        TS._run_cases(torch, eng, U, cases, rng, 64 * len(cases), use_reads=len(v.get("reads", [0])) > 0
                      and v.get("reads", [0]) != [0])
        torch.cuda.synchronize()
        kinds = sorted({r[1] for r in eng.read_stamps()})
        eng.set_stamps(False)
        path = "walk" if "walk" in kinds else "speculative" if "spec_plan" in kinds else "?"
        print(f"{str(v):60s} -> {path:12s} kernels {kinds}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
