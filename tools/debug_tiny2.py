#!/usr/bin/env python3
"""Debug: replay test_tiny_batches[1] of tests/test_gpu_summary_compact.py step by step."""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _oracle  # noqa: E402
import uvhttp_amd as U  # noqa: E402
import test_gpu_summary_compact as T  # noqa: E402

fast = U.GpuEngine(0)
fast.set_stamps(True)
os.environ["UVHTTP_WS_SUMMARY_FAST"] = "0"
slow = U.GpuEngine(0)
del os.environ["UVHTTP_WS_SUMMARY_FAST"]
n, stride = 1, 264
rng = random.Random(100 + n)
p = T._uniform_p(stride)
cases = [("frag0", T._batch(rng, n, stride, frag=0.0)), ("frag1", T._batch(rng, n, stride, frag=1.0)),
         ("rsv", T._batch(rng, n, stride, tweak=T._tweak("rsv", 0, p)))]
for name, wire in cases:
    ref = _oracle.decode_batch(wire, n, stride=stride, wire_len=wire.size, max_frame_size=T.MF, max_message_size=0,
                               compact=True, arena_cap=wire.size + 64)
    print(name, "wire[:4]", bytes(wire[:4]).hex(), "ref", ref["summary"]["n_delivered"], ref["summary"]["first_status"], flush=True)
    for k, e in enumerate((fast, slow)):
        for rep in range(2):
            d = torch.from_numpy(wire.copy()).to("cuda")
            arena = torch.zeros(wire.size + 64, dtype=torch.uint8, device="cuda")
            e.read_stamps() if k == 0 else None
            _, msgs, summ = e.decode_compact(d, n, arena, stride=stride, wire_len=wire.size, max_frame_size=T.MF,
                                             max_message_size=0, no_desc=True)
            torch.cuda.synchronize()
            s = e.read_summary(summ)
            kinds = sorted({r[1] for r in e.read_stamps()}) if k == 0 else []
            print("  ", "fast" if k == 0 else "slow", rep, "OK" if s == ref["summary"] else "BAD", s["n_delivered"], s["first_status"], kinds, flush=True)
