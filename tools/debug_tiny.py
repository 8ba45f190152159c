#!/usr/bin/env python3
"""Debug: a 1-3 frame compact summary-only decode with a failure at frame 0 (stamps show the path)."""
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
from test_gpu_parity import _frame  # noqa: E402

e = U.GpuEngine(0)
e.set_stamps(True)
rng = random.Random(1)
for n in (1, 2, 3):
    for at in range(n):
        frames = []
        for i in range(n):
            f = bytearray(_frame(2, 1, rng.randbytes(256), rng.randbytes(4)))
            if i == at:
                f[0] |= 0x40
            frames.append(bytes(f))
        wire = np.frombuffer(b"".join(frames), np.uint8).copy()
        ref = _oracle.decode_batch(wire, n, stride=264, max_message_size=0, compact=True, arena_cap=wire.size + 64)
        for nd in (True, False):
            d = torch.from_numpy(wire.copy()).to("cuda")
            arena = torch.zeros(wire.size + 64, dtype=torch.uint8, device="cuda")
            e.read_stamps()
            _, msgs, summ = e.decode_compact(d, n, arena, stride=264, max_message_size=0, wire_len=wire.size, no_desc=nd)
            torch.cuda.synchronize()
            s = e.read_summary(summ)
            kinds = sorted({r[1] for r in e.read_stamps()})
            ok = s == ref["summary"]
            print(n, at, "no_desc" if nd else "desc", "OK" if ok else "BAD", s["n_delivered"], s["first_status"], kinds, flush=True)
