#!/usr/bin/env python3
"""A host decode after graph replays of the same engine, per library build: the replays leave
first-failure and tile-map tags with device epochs, larger than any host call's; the host call
must still report its own first failure.  usage: graph_then_host.py LIB [LIB ...]"""
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

rng = random.Random(3)
n, plen = 20000, 200
def batch(fail_at):
    return b"".join(_frame(0 if i == fail_at else 2, 1, rng.randbytes(plen), rng.randbytes(4), True, 0) for i in range(n))
ok_b, bad_b = batch(None), batch(777)
stride = len(ok_b) // n
wl = len(ok_b)
for lib in sys.argv[1:]:
    eng = U.GpuEngine(0, library=U.load_library(lib if lib != "tree" else U.LIB_PATH))
    wire = torch.zeros(wl + 64, dtype=torch.uint8, device="cuda")
    desc, summ = eng.alloc_outputs(n)
    eng.reserve(n, wl, 0)
    s = torch.cuda.Stream()
    wire[:wl].copy_(torch.from_numpy(np.frombuffer(bad_b, np.uint8).copy()))
    eng.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ, stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        eng.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ, stream=s)
    for _ in range(3):
        wire[:wl].copy_(torch.from_numpy(np.frombuffer(bad_b, np.uint8).copy()))
        torch.cuda.synchronize()
        g.replay()
    torch.cuda.synchronize()
    wire[:wl].copy_(torch.from_numpy(np.frombuffer(bad_b, np.uint8).copy()))
    eng.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ, stream=s)
    s.synchronize()
    ref = _oracle.decode_batch(np.frombuffer(bad_b, np.uint8).copy(), n, stride=stride, wire_len=wl)
    got = eng.read_summary(summ)
    print(os.path.basename(lib), "host call after replays:", "OK" if got == ref["summary"] else "WRONG",
          "n_delivered", got["n_delivered"], "expected", ref["summary"]["n_delivered"], flush=True)
    eng.close()
