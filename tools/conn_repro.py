#!/usr/bin/env python3
"""One connection's reads (tests/test_batcher_group.py seed 2, connection 3: a 126-byte text
message, an empty non-final binary frame, a 5000-byte continuation cut part-way; max_message_size
0) through a device batcher under several flush patterns, each compared with the oracle fed the
same reads.  Prints the first divergence per pattern."""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import uvhttp_amd as U  # noqa: E402
import _oracle  # noqa: E402
from test_batcher_transitions import Pair, _conn_reads  # noqa: E402


def conn_reads():
    rng = random.Random(602)
    pairs = [Pair(U, rng, reads=_conn_reads(rng, big=0)) for _ in range(45)]
    p = pairs[3]
    c = p.prod.struct.config
    return p.reads, c.max_frame_size, c.max_message_size


def run(device, reads, mf, mm, flush_after, label):
    b = U.Batcher(device, min_device_bytes=0, max_bytes=1 << 20, max_connections=64, max_reads=4000)
    prod = U.WsConnection(1, mf, mm, user_data=False)
    orc = _oracle.OracleConn(1, mf, mm, record=1)
    import ctypes as C
    key = C.addressof(prod.ptr.contents)
    out = []
    for i, r in enumerate(reads):
        rc = b.submit(prod, r)
        orc_rc = orc.process_data(r)
        if i in flush_after:
            b.flush()
        failed = key in b.failures or rc != 0
        out.append((i, len(r), rc, b.failures.get(key), orc_rc))
        if orc_rc != 0 or failed:
            break
    b.flush()
    pev = [(t, a, len(x) if x else None) for t, a, x in prod.events if t in ("message", "close")]
    oev = [(t, a, len(x) if x else None) for t, a, x in orc.events() if t in ("message", "close")]
    s = prod.struct
    ok = pev == oev and s.recv_buffer_pos == orc.recv_pos and (key in b.failures or out[-1][2] != 0) == (out[-1][4] != 0)
    print(f"{label:28s} dev {device:2d} {'OK ' if ok else 'BAD'} calls {out} events {pev} / {oev} "
          f"recv {s.recv_buffer_pos}/{orc.recv_pos} stats dev_flushes {b.stats()['device_flushes']}")
    b.close()


def main():
    reads, mf, mm = conn_reads()
    print("mf", mf, "mm", mm, "reads", [len(r) for r in reads])
    n = len(reads)
    pats = {"flush each": set(range(n)), "flush after 0,1": {0, 1}, "flush after 1": {1},
            "flush after 0": {0}, "one flush at end": set(), "flush after 2": {2}}
    for dev in (-1, 0):
        for label, fa in pats.items():
            run(dev, reads, mf, mm, fa, label)
    # smaller: the first three reads as one read, and with the 2-byte carry
    joined = [b"".join(reads[:3])] + reads[3:]
    for dev in (-1, 0):
        run(dev, joined, mf, mm, {0}, "first three joined")
        run(dev, reads, mf, 64 << 20, set(range(n)), "flush each, mm 64M")


if __name__ == "__main__":
    main()
