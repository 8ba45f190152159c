#!/usr/bin/env python3
"""Replays tests/test_batcher_group.py's random loop for one seed over several member lists and
prints, per list, every connection whose outcome differs from the oracle's (failure code,
transcript lengths, recv-buffer state).  usage: python tools/group_diag.py SEED"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import uvhttp_amd as U  # noqa: E402
import _oracle  # noqa: E402
from test_batcher_group import _drive  # noqa: E402
from test_batcher_transitions import Pair, _conn_reads  # noqa: E402


def run(devices, seed):
    rng = random.Random(600 + seed)
    b = U.BatcherGroup(devices, min_device_bytes=0, max_bytes=[64 << 10, 1 << 20, 8 << 20][seed - 1],
                       max_connections=64, max_reads=4000)
    pairs = [Pair(U, rng, reads=_conn_reads(rng, big=70000 if seed == 1 else 0)) for _ in range(45)]
    _drive(b, rng, pairs, forget_some=seed == 3)
    bad = []
    for i, p in enumerate(pairs):
        failed = p.key in b.failures or p.submit_failed
        pev, oev = p.events()
        s = p.prod.struct
        if failed != p.orc_failed or pev != oev or s.recv_buffer_pos != p.orc.recv_pos:
            bad.append((i, b.member(p.prod), b.failures.get(p.key), p.submit_failed, p.orc_failed,
                        len(pev), len(oev), s.recv_buffer_pos, p.orc.recv_pos,
                        [len(r) for r in p.reads]))
    st = b.stats()
    b.close()
    print(devices, "seed", seed, "mismatches", len(bad), "stats", {k: st[k] for k in (
        "flushes", "device_flushes", "host_flushes", "capacity_flushes", "fallback_flushes",
        "device_errors", "failures")})
    for x in bad:
        print("   conn %d member %d code %s submit_failed %s orc_failed %s events %d/%d recv %d/%d reads %s" % x)


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for devices in ([-1, -1], [0], [0, 0], [0, -1], [0, 0]):
        run(devices, seed)


if __name__ == "__main__":
    main()
