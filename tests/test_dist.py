"""Multi-rank path of bench.py on CPU (gloo, world_size 2): shards cover every frame exactly
once with no shared frame (so no data-path collective), and the timed region is the slowest
rank's.  The GPU side of each rank is the single-GPU path tested in test_gpu_parity.py."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plans = {c: bench.shard_plan(c, rank, world) for c in ("c3", "c5")}
    slowest = bench.max_over_ranks(1.0 + rank, world)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, plans, slowest))


@pytest.mark.parametrize("world", [2, 4])
def test_shards_and_max_reduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # timed region = max over ranks
    assert all(r[2] == float(world) for r in res)
    # c5: contiguous, disjoint shards covering all 8 388 608 frames, resident chunks <= 2^20
    covered = []
    for _, plans, _ in res:
        first, per, passes = plans["c5"]
        assert per <= 1048576 and per * passes == 8388608 // world
        covered.append((first, first + per * passes))
    covered.sort()
    assert covered[0][0] == 0 and covered[-1][1] == 8388608
    assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
    # c3: every rank decodes its own full batch (weak scaling)
    assert all(plans["c3"][1] == 65536 and plans["c3"][2] == 1 for _, plans, _ in res)
