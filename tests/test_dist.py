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


@pytest.mark.parametrize("world", [2, 4])
def test_bench_self_spawns_ranks(world):
    """`python bench.py --gpus N` with no launcher: the parent spawns N rank processes (before
    any GPU call), every rank bootstraps gloo, runs the timed region between barriers, and rank
    0's line reports N GPUs and the C5 strong-scaling workload.  --stub swaps the device step
    for a host sleep; everything else is the real main()."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", str(world),
                        "--stub", "--steps", "3", "--warmup", "1"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=repo)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["stub"] is True
    assert out["scaling"] == "strong" and out["config"]["workload"].startswith("C5")
    # the shard each rank timed: 8 388 608 / world frames in resident passes
    assert out["config"]["frames_per_gpu"] == 8388608 // world
    assert out["steps"] == 3 and out["ms_per_step"] > 0
    # every rank got past its post-run check, each on its own device
    assert out["ranks_checked"] == world and out["rank_devices"] == list(range(world))
    # the parent spawned its ranks without importing torch / touching HIP
    assert out["spawned_from_gpu_process"] is False


def test_bench_rank_failure_fails_the_run():
    """every rank checks its decode; one failing rank makes `bench.py --gpus 2` exit non-zero"""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["UVHTTP_WS_STUB_FAIL_RANK"] = "1"
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2",
                        "--stub", "--steps", "2", "--warmup", "0"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=repo)
    assert p.returncode != 0


def test_visible_gpus_without_hip(monkeypatch):
    """device counting for the spawn never calls into HIP"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3,5")
    assert bench.visible_gpus() == 3
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    for v in ("ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.visible_gpus() >= 0  # KFD topology (0 in a container without a GPU)
    assert "torch" not in sys.modules or not sys.modules["torch"].cuda.is_initialized()


def test_bench_torchrun_form_single_process():
    """WORLD_SIZE=1 set by a launcher: no spawning, one rank, C3 default."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--stub", "--steps", "2",
                        "--warmup", "0"], capture_output=True, text=True, timeout=300, env=env,
                       cwd=repo)
    assert p.returncode == 0, p.stderr
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["scaling"] == "weak"
    assert out["config"]["workload"].startswith("C3")


def test_rank_shards_are_global_c5_frames():
    """bench.py's rank r decodes frames [lo, ..) of THE C5 batch: its
    generator arguments name global frame indices, so rank 1 of 2 holds frame 4 194 304 of the
    8 388 608-frame batch, byte for byte the oracle's; c2-c4 ranks hold the config's batch."""
    import sys
    import numpy as np
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import bench
    import _oracle
    n_c5, plen = bench.CONFIGS["c5"][0], bench.CONFIGS["c5"][1]
    first, count, total = bench.gen_plan("c5", 1, 2)
    assert (first, count, total) == (n_c5 // 2, 1048576, n_c5)
    got, stride = _oracle.gen_frames(count, plen, bench.SEED, first=first, count=2, total=total)
    exp, _ = _oracle.gen_frames(n_c5, plen, bench.SEED, first=n_c5 // 2, count=2, total=n_c5)
    assert np.array_equal(got, exp)
    # and it is not rank 0's frame (the shards hold different frames)
    r0, _ = _oracle.gen_frames(count, plen, bench.SEED, first=0, count=1, total=total)
    assert not np.array_equal(got[:stride], r0)
    for w in (2, 4, 8):
        for r in range(w):
            f, c, t = bench.gen_plan("c5", r, w)
            assert f == r * n_c5 // w and c == min(1048576, n_c5 // w) and t == n_c5
    for cfg in ("c2", "c3", "c4"):
        n = bench.CONFIGS[cfg][0]
        assert bench.gen_plan(cfg, 1, 2) == (0, n, n)
