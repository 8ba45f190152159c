#!/usr/bin/env python3
"""bench.py — WebSocket payload unmask GiB/s (device-resident) on MI355X.

Metric (BASELINE.json): "WebSocket payload unmask GiB/s (device-resident), 64 KiB frames,
1/2/4/8 GPU".  One *step* = one pass of the hot path — frame-header parse + validation +
fragment state machine + payload unmask (include/uvhttp_ws_amd.h, decode_inplace) — over one
batch of synthetic masked frames already resident in HBM.  Default workload = BASELINE
config C3: 65 536 x 64 KiB masked BINARY frames per GPU.  Multi-GPU: one process per GPU
(torch.distributed.run), each rank decodes its own shard (frames are independent: weak
scaling, no data-path collective); a gloo barrier brackets the timed region and the max
elapsed time over ranks is used.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4] [--mode inplace|compact]

--config c5 runs BASELINE config C5 instead: 8 388 608 x 64 KiB frames in total, split into
contiguous per-rank shards (strong scaling), each decoded in resident 1 048 576-frame passes.

Rank 0 prints ONE JSON line.  `roofline` comes from HIP events bracketing the payload kernel
on its stream during the timed steps; `cpu_baseline` times the CPU port of the reference path
(oracle/, test infrastructure) on this host, rank 0 at N=1 only.
"""
import argparse
import ctypes as C
import json
import os
import platform
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    # name: (frames, payload bytes, fragmented, max_message_size)
    # c2/c3/c4: frames per GPU (weak scaling); c5: frames in total, sharded (strong scaling)
    "c2": (65536, 4096, False, 64 * 1024 * 1024),
    "c3": (65536, 65536, False, 64 * 1024 * 1024),
    "c4": (1048576, 256, True, 256 * 1024 * 1024),
    "c5": (8388608, 65536, False, 64 * 1024 * 1024),
}
C5_CHUNK = 1048576  # frames resident per decode pass (68.7 GB of wire at 64 KiB frames)
WORKLOAD = {
    "c2": "C2: 65536 x 4 KiB masked BINARY frames per GPU",
    "c3": "C3: 65536 x 64 KiB masked BINARY frames per GPU (C5 shard shape)",
    "c4": "C4: 1048576 x 256 B masked frames, one fragmented message per GPU",
    "c5": "C5: 8388608 x 64 KiB masked BINARY frames sharded evenly over the GPUs",
}


def shard_plan(cfg_name, rank, world):
    """Frames this rank decodes: (first_frame, frames_per_pass, passes).  c2-c4 give every
    rank its own full batch (weak scaling); c5 splits 8 388 608 frames into contiguous
    per-rank ranges [r*N/W, (r+1)*N/W), each decoded in resident chunks of <= 1 048 576
    frames; no frame is shared, so no data-path collective exists."""
    n, _, _, _ = CONFIGS[cfg_name]
    if cfg_name != "c5":
        return rank * n, n, 1
    lo, hi = rank * n // world, (rank + 1) * n // world
    per = min(hi - lo, C5_CHUNK)
    passes = (hi - lo + per - 1) // per
    return lo, per, passes


def max_over_ranks(value, world):
    """The timed region is the slowest rank's (gloo all_reduce MAX of a host scalar)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
SEED = 0x5EED0001
GIB = float(1 << 30)


def header_size(p):
    return 2 if p < 126 else 4 if p < 65536 else 10


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(cfg_name, target_s=10.0):
    """Time the oracle (CPU port of src/uvhttp_websocket.c, gcc -O2) on a bounded sample of
    the same workload: per-frame header parse + apply_mask (the unmask path), 1 thread.
    Also times the process_data loop fed 16 KiB reads (the live libuv shape)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle  # test infrastructure: CPU baseline leg only
    L = _oracle.load()
    n, plen, frag, mm = CONFIGS[cfg_name]
    sample = max(1, min(n, (128 << 20) // max(plen, 1)))  # ~128 MiB of payload
    wire, stride = _oracle.gen_frames(sample, plen, SEED, fragmented=frag, total=sample)
    ptr = _oracle._ptr(wire)
    payload = 0
    t0 = time.perf_counter()
    passes = 0
    while True:
        payload += L.oracle_unmask_frames(ptr, sample, stride)
        passes += 1
        el = time.perf_counter() - t0
        if el >= target_s * 0.5 or passes >= 1000:
            break
    unmask_gibs = payload / el / GIB
    # stream decode of the (re-masked) sample in 16 KiB reads
    if passes % 2:
        L.oracle_unmask_frames(ptr, sample, stride)  # restore masked bytes
    sp = 0
    t1 = time.perf_counter()
    spasses = 0
    while True:
        sp += L.oracle_stream_decode(ptr, wire.size, 16384, 16 * 1024 * 1024, mm, None)
        spasses += 1
        el2 = time.perf_counter() - t1
        if el2 >= target_s * 0.5 or spasses >= 1000:
            break
    stream_gibs = sp / el2 / GIB
    mt = cpu_baseline_threads(L, _oracle, cfg_name, target_s * 0.5)
    cc = subprocess.run(["gcc", "--version"], capture_output=True, text=True).stdout
    return {
        "value": round(unmask_gibs, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"{sample} frames x {plen} B of the {cfg_name.upper()} workload "
                  f"({sample * plen / GIB:.3f} GiB payload), header parse + apply_mask per "
                  f"frame, {passes} passes in {el:.1f} s",
        "stream_decode_16k_reads": round(stream_gibs, 3),
        "stream_decode_sample": f"process_data fed 16 KiB reads, {spasses} passes in {el2:.1f} s",
        "compiler": cc.splitlines()[0] if cc else "gcc", "flags": "-O2 -DNDEBUG",
        "cpu": cpu_model(), "host_threads": os.cpu_count(),
        "multi_thread": mt,
    }


def cpu_baseline_threads(L, orc, cfg_name, seconds):
    """SURVEY §8(d)'s all-cores variant: T threads, one independent connection stream each
    (its own ~32 MiB sample of the workload), header parse + apply_mask, timed together.
    T = this process's CPU share (16 on the GPU box; UVHTTP_WS_CPU_THREADS overrides)."""
    import threading
    n, plen, frag, _ = CONFIGS[cfg_name]
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    T = int(os.environ.get("UVHTTP_WS_CPU_THREADS", min(16, share)))
    sample = max(1, min(n, (32 << 20) // max(plen, 1)))
    bufs = [orc.gen_frames(sample, plen, SEED + 1 + t, fragmented=frag, total=sample)
            for t in range(T)]
    done = [0] * T
    start = threading.Barrier(T + 1)
    stop = threading.Event()

    def work(t):
        w, stride = bufs[t]
        ptr = orc._ptr(w)
        start.wait()
        while not stop.is_set():  # ctypes drops the GIL inside the call
            done[t] += L.oracle_unmask_frames(ptr, sample, stride)

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    start.wait()
    t0 = time.perf_counter()
    time.sleep(seconds)
    stop.set()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    return {"value": round(sum(done) / el / GIB, 3), "unit": "GiB/s", "cores": T,
            "sample": f"{T} threads x {sample} frames x {plen} B, {el:.1f} s"}


def pmc_traffic(cfg_name, mode):
    """HBM bytes per payload-kernel launch measured with rocprofv3 PMC counters (collected by
    tools/profile.sh into profiles/, FETCH_SIZE doubled per the gfx950 calibration)."""
    p = os.path.join(REPO, "profiles", f"traffic_{cfg_name}_{mode}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="inplace",
                    choices=["inplace", "compact", "streams", "build", "build_masked"])
    ap.add_argument("--conns", type=int, default=0,
                    help="streams mode: connections the frames are split over "
                         "(default: one frame per connection, 4096 for c4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--e2e", action="store_true", help="also time host->device->host")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)

    import torch
    import torch.distributed as dist
    import uvhttp_amd as U

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"

    _, plen, frag, mm = CONFIGS[args.config]
    first, n, passes = shard_plan(args.config, rank, world)
    stride = U.gen_frame_stride(plen)
    wire_len = stride * n
    eng = U.GpuEngine(local)
    stream = torch.cuda.current_stream(local)
    wire = torch.empty(wire_len + 64, dtype=torch.uint8, device=dev)
    eng.gen_frames(wire, n, plen, SEED + first, opcode0=2, fragmented=frag, stream=stream)
    desc, summ = eng.alloc_outputs(n)
    arena = msgs = None
    if args.mode == "compact":
        arena = torch.empty(n * plen + 64, dtype=torch.uint8, device=dev)
        msgs = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    eng.reserve(n, wire_len, n * plen if arena is not None else 0)
    streams_dev = build_dev = None
    if args.mode.startswith("build"):
        # send side: frame n payloads of the config (server echo: unmasked; client: masked)
        import numpy as np
        fr = np.zeros(n, dtype=[("po", "<u8"), ("pl", "<u8"), ("key", "<u4"), ("op", "u1"),
                                ("fin", "u1"), ("mask", "u1"), ("r0", "u1"), ("r1", "<u8")])
        fr["po"] = np.arange(n, dtype=np.uint64) * plen
        fr["pl"] = plen
        fr["key"] = np.arange(n, dtype=np.uint32) * 2654435761
        fr["op"], fr["fin"] = 2, 1
        fr["mask"] = 1 if args.mode == "build_masked" else 0
        build_dev = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
        build_src = torch.empty(n * plen + 64, dtype=torch.uint8, device=dev)
        build_src.random_(0, 256)
        build_out = torch.empty(n * (plen + 14) + 64, dtype=torch.uint8, device=dev)
        build_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    if args.mode == "streams":
        import numpy as np
        conns = args.conns or (4096 if frag else n)
        per = n // conns
        st = np.zeros(conns, dtype=[("begin", "<u8"), ("len", "<u8"), ("rbs", "<u8"),
                                    ("pend", "<u8"), ("pop", "<i4"), ("mf", "<i4"),
                                    ("mm", "<i4"), ("srv", "<i4")])
        st["begin"] = np.arange(conns, dtype=np.uint64) * per * stride
        st["len"] = per * stride
        st["rbs"] = max(65536, per * stride)
        st["mf"], st["mm"], st["srv"] = 16 * 1024 * 1024, mm, 1
        if frag:  # connection k continues the message: all its frames are continuations
            st["pend"][1:] = 1
            st["pop"] = 2
        streams_dev = torch.from_numpy(st.view(np.uint8).copy()).to(dev)
        s_desc = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        s_res = torch.empty(conns * 48, dtype=torch.uint8, device=dev)

    def step():
        for _ in range(passes):
            one_pass()

    def one_pass():
        if build_dev is not None:
            eng.build_frames(build_src, build_dev, n, build_out, out_off=build_off, stream=stream)
        elif streams_dev is not None:
            eng.decode_streams(wire, streams_dev, streams_dev.numel() // 48, n, desc=s_desc,
                               results=s_res, wire_len=wire_len, stream=stream)
        elif arena is None:
            eng.decode_inplace(wire, n, stride=stride, max_message_size=mm, wire_len=wire_len,
                               desc=desc, summary=summ, stream=stream)
        else:
            eng.decode_compact(wire, n, arena, stride=stride, max_message_size=mm,
                               wire_len=wire_len, desc=desc, msgs=msgs, summary=summ,
                               stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if build_dev is not None:
        if int(build_off[n].item()) != n * (stride - (0 if args.mode == "build_masked" else 4)):
            raise SystemExit("build failed")
    elif streams_dev is not None:
        rs = eng.read_stream_results(s_res, streams_dev.numel() // 48)
        if sum(r.n_delivered for r in rs) != n or any(r.status for r in rs):
            raise SystemExit(f"stream decode failed: {rs[0].as_dict()}")
    else:
        s = eng.read_summary(summ)
        if s["n_delivered"] != n or s["status"] != 0:
            raise SystemExit(f"decode failed: {s}")
    eng.kernel_time()  # discard warmup events

    eng.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    k_ms, k_n = eng.kernel_time()
    if streams_dev is None and build_dev is None:
        s = eng.read_summary(summ)
        assert s["n_delivered"] == n and s["status"] == 0, s

    el_max = max_over_ranks(elapsed, world)
    payload_per_rank = n * plen * passes
    total_payload = payload_per_rank * world * args.steps
    value = total_payload / el_max / GIB

    # algorithmic bytes of the payload kernel per launch: in place, every
    # frame's header+key+payload is read and its payload written; compact reads the same
    # and writes the payload into the arena.
    alg_bytes = n * ((header_size(plen) + 4 + plen) + plen)
    if build_dev is not None:  # payload read + frame written
        alg_bytes = n * (plen + header_size(plen) + (4 if args.mode == "build_masked" else 0) + plen)
    avg_kernel_s = (k_ms / 1e3 / k_n) if k_n else float("nan")
    achieved = alg_bytes / avg_kernel_s / 1e9 if k_n else None
    traffic = pmc_traffic(args.config, args.mode)

    e2e = None
    if args.e2e and rank == 0:
        e2e = e2e_rate(n, plen, stride, mm, local)

    if rank == 0:
        out = {
            "metric": "WebSocket payload unmask GiB/s (device-resident), 64 KiB frames, 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "c5" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 payload + per-frame keys, generated on device)",
            "config": {
                "workload": WORKLOAD[args.config],
                "mode": args.mode,
                "frames_per_gpu": n * passes,
                "decode_passes_per_step": passes,
                "payload_bytes_per_frame": plen,
                "wire_bytes_per_frame": stride,
                "parallelism": f"shard{world} (independent frames, no collective)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": {"compact": "k_gather_compact", "build": "kb_emit",
                           "build_masked": "kb_emit"}.get(args.mode, "k_unmask_inplace"),
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes,
                "avg_kernel_us": round(avg_kernel_s * 1e6, 2) if k_n else None,
                "launches_timed": k_n,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        if e2e:
            out["e2e_pcie"] = e2e
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


def e2e_rate(n, plen, stride, mm, local, depth=3, slot_frames=1024):
    """Host-memory pipeline (uvhttp_ws_gpu_pipeline_*): masked frames in pinned host slots
    -> H2D -> decode_inplace -> D2H, `depth` slots on their own streams so copies and kernels
    overlap.  PCIe-bound; recorded in DESIGN.md, never the metric."""
    import uvhttp_amd as U
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle  # bench input generation only (host frames)
    slot_frames = min(slot_frames, n)
    wl = stride * slot_frames
    pipe = U.GpuPipeline(local, depth=depth, slot_bytes=wl, slot_frames=slot_frames)
    host, _ = _oracle.gen_frames(slot_frames, plen, SEED)
    for k in range(depth):
        pipe.buffer(k)[:wl] = host
    total = max(depth, n // slot_frames)
    for k in range(depth):  # warm
        pipe.submit(k, wl, slot_frames, stride=stride, max_message_size=mm)
    for k in range(depth):
        pipe.wait(k)
    t0 = time.perf_counter()
    busy = set()
    for k in range(total):
        slot = k % depth
        if slot in busy:
            _, _, s = pipe.wait(slot)
            assert s["n_delivered"] == slot_frames
        pipe.submit(slot, wl, slot_frames, stride=stride, max_message_size=mm)
        busy.add(slot)
    for slot in busy:
        pipe.wait(slot)
    el = time.perf_counter() - t0
    pipe.close()
    return {"value": round(total * slot_frames * plen / el / GIB, 2), "unit": "GiB/s",
            "slots": depth, "slot_frames": slot_frames, "batches": total,
            "note": "pinned host slots -> H2D -> decode_inplace -> D2H, overlapped across slots"}


if __name__ == "__main__":
    main()
