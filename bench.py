#!/usr/bin/env python3
"""bench.py — WebSocket payload unmask GiB/s (device-resident) on MI355X.

Metric (BASELINE.json): "WebSocket payload unmask GiB/s (device-resident), 64 KiB frames,
1/2/4/8 GPU".  One *step* = one pass of the hot path — frame-header parse + validation +
fragment state machine + payload unmask (include/uvhttp_ws_amd.h, decode_inplace) — over one
batch of synthetic masked frames already resident in HBM.  Default workload = BASELINE
config C3: 65 536 x 64 KiB masked BINARY frames on one GPU.  Multi-GPU (default C5): one
process per GPU, each rank decodes its own contiguous shard of the 8 388 608 frames (frames
are independent: strong scaling, no data-path collective); a gloo barrier brackets the timed
region and the max elapsed time over ranks is used.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5] [--mode inplace|compact]
                  [--rotate R]

--config c5 runs BASELINE config C5 instead: 8 388 608 x 64 KiB frames in total, split into
contiguous per-rank shards (strong scaling), each decoded in resident 1 048 576-frame passes.
It is the default whenever more than one GPU runs (BASELINE config 5, "reported at 1/2/4/8
GPUs"); the N=1 default (C3) also times C5 on its one GPU ("c5_1gpu", and "c5_base": that
value in the N>1 lines' unit) so the curve has a base.

--rotate R decodes R independent copies of the batch round-robin (one per step), so a step's
wire was last touched R-1 steps earlier: with R copies larger than the 256 MB Infinity Cache
the rate is the cold-HBM one (C2 / C4 fit the cache once).

Launch: under torch.distributed.run (RANK/WORLD_SIZE set) every process is one rank.  Started
directly with --gpus N > 1, this process spawns the N rank processes itself (before anything
touches a GPU), waits for them and prints rank 0's line.

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


def gen_plan(cfg_name, rank, world):
    """What this rank's resident frames are, as generator arguments: (first, count, total).
    c2-c4: every rank holds the config's whole batch (frames 0 .. n-1, the batch the full-size
    parity tests check).  c5: rank r's shard is frames [lo, lo + per) of the one 8 388 608-frame
    C5 batch (global frame indices, so rank r decodes exactly the frames a single process
    decoding all of C5 would give it; tests/test_dist.py pins rank 1's first frame)."""
    first, per, _ = shard_plan(cfg_name, rank, world)
    if cfg_name != "c5":
        return 0, per, per
    return first, per, CONFIGS["c5"][0]


def max_over_ranks(value, world):
    """The timed region is the slowest rank's (gloo all_reduce MAX of a host scalar)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


TIMING_EVERY = int(os.environ.get("UVHTTP_WS_TIMING_EVERY", "10"))
# the roofline's event-timed launches: at least this many, the missing ones timed in an untimed
# window after the timed steps (GpuWorkload.event_window)
MIN_EVENT_LAUNCHES = 10
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
        "cpu": cpu_model(), "machine_cpus": os.cpu_count(), "process_cpus": _cpu_share(),
        "multi_thread": mt,
    }


def _cpu_share():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_quota():
    """CPUs the cgroup grants this process (cgroup v2 cpu.max "quota period"), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return None


def cpu_threads():
    """(threads, source) for the all-cores baseline: UVHTTP_WS_CPU_THREADS, else the cgroup CPU
    quota when one is set (the box grants a share of a larger machine), else every CPU in this
    process's affinity mask."""
    if os.environ.get("UVHTTP_WS_CPU_THREADS"):
        return int(os.environ["UVHTTP_WS_CPU_THREADS"]), "UVHTTP_WS_CPU_THREADS"
    aff, quota = _cpu_share(), cpu_quota()
    if quota is not None and quota < aff:
        return quota, f"cgroup cpu.max quota ({quota} CPUs; affinity mask {aff})"
    return aff, f"sched_getaffinity ({aff} CPUs; cgroup cpu.max {'max' if quota is None else quota})"


def cpu_baseline_threads(L, orc, cfg_name, seconds):
    """SURVEY §8(d)'s all-cores variant: T threads, one independent connection stream each
    (its own ~32 MiB sample of the workload), header parse + apply_mask, timed together.
    T = cpu_threads(): the CPUs this process may really use (cgroup quota, else affinity),
    named in the record."""
    import threading
    n, plen, frag, _ = CONFIGS[cfg_name]
    T, source = cpu_threads()
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
            "cores_source": source,
            "sample": f"{T} threads x {sample} frames x {plen} B, {el:.1f} s",
            "note": "every CPU this process may use, one connection stream each"}


def pmc_traffic(cfg_name, mode):
    """(HBM bytes per payload-kernel launch, source) measured with rocprofv3 PMC counters
    (collected by tools/profile.sh / tools/pmc_traffic.py into profiles/, FETCH_SIZE doubled per
    the gfx950 calibration); source names the file and the run tag it came from."""
    name = f"traffic_{cfg_name}_{mode}.json"
    p = os.path.join(REPO, "profiles", name)
    if not os.path.exists(p):
        return None, None
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    src = f"profiles/{name}" + (f" (run {d['tag']}, kernel avg {d.get('payload_kernel_avg_ns_rocprof', 0) / 1e3:.1f} us)"
                                if d.get("tag") else "")
    return d.get("hbm_bytes_per_launch"), src


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus():
    """GPUs this process could use, without initialising HIP: HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set, else the KFD topology nodes that
    have SIMDs (/sys/class/kfd/kfd/topology/nodes/*/properties: simd_count > 0)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "properties")) as f:
                    props = dict(line.split() for line in f if len(line.split()) == 2)
                if int(props.get("simd_count", "0")) > 0:
                    n += 1
            except (OSError, ValueError):
                continue
    except OSError:
        pass
    return n


def parent_touched_gpu():
    """True if this process imported torch and initialised its GPU state (never before a spawn)"""
    t = sys.modules.get("torch")
    return bool(t is not None and t.cuda.is_initialized())


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each), wait for all of them and
    pass rank 0's JSON line through.  Called before anything in this process touches a GPU, so
    the children are fresh processes, never an exec of a GPU-initialised one."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   UVHTTP_WS_SPAWNED_FROM_GPU_PROCESS="1" if parent_touched_gpu() else "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else None,
                                      text=True))
    out0, _ = procs[0].communicate()
    rcs = [p.wait() for p in procs]
    sys.stdout.write(out0)
    sys.stdout.flush()
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


class StubWorkload:
    """--stub (tests only): the launcher, rank bootstrap, barrier, timing and reporting of the
    real run with a host sleep as the step — no GPU, no library."""

    def __init__(self, args, cfg, rank, world, local):
        _, self.plen, _, _ = CONFIGS[cfg]
        self.first, self.n, self.passes = shard_plan(cfg, rank, world)
        self.stride = self.plen + header_size(self.plen) + 4
        self.kernel = "stub"

    def step(self):
        time.sleep(0.001 * self.passes)

    def sync(self):
        pass

    def set_timing(self, on):
        pass

    def kernel_time(self):
        return 0.0, 0

    def check(self):
        # tests: a rank whose decode "fails" must make the whole run exit non-zero
        if os.environ.get("UVHTTP_WS_STUB_FAIL_RANK") == os.environ.get("RANK", "0"):
            raise SystemExit("stub decode failed")

    def close(self):
        pass


class GpuWorkload:
    """One rank's shard of a config, resident in HBM, decoded through the C-ABI."""

    def __init__(self, args, cfg, rank, world, local):
        import torch
        import uvhttp_amd as U
        self.torch = torch
        torch.cuda.set_device(local)
        dev = f"cuda:{local}"
        mode = args.mode
        _, plen, frag, mm = CONFIGS[cfg]
        first, n, passes = shard_plan(cfg, rank, world)
        self.plen, self.n, self.passes, self.mode, self.mm = plen, n, passes, mode, mm
        self.use_graph = bool(getattr(args, "graph", False))
        self.no_desc = bool(getattr(args, "no_desc", False)) and mode in ("inplace", "compact")
        self.stride = stride = U.gen_frame_stride(plen)
        self.wire_len = wire_len = stride * n
        self.eng = eng = U.GpuEngine(local)
        self.stream = stream = torch.cuda.current_stream(local)
        self.wire = torch.empty(wire_len + 64, dtype=torch.uint8, device=dev)
        g_first, g_count, g_total = gen_plan(cfg, rank, world)
        eng.gen_frames(self.wire, n, plen, SEED, opcode0=2, fragmented=frag, stream=stream,
                       first=g_first, count=g_count, total=g_total)
        # --rotate R: R copies decoded round-robin, so a step's bytes are not the ones the
        # previous step just wrote (cold HBM once R copies exceed the Infinity Cache)
        self.wires = [self.wire] + [self.wire.clone() for _ in range(max(1, args.rotate) - 1)]
        self.turn = 0
        self.desc, self.summ = eng.alloc_outputs(n)
        self.arena = self.msgs = None
        if mode == "compact":
            self.arena = torch.empty(n * plen + 64, dtype=torch.uint8, device=dev)
            self.msgs = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        eng.reserve(n, wire_len, n * plen if self.arena is not None else 0)
        self.build_dev = self.streams_dev = None
        self.graph = None
        # the payload kernel that actually runs (ws_gpu.hip run_decode): a compact decode takes
        # the wire-driven scatter below 16 KiB of wire per frame, the arena-driven gather above
        # (UVHTTP_WS_COMPACT=gather|scatter pins it); the send side's small-frame kernel below
        # 4 KiB per frame (UVHTTP_WS_BUILD_FRAMES)
        cm = os.environ.get("UVHTTP_WS_COMPACT", "")
        scatter = cm == "scatter" or (cm != "gather" and stride < 16384)
        small_build = stride < int(os.environ.get("UVHTTP_WS_BUILD_FRAMES", "4096") or 0)
        self.kernel = {"compact": "k_scatter_compact" if scatter else "k_gather_compact",
                       "build": "kb_emit_frames" if small_build else "kb_emit",
                       "build_masked": "kb_emit_frames" if small_build else "kb_emit",
                       }.get(mode, "k_unmask_inplace")
        # in place, a batch of equal-stride small frames takes the fused path (ws_gpu.hip
        # run_decode: payload before plan, stride <= UVHTTP_WS_FUSED_MAX, default 2560 B)
        fused_max = int(os.environ.get("UVHTTP_WS_FUSED_MAX", "2560") or 2560)
        if mode == "inplace" and os.environ.get("UVHTTP_WS_FUSED", "1") != "0" and 64 <= stride <= fused_max:
            self.kernel = "k_unmask_stride"
            # summary-only: the one-pass decode (its summary tail after it) when the message
            # limit cannot bind (ws_gpu.hip run_decode)
            if self.no_desc and stride >= 140 and os.environ.get("UVHTTP_WS_SUMMARY_FAST", "1") != "0" \
                    and (mm == 0 or n * (stride - 8) <= mm):
                self.kernel = "k_unmask_stride (summary-only one-pass decode)"
        # compact, the same stride range: the speculative pass (k_unmask_stride writing the
        # arena, ws_gpu.hip run_decode) unless UVHTTP_WS_SPEC=0
        spec_max = int(os.environ.get("UVHTTP_WS_SPEC_MAX", "2560") or 2560)
        if mode == "compact" and os.environ.get("UVHTTP_WS_SPEC", "1") != "0" and 64 <= stride <= spec_max:
            self.kernel = "k_unmask_stride (speculative compact pass)"
            if self.no_desc and stride >= 140 and os.environ.get("UVHTTP_WS_SUMMARY_FAST", "1") != "0" \
                    and (mm == 0 or n * (stride - 8) <= mm):
                self.kernel = "k_unmask_stride (summary-only speculative compact pass)"
        if mode.startswith("build"):
            # send side: frame n payloads of the config (server echo: unmasked; client: masked)
            import numpy as np
            fr = np.zeros(n, dtype=[("po", "<u8"), ("pl", "<u8"), ("key", "<u4"), ("op", "u1"),
                                    ("fin", "u1"), ("mask", "u1"), ("r0", "u1"), ("r1", "<u8")])
            fr["po"] = np.arange(n, dtype=np.uint64) * plen
            fr["pl"] = plen
            fr["key"] = np.arange(n, dtype=np.uint32) * 2654435761
            fr["op"], fr["fin"] = 2, 1
            fr["mask"] = 1 if mode == "build_masked" else 0
            self.build_dev = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
            self.build_src = torch.empty(n * plen + 64, dtype=torch.uint8, device=dev)
            self.build_src.random_(0, 256)
            self.build_out = torch.empty(n * (plen + 14) + 64, dtype=torch.uint8, device=dev)
            self.build_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        if mode == "streams":
            import numpy as np
            conns = args.conns or (4096 if frag else n)
            per = n // conns
            st = np.zeros(conns, dtype=U.STREAM_DT)
            st["begin"] = np.arange(conns, dtype=np.uint64) * per * stride
            st["len"] = per * stride
            st["recv_buffer_size"] = max(65536, per * stride)
            st["max_frame_size"], st["max_message_size"], st["is_server"] = 16 << 20, mm, 1
            if frag:  # connection k continues the message: all its frames are continuations
                st["pending_bytes"][1:] = 1
                st["pending_opcode"] = 2
            self.conns = conns
            self.streams_dev = torch.from_numpy(st.view(np.uint8).copy()).to(dev)
            self.s_desc = torch.empty(n * 32, dtype=torch.uint8, device=dev)
            self.s_res = torch.empty(conns * U.STREAM_RESULT_BYTES, dtype=torch.uint8, device=dev)

    def one_pass(self):
        eng, stream = self.eng, self.stream
        self.wire = self.wires[self.turn % len(self.wires)]
        self.turn += 1
        if self.build_dev is not None:
            eng.build_frames(self.build_src, self.build_dev, self.n, self.build_out,
                             out_off=self.build_off, stream=stream)
        elif self.streams_dev is not None:
            eng.decode_streams(self.wire, self.streams_dev, self.conns, self.n, desc=self.s_desc,
                               results=self.s_res, wire_len=self.wire_len, stream=stream)
        elif self.arena is None:
            eng.decode_inplace(self.wire, self.n, stride=self.stride, max_message_size=self.mm,
                               wire_len=self.wire_len, desc=self.desc, summary=self.summ,
                               stream=stream, no_desc=self.no_desc)
        else:
            eng.decode_compact(self.wire, self.n, self.arena, stride=self.stride,
                               max_message_size=self.mm, wire_len=self.wire_len, desc=self.desc,
                               msgs=self.msgs, summary=self.summ, stream=stream,
                               no_desc=self.no_desc)

    def step(self):
        if self.graph is not None:
            self.graph.replay()
            return
        for _ in range(self.passes):
            self.one_pass()

    def capture(self):
        """--graph: one step captured as a HIP graph (torch.cuda.CUDAGraph), replayed per step —
        one submission per step instead of one per kernel.  The engine's calls see a capturing
        stream (ws_gpu.hip call_begin: device-side epochs, no timing events), so the roofline
        then has no kernel time; used to tell dispatch-path idle from kernel time."""
        t = self.torch
        self.sync()
        cs = t.cuda.Stream()
        g = t.cuda.CUDAGraph()
        old = self.stream
        self.stream = cs
        with t.cuda.graph(g, stream=cs):
            for _ in range(self.passes):
                self.one_pass()
        self.stream = old
        self.graph = g
        self.sync()

    def sync(self):
        self.torch.cuda.synchronize()

    def set_timing(self, on):
        # events around every TIMING_EVERY-th payload kernel: a timed marker idles the device
        # ~4.6 us per event (rocprofv3 trace, profiles/r03p4_*), so timing every launch would
        # inflate the step it measures
        self.eng.set_timing(on, every=TIMING_EVERY)

    def kernel_time(self):
        return self.eng.kernel_time()

    def event_window(self, launches):
        """Untimed, right after the timed steps: `launches` more passes with HIP events around
        EVERY payload kernel (the timed steps bracket every TIMING_EVERY-th launch only, which at
        --steps 20 is 2 launches) -> (ms, launches).  A pass launched as several dispatch pieces
        (C5) is bracketed as a whole."""
        self.eng.set_timing(True, every=1)
        for _ in range(launches):
            self.one_pass()
        self.sync()
        self.eng.set_timing(False)
        return self.eng.kernel_time()

    def copy_ceiling(self, reps=10):
        """Same-run streaming ceiling: uvhttp_ws_gpu_apply_mask — one key XOR-ed
        over the whole wire in place, the payload kernel's access pattern with no framing —
        timed with HIP events on the same stream; an even count leaves the wire as it was.
        -> (GB/s of read + write, average µs)"""
        eng, w = self.eng, self.wires[0]
        eng.kernel_time()
        eng.set_timing(True)
        for _ in range(reps + reps % 2):
            eng.apply_mask(w, b"\x5a\xa5\x3c\xc3", length=self.wire_len, stream=self.stream)
        self.torch.cuda.synchronize()
        eng.set_timing(False)
        ms, k = eng.kernel_time()
        avg = ms / 1e3 / k
        return 2 * self.wire_len / avg / 1e9, avg * 1e6

    def timeline(self, calls=16, step_ms=None):
        """Device-side kernel stamps (uvhttp_ws_gpu_engine_set_stamps) over `calls` more steps
        after the timed region, same process and buffers: when each kernel of a call ran on the
        device, so the payload kernel's own duration (no timing event beside it) and the gaps
        between kernels and between calls are measured where they happen (the send side's
        kernels too: kb_size, the scans, the emit kernel as "payload").
        The clearing read_stamps() copies the 71 MB ring back while the device idles, and the
        calls right after an idle run slower until its clocks are back up: C3's payload kernel
        read 1301 us there and 1251 us after 40 more calls, against 1256 us by HIP events in
        steady state (tools/stamp_probe.py, profiles/r06d_stamp_probe.txt) — the "stamps
        exceed the step" rejections of round 5.  So warm-up passes (>= 60 ms of them) run after
        the clear, and only the last `calls` calls are read."""
        if self.graph is not None:
            return None
        eng = self.eng
        eng.set_stamps(True)
        eng.read_stamps()  # drop anything older
        keep = min(calls, 15)
        warm = max(10, int(60.0 / step_ms)) if step_ms else 40
        warm = min(warm, 128 - keep)  # (the ring holds the last 128 calls)
        for _ in range(warm + keep):
            self.one_pass()
        self.sync()
        recs = eng.read_stamps()
        eng.set_stamps(False)
        last = []  # the last `keep` calls (records come oldest call first)
        for r in recs:
            if not last or last[-1] != r[0]:
                last.append(r[0])
        tail = set(last[-keep:])
        out = summarize_stamps([r for r in recs if r[0] in tail])
        if out:
            out["calls_from"] = f"{keep} more steps after the timed region, after {warm} warm-up steps"
        return out

    def check(self):
        """Every frame of the shard must have been delivered (the decode really ran)."""
        n = self.n
        if self.build_dev is not None:
            want = n * (self.stride - (0 if self.mode == "build_masked" else 4))
            if int(self.build_off[n].item()) != want:
                raise SystemExit("build failed")
        elif self.streams_dev is not None:
            rs = self.eng.read_stream_results(self.s_res, self.conns)
            if sum(r.n_delivered for r in rs) != n or any(r.status for r in rs):
                raise SystemExit(f"stream decode failed: {rs[0].as_dict()}")
        else:
            s = self.eng.read_summary(self.summ)
            if s["n_delivered"] != n or s["status"] != 0:
                raise SystemExit(f"decode failed: {s}")

    def close(self):
        self.eng.close()
        for k in ("wire", "wires", "desc", "summ", "arena", "msgs", "build_src", "build_out",
                  "streams_dev", "s_desc"):
            setattr(self, k, None)
        self.torch.cuda.empty_cache()


def summarize_stamps(recs):
    """Per-call device timeline -> medians: payload-kernel duration, whole chain (first
    kernel start .. last kernel end), the gap at every kernel boundary inside a call, and the
    idle between one call's last kernel and the next call's first."""
    import statistics
    calls = {}  # in the order read_stamps returns them: oldest call first (tags wrap)
    for call, kern, b, e in recs:
        calls.setdefault(call, []).append((b, e, kern))
    order = list(calls)
    if not order:
        return None
    med = lambda xs: round(statistics.median(xs) / 1e3, 2) if xs else None  # noqa: E731
    pay, chain, inter, gaps, durs = [], [], [], {}, {}
    prev_end, prev_c = None, None
    for c in order:
        ks = sorted(calls[c])
        chain.append(ks[-1][1] - ks[0][0])
        pay += [e - b for b, e, k in ks if k == "payload"]
        for b, e, k in ks:
            durs.setdefault(k, []).append(e - b)
        for (b0, e0, k0), (b1, e1, k1) in zip(ks, ks[1:]):
            gaps.setdefault(f"{k0}->{k1}", []).append(b1 - e0)
        if prev_end is not None and (c - prev_c) % ((1 << 24) - 1) == 1:  # consecutive calls
            inter.append(ks[0][0] - prev_end)
        prev_end, prev_c = max(e for _, e, _ in ks), c
    mean = lambda xs: round(sum(xs) / len(xs) / 1e3, 2) if xs else None  # noqa: E731
    return {"calls": len(order), "kernels": [k for _, _, k in sorted(calls[order[-1]])],
            "payload_us": med(pay), "chain_us": med(chain),
            "gap_between_calls_us": med(inter),
            "gap_between_calls_max_us": round(max(inter) / 1e3, 2) if inter else None,
            "gaps_us": {k: med(v) for k, v in gaps.items()},
            "kernels_us": {k: med(v) for k, v in durs.items()},
            # means and maxima too: an idle that comes in bursts moves these, not the medians
            "chain_mean_us": mean(chain),
            "gap_between_calls_mean_us": mean(inter),
            "gaps_mean_us": {k: mean(v) for k, v in gaps.items()},
            "gaps_max_us": {k: round(max(v) / 1e3, 2) for k, v in gaps.items()},
            "source": "device wall clock (uvhttp_ws_gpu_engine_read_stamps), medians unless named"}


def timed_run(wl, steps, warmup, world):
    """W untimed steps, then exactly K timed steps bracketed by barrier + device sync on both
    sides; returns (max elapsed over ranks, kernel ms, kernel launches)."""
    import torch.distributed as dist
    for _ in range(warmup):
        wl.step()
    wl.sync()
    if getattr(wl, "use_graph", False):
        wl.capture()
        wl.step()
    wl.check()
    wl.kernel_time()  # discard warmup events
    wl.set_timing(True)
    if world > 1:
        dist.barrier()
    wl.sync()
    t0 = time.perf_counter()
    host = 0.0  # time the host spends issuing the steps (device idle if it exceeds the GPU's)
    for _ in range(steps):
        h0 = time.perf_counter()
        wl.step()
        host += time.perf_counter() - h0
    wl.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    wl.set_timing(False)
    k_ms, k_n = wl.kernel_time()
    wl.check()
    wl.host_issue_s = host
    return max_over_ranks(elapsed, world), k_ms, k_n


def c5_one_gpu(args, local, steps=2, warmup=1):
    """BASELINE C5 on this one GPU (8 resident passes of 1 048 576 frames per step): the N=1
    point of the C5 curve the multi-GPU runs report."""
    a = argparse.Namespace(**vars(args))
    a.mode = "inplace"
    wl = GpuWorkload(a, "c5", 0, 1, local)
    el, k_ms, k_n = timed_run(wl, steps, warmup, 1)
    n_total = CONFIGS["c5"][0]
    out = {"value": round(n_total * wl.plen * steps / el / GIB, 2), "unit": "GiB/s",
           "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
           "avg_kernel_us": round(k_ms * 1e3 / k_n, 2) if k_n else None,
           "note": "C5 8388608 x 64 KiB frames on 1 GPU: 8 resident passes of 1048576 frames"}
    wl.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: c3 on one GPU, c5 (strong scaling) on more")
    ap.add_argument("--mode", default="inplace",
                    choices=["inplace", "compact", "streams", "build", "build_masked"])
    ap.add_argument("--conns", type=int, default=0,
                    help="streams mode: connections the frames are split over "
                         "(default: one frame per connection, 4096 for c4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5-base", action="store_true",
                    help="N=1: skip the extra C5-on-one-GPU measurement")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--e2e", action="store_true", help="also time host->device->host")
    ap.add_argument("--rotate", type=int, default=1,
                    help="decode R copies of the batch round-robin (cold-cache rates)")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the copy-ceiling timing")
    ap.add_argument("--no-stamps", action="store_true",
                    help="skip the device-timeline (kernel stamp) steps after the timed region")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as one captured HIP graph (diagnostic: no kernel timing)")
    ap.add_argument("--no-desc", action="store_true",
                    help="inplace / compact: d_desc = NULL (summary-only decode: no per-frame "
                         "descriptors; fixed-stride batches of >= 140 B frames in place take the "
                         "one-pass decode)")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="allow more ranks than GPUs: rank r uses device LOCAL_RANK %% visible "
                         "(launcher readiness runs on a one-GPU box; the ranks share one HBM)")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)  # launcher tests
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the parent never touches HIP (nor imports torch): it only counts devices from the
        # environment / KFD topology and starts fresh rank processes
        if not args.stub:
            have = visible_gpus()
            if have < args.gpus and not args.oversubscribe:
                raise SystemExit(f"--gpus {args.gpus} but only {have} GPU(s) visible "
                                 "(--oversubscribe maps several ranks to one device)")
        raise SystemExit(spawn_ranks(args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    cfg = args.config or ("c5" if world > 1 else "c3")

    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    device = local
    if args.oversubscribe and not args.stub:
        import torch
        device = local % max(1, torch.cuda.device_count())  # counts devices, no HIP context
    wl = (StubWorkload if args.stub else GpuWorkload)(args, cfg, rank, world, device)
    wl.no_stamps = args.no_stamps
    el_max, k_ms, k_n = timed_run(wl, args.steps, args.warmup, world)
    timed_launches = k_n
    if rank == 0 and hasattr(wl, "event_window") and k_n < MIN_EVENT_LAUNCHES and wl.graph is None:
        w_ms, w_n = wl.event_window(MIN_EVENT_LAUNCHES - k_n)
        k_ms, k_n = k_ms + w_ms, k_n + w_n
    n, plen, passes, stride = wl.n, wl.plen, wl.passes, wl.stride
    payload_per_rank = n * plen * passes
    total_payload = payload_per_rank * world * args.steps
    value = total_payload / el_max / GIB

    # algorithmic bytes of the payload kernel per launch: in place, every
    # frame's header+key+payload is read and its payload written; compact reads the same
    # and writes the payload into the arena.
    alg_bytes = n * ((header_size(plen) + 4 + plen) + plen)
    if args.mode.startswith("build"):  # payload read + frame written
        alg_bytes = n * (plen + header_size(plen) + (4 if args.mode == "build_masked" else 0) + plen)
    avg_kernel_s = (k_ms / 1e3 / k_n) if k_n else float("nan")
    achieved = alg_bytes / avg_kernel_s / 1e9 if k_n else None
    traffic, traffic_src = pmc_traffic(cfg, args.mode + ("_summary_only" if getattr(args, "no_desc", False) else ""))
    ceiling = None
    if rank == 0 and not args.stub and not args.no_ceiling:
        ceiling = wl.copy_ceiling()
    tl = None
    if rank == 0 and not args.stub and not args.no_stamps:
        tl = wl.timeline(step_ms=el_max / args.steps * 1e3)
    # every rank ran check() before and after its timed steps (a failing rank exits non-zero);
    # count the ranks that got here, and the devices they ran on
    ranks_checked, devices = world, [device]
    if world > 1:
        import torch
        t = torch.tensor([1.0])
        dist.all_reduce(t)
        ranks_checked = int(t.item())
        got = [None] * world
        dist.all_gather_object(got, device)
        devices = got
    wl.close()
    # the dominant kernel's duration: the device stamps' payload-kernel median when stamped
    # (no timing event beside the kernel), else the HIP events.  A duration is used only if it
    # is physically possible: not longer than the step's share (a kernel of the step cannot
    # outlast it), not so short that the algorithmic bytes would exceed the HBM peak, and not
    # faster than 1.05 x the same-run copy ceiling (a stamp ring that kept one piece of a
    # multi-piece pass read a C5 pass as 6.7 us, frac 2568: VERDICT r05).  Stamps first, then
    # events, then the step itself; none valid -> the run fails.
    event_us = avg_kernel_s * 1e6 if k_n else None
    step_us = el_max / args.steps * 1e6
    share_us = step_us / passes
    ceil_gbs = ceiling[0] if ceiling else None

    def why_invalid(us):
        if not us or us <= 0:
            return "no measurement"
        if us > share_us * (1 + 1e-9):
            return f"{us:.1f} us exceeds the step's {share_us:.1f} us"
        gbs = alg_bytes / (us / 1e6) / 1e9
        if gbs > HBM_PEAK_GBS:
            return f"{us:.1f} us means {gbs:.0f} GB/s > the {HBM_PEAK_GBS:.0f} GB/s peak"
        if ceil_gbs and gbs > 1.05 * ceil_gbs:
            return f"{us:.1f} us means {gbs:.0f} GB/s > 1.05 x the copy ceiling ({ceil_gbs:.0f})"
        return None

    stamp_us = tl.get("payload_us") if tl else None
    cands = [("device stamps (median of the timeline calls)", stamp_us),
             (f"hip events ({k_n} launches: {timed_launches} sampled in the timed steps, "
              f"{k_n - timed_launches} in the window after them)", event_us),
             ("step time (upper bound of the kernel)", share_us)]
    rejected, kern_us, kern_src = [], None, None
    for name, us in cands:
        bad = why_invalid(us)
        if bad is None:
            kern_us, kern_src = us, name
            break
        if us:
            rejected.append(f"{name.split(' (')[0]}: {bad}")
    if kern_us is None and not args.stub:
        raise SystemExit("no physically possible kernel time: " + "; ".join(rejected))
    if rejected and kern_us is not None:
        kern_src += " [rejected: " + "; ".join(rejected) + "]"
    achieved = alg_bytes / (kern_us / 1e6) / 1e9 if kern_us else None

    extra = {}
    if rank == 0 and world == 1 and not args.stub:
        if cfg == "c3" and args.mode == "inplace" and not args.no_c5_base:
            extra["c5_1gpu"] = c5_one_gpu(args, local)
            # the N>1 lines (default config C5) divide by this: same metric, same unit
            extra["c5_base"] = extra["c5_1gpu"]["value"]
        if args.e2e:
            warm = e2e_warmup(local)
            # the pipeline once untimed (its first pass over fresh pinned slots runs slow:
            # profiles/r04_pipeline_sweep.jsonl), then the measured pass; 2048-frame slots
            first = e2e_rate(n, plen, stride, CONFIGS[cfg][3], local, slot_frames=2048)
            extra["e2e_pcie"] = e2e_rate(n, plen, stride, CONFIGS[cfg][3], local, slot_frames=2048)
            extra["e2e_pcie"]["warmup_value"] = first["value"]
            extra["e2e_live"] = e2e_live(local)
            extra["e2e_live"]["warmup_runs"] = warm

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
            "scaling": "strong" if cfg == "c5" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 payload + per-frame keys, generated on device)",
            "config": {
                "workload": WORKLOAD[cfg],
                "mode": args.mode + ("_summary_only" if getattr(wl, "no_desc", False) else ""),
                "frames_per_gpu": n * passes,
                "decode_passes_per_step": passes,
                "payload_bytes_per_frame": plen,
                "wire_bytes_per_frame": stride,
                "parallelism": f"shard{world} (independent frames, no collective)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": wl.kernel,
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": alg_bytes,
                "avg_kernel_us": round(kern_us, 2) if kern_us else None,
                "avg_kernel_source": kern_src,
                "event_kernel_us": round(event_us, 2) if event_us else None,
                "stamp_kernel_us": stamp_us,
                "launches_timed": k_n,
                "copy_ceiling": None if ceiling is None else {
                    "kernel": "k_apply_mask (uvhttp_ws_gpu_apply_mask over the whole wire)",
                    "achieved": round(ceiling[0], 1), "unit": "GB/s",
                    "avg_us": round(ceiling[1], 2),
                    "frac_of_peak": round(ceiling[0] / HBM_PEAK_GBS, 4),
                    "kernel_frac_of_ceiling": round(achieved / ceiling[0], 4) if achieved else None},
            },
            "host_issue_us_per_step": round(getattr(wl, "host_issue_s", 0.0) / args.steps * 1e6, 2),
        }
        if tl:
            out["device_timeline"] = tl
        if cfg == "c5":
            out["config"]["c5_model"] = (
                "each rank decodes its contiguous share of the 8388608 frames as passes of one "
                "resident 1048576-frame chunk (generated once; alternate passes re-mask it): the "
                "bytes moved per pass are the chunk's, the frames past the first chunk are not "
                "materialised")
        if world > 1:
            out["ranks_checked"] = ranks_checked
            out["rank_devices"] = devices
        if args.oversubscribe:
            out["oversubscribed"] = len(set(devices)) < world
            out["config"]["oversubscribe_note"] = (
                "launcher readiness: ranks share devices (LOCAL_RANK % visible), so they share "
                "one HBM — not a scaling measurement")
        if args.stub:
            out["stub"] = True
        if "UVHTTP_WS_SPAWNED_FROM_GPU_PROCESS" in os.environ:
            out["spawned_from_gpu_process"] = os.environ["UVHTTP_WS_SPAWNED_FROM_GPU_PROCESS"] == "1"
        if args.rotate > 1:
            out["config"]["rotate"] = args.rotate
        if args.graph:
            out["config"]["graph"] = True
        if world == 1 and not args.no_cpu_baseline and not args.stub:
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        out.update(extra)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def e2e_warmup(local, min_runs=4, max_runs=8):
    """PCIe/host-path warm-up before the e2e numbers: on a fresh box the first few seconds of
    host<->device traffic run slower (the live harness: 17 then 24 then 40 GiB/s in three
    consecutive processes, the same 40 after; tools/e2e_order.sh,
    profiles/r04_e2e_order.jsonl) — the link's power state ramps with sustained traffic.  Runs
    the async live harness at least min_runs times (two runs of a cold box can agree at the cold
    rate: 24.1, 23.7 GiB/s, then 40 — r04_pipeline_sweep2.jsonl) and until two consecutive runs
    agree within 5 %; returns their values."""
    exe = os.path.join(REPO, "tests", "c", "_build", "batcher_e2e")
    vals = []
    for _ in range(max_runs):
        p = subprocess.run([exe, "--conns", "1024", "--frames", "4", "--size", "65536", "--flushes",
                            "20", "--device", str(local), "--async", "1", "--cap", "0.5", "--pin", "1"],
                           capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            break
        vals.append(json.loads(p.stdout.strip().splitlines()[-1])["value"])
        if len(vals) >= min_runs and abs(vals[-1] - vals[-2]) <= 0.05 * vals[-1]:
            break
    return vals


def e2e_live(local, conns=1024, frames=4, size=65536, flushes=20):
    """The live shape end to end (tests/c/batcher_e2e.c): 16 KiB libuv reads of `conns`
    connections queued in the batcher, one device flush per round (stage, H2D,
    decode_reads, D2H, on_message per connection), synchronous and asynchronous
    (flush_async + poll on on_ready); the same reads through the host decoder
    on one core beside it.  PCIe- and host-memcpy-bound; recorded in DESIGN.md, never the
    metric."""
    exe = os.path.join(REPO, "tests", "c", "_build", "batcher_e2e")
    out = {}
    # device runs: the loop thread on the GPU's NUMA node (--pin 1)
    # async: queues of half a round (max_bytes = half the bytes one loop pass reads, the sizing
    # INTEGRATION.md §3 recommends) — a loop that outruns PCIe waits on a flush twice per round
    # for half as long, and copies overlap better: 40 GiB/s with p99 blocked < 1 ms where whole-
    # round queues gave 23-40 GiB/s and p99 3.6-8 ms (profiles/r04_bench_e2e.json);
    # device_async_round keeps the whole-round queues for comparison
    # read models (tests/c/batcher_e2e.c --reads): "submit" — the bytes are already in a buffer
    # and submit_read copies them into the pinned arena; "kcopy" — the socket read is modelled as
    # a copy into a 16 KiB libuv buffer, then submit_read (the reference's shape: two copies on
    # the loop thread); "zc" — alloc_read / commit_read, the socket read lands in the arena (one)
    for name, dev, asy, cap, reads in (
            ("device", local, 0, 1.0, "submit"), ("device_async", local, 1, 0.5, "submit"),
            ("device_async_kcopy", local, 1, 0.5, "kcopy"), ("device_async_zc", local, 1, 0.5, "zc"),
            ("device_async_round", local, 1, 1.0, "submit"), ("host_1core", -1, 0, 1.0, "submit")):
        p = subprocess.run([exe, "--conns", str(conns), "--frames", str(frames), "--size",
                            str(size), "--flushes", str(flushes if dev >= 0 else 3),
                            "--device", str(dev), "--async", str(asy), "--cap", str(cap),
                            "--pin", "1" if dev >= 0 else "0", "--reads", reads],
                           capture_output=True, text=True, timeout=600)
        out[name] = json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else \
            {"error": p.returncode, "stderr": p.stderr[-300:]}
    # the PCIe ceiling of this box for the same bytes (tools/pcie_probe.hip): one flush's wire up
    # and down; the live shape cannot beat batcher_shape_ms per 256 MiB round
    probe = os.path.join(REPO, "tools", "bin", "pcie_probe")
    if os.path.exists(probe):
        p = subprocess.run([probe, "256", "2"], capture_output=True, text=True, timeout=300)
        if p.returncode == 0:
            pc = json.loads(p.stdout.strip().splitlines()[-1])
            wire = conns * frames * (size + (10 if size >= 65536 else 4 if size >= 126 else 2) + 4)
            pc["ceiling_GiBs_for_this_payload"] = round(
                conns * frames * size / (pc["batcher_shape_ms"] / 1e3 * wire / pc["bytes"]) / GIB, 2)
            out["pcie"] = pc
    return out


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
