"""The batcher's state transitions (include/uvhttp_ws_amd.h, uvhttp_ws_amd_batcher_*), each
checked against the oracle fed the same reads per connection (the reference's
on_websocket_read loop: process_data per read until one fails, src/uvhttp_connection.c:
1098-1175):

* a queue that overflows max_bytes / max_reads / max_connections inside submit_read (the
  queue is handed over there), reads larger than a whole flush (decoded in submit_read after
  the connection's earlier reads), flush / flush_async / poll interleaved at random;
* reads submitted and connections forgotten (and re-created) from inside on_message while a
  flush delivers — on the host path and, with a device, while the other queue fills;
* (device) client-side connections whose tiny unmasked frames overflow the frame capacity
  (ERR_CAPACITY -> the queue re-runs on the host) and injected device failures
  (UVHTTP_WS_BATCHER_FAIL_EVERY -> the queue decodes on the host, the error is returned).

device = -1 runs here on the CPU (host decoder); device = 0 is marked gpu.
"""
import ctypes as C
import os
import random

import pytest

import _oracle
from test_gpu_streams import _frame, _frames

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEVICES = [-1, pytest.param(0, marks=pytest.mark.gpu)]


def _need_device(device):
    if device >= 0:
        import torch
        if not torch.cuda.is_available():
            pytest.skip("no GPU")


def _conn_reads(rng, big=0):
    frames, _ = _frames(rng, rng.randint(0, 10), False, bad=rng.random() < 0.3)
    data = b"".join(frames)
    reads, pos = [], 0
    while pos < len(data):
        n = rng.choice([1, 7, 300, 4096, 16384, rng.randint(1, 20000)] + ([big] if big else []))
        reads.append(data[pos:pos + n])
        pos += n
    return reads


class Pair:
    """A product connection and its oracle twin fed the same reads."""

    def __init__(self, U, rng, mf=None, mm=None, reads=None, zc=False):
        mf = mf or rng.choice([16 * 1024 * 1024, 65536, 4000])
        mm = mm if mm is not None else rng.choice([64 * 1024 * 1024, 9000, 0])
        self.prod = U.WsConnection(1, mf, mm, user_data=False)
        self.orc = _oracle.OracleConn(1, mf, mm, record=1)
        self.reads = reads if reads is not None else []
        self.next = 0
        self.orc_failed = False
        self.submit_failed = False
        self.dead = False  # forgotten and freed
        self.zc = zc  # reads through alloc_read / commit_read (the libuv alloc + read shape)

    @property
    def key(self):
        return C.addressof(self.prod.ptr.contents)

    def feed(self, b, data):
        """one read: to the batcher and (until it fails) to the oracle"""
        if self.orc_failed or self.submit_failed or self.dead:
            return
        if self.zc:
            # the socket read lands in the staging arena; a short allocation splits it into
            # several reads, which the oracle gets as the same process_data calls
            rc, pieces = b.submit_zero_copy(self.prod, data)
            pos = 0
            for k in pieces:
                if self.orc.process_data(data[pos:pos + k]) != 0:
                    self.orc_failed = True
                    break
                pos += k
            if rc != 0:
                self.submit_failed = True
            return
        rc = b.submit(self.prod, data)
        # (a read larger than a flush is decoded inside submit_read: its rc is process_data's)
        if self.orc.process_data(data) != 0:
            self.orc_failed = True
        if rc != 0:
            self.submit_failed = True

    def events(self):
        pev = [(t, a, p) for t, a, p in self.prod.events if t in ("message", "close")]
        oev = [(t, a, p if t == "message" else None) for t, a, p in self.orc.events()
               if t in ("message", "close")]
        return pev, oev

    def check(self, b, L):
        if self.dead:  # delivered up to the forget: a prefix of the oracle's transcript
            pev, oev = self.events()
            assert pev == oev[:len(pev)]
            return
        failed = self.key in b.failures or self.submit_failed
        assert failed == self.orc_failed
        pev, oev = self.events()
        assert pev == oev
        s = self.prod.struct
        assert s.recv_buffer_pos == self.orc.recv_pos
        assert C.string_at(s.recv_buffer, s.recv_buffer_pos) == self.orc.recv_bytes()
        assert s.recv_buffer_size == self.orc.recv_size
        assert (s.fragmented_size if s.fragmented_message else 0) == L.oracle_conn_frag_size(self.orc.c)
        assert s.fragmented_opcode == self.orc.frag_opcode


def _drive(U, b, rng, pairs):
    """random loop iterations: some connections get a read each, then flush / flush_async /
    poll / nothing; finally flush"""
    while any(p.next < len(p.reads) for p in pairs):
        for p in rng.sample(pairs, len(pairs)):
            if p.next >= len(p.reads) or rng.random() < 0.3:
                continue
            p.feed(b, p.reads[p.next])
            p.next += 1
        act = rng.random()
        if act < 0.3:
            assert b.flush() == 0
        elif act < 0.6:
            assert b.flush_async() == 0
        elif act < 0.8:
            assert b.poll() in (0, 1)
    assert b.flush() == 0
    assert not b.in_flight()


@pytest.mark.parametrize("zc", [False, True], ids=["submit", "zero_copy"])
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("seed", [1, 2])
def test_overflow_and_oversize_reads(device, seed, zc):
    """tiny queue limits: flushes start inside submit_read (alloc_read); 70 000-byte reads
    exceed a whole flush (max_bytes 48 KiB) and are decoded directly, after the connection's
    queued reads — or, zero-copy, land in pieces of what one flush holds"""
    _need_device(device)
    import uvhttp_amd as U
    rng = random.Random(seed)
    b = U.Batcher(device=device, min_device_bytes=0, max_bytes=48 * 1024,
                  max_connections=6, max_reads=40)
    pairs = [Pair(U, rng, reads=_conn_reads(rng, big=70000), zc=zc) for _ in range(24)]
    _drive(U, b, rng, pairs)
    st = b.stats()
    assert st["flushes"] > 10
    assert st["zero_copy_reads"] > 0 if zc else st["direct_reads"] > 0
    if device >= 0:
        assert st["device_flushes"] > 0 and st["async_flushes"] > 0
    L = _oracle.load()
    for p in pairs:
        p.check(b, L)
    b.close()


@pytest.mark.parametrize("zc", [False, True], ids=["submit", "zero_copy"])
@pytest.mark.parametrize("device", DEVICES)
def test_submit_and_forget_from_callbacks(device, zc):
    """on_message of the 'driver' connections submits a read for a 'chained' connection (it
    lands in the queue being filled, never the one being delivered) and forgets a 'victim'
    connection mid-stream, re-creating a fresh connection that then gets reads of its own"""
    _need_device(device)
    import uvhttp_amd as U
    rng = random.Random(7)
    b = U.Batcher(device=device, min_device_bytes=0)
    key = b"\x11\x22\x33\x44"
    # chained connections: their whole stream is submitted from callbacks, one read per event
    chained = [Pair(U, rng, mf=16 << 20, mm=64 << 20, zc=zc,
                    reads=_conn_reads(rng)) for _ in range(6)]
    victims = [Pair(U, rng, mf=16 << 20, mm=64 << 20, zc=zc,
                    reads=[_frame(2, 1, rng.randbytes(100), key, True, 0)] * 40) for _ in range(4)]
    fresh = []
    drivers = [Pair(U, rng, mf=16 << 20, mm=64 << 20, zc=zc,
                    reads=[_frame(1, 1, b"tick %d" % i, key, True, 0) for i in range(60)])
               for _ in range(3)]

    def hook(conn, ev):
        for c in chained:
            if c.next < len(c.reads) and rng.random() < 0.5:
                c.feed(b, c.reads[c.next])
                c.next += 1
        if victims and rng.random() < 0.1:
            v = victims.pop()
            b.forget(v.prod)
            v.dead = True
            v.prod.close()  # a new connection may now get the same address
            n = Pair(U, rng, mf=16 << 20, mm=64 << 20, reads=_conn_reads(rng), zc=zc)
            fresh.append(n)
            n.feed(b, n.reads[0])
            n.next = 1
            forgotten_pairs.append(v)

    forgotten_pairs = []
    all_victims = list(victims)
    for d in drivers:
        d.prod.hook = hook
    _drive(U, b, rng, drivers + victims + fresh)
    # whatever the callbacks queued last
    while any(c.next < len(c.reads) for c in chained + fresh):
        for c in chained + fresh:
            if c.next < len(c.reads):
                c.feed(b, c.reads[c.next])
                c.next += 1
        assert b.flush() == 0
    assert b.flush() == 0
    L = _oracle.load()
    for p in drivers + chained + fresh + all_victims:
        p.check(b, L)
    assert forgotten_pairs, "no connection was forgotten from a callback"
    b.close()


@pytest.mark.gpu
def test_capacity_and_device_failure_fall_back_to_host():
    """client-side connections of 2-byte unmasked frames overflow the frame capacity
    (a queue's descriptors: max(65 536, bytes / 6 + connections)): the device reports
    ERR_CAPACITY and the queue re-runs on the host.  Then every device launch fails (test hook): each queue is decoded on the host,
    flush returns ELAUNCH and nothing is lost."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import uvhttp_amd as U
    rng = random.Random(5)
    L = _oracle.load()
    b = U.Batcher(device=0, min_device_bytes=0)
    prods, orcs = [], []
    for k in range(8):
        prod = U.WsConnection(0, 16 << 20, 64 << 20)
        orc = _oracle.OracleConn(0, 16 << 20, 64 << 20, record=1)
        data = b"".join(_frame(2, 1, b"", b"", False, 0) for _ in range(12000))
        assert b.submit(prod, data) == 0
        assert orc.process_data(data) == 0
        prods.append(prod)
        orcs.append(orc)
    assert b.flush() == 0
    st = b.stats()
    assert st["capacity_flushes"] == 1 and st["host_reads"] == 8
    for prod, orc in zip(prods, orcs):
        assert len(prod.events) == len(orc.events()) == 12000
    b.close()

    # server connections: 6-byte frames (empty masked payloads) beyond the initial 65 536
    # descriptors but within the bytes / 6 bound: the decode re-runs on the device with more
    b = U.Batcher(device=0, min_device_bytes=0)
    prod = U.WsConnection(1, 16 << 20, 64 << 20)
    orc = _oracle.OracleConn(1, 16 << 20, 64 << 20, record=1)
    data = b"".join(_frame(2, 1, b"", rng.randbytes(4), True, 0) for _ in range(70000))
    assert b.submit(prod, data) == 0 and orc.process_data(data) == 0
    assert b.flush() == 0
    st = b.stats()
    assert st["capacity_flushes"] == 0 and st["host_reads"] == 0 and st["device_frames"] == 70000
    assert len(prod.events) == len(orc.events()) == 70000
    b.close()

    os.environ["UVHTTP_WS_BATCHER_FAIL_EVERY"] = "1"
    try:
        b = U.Batcher(device=0, min_device_bytes=0, library=U.test_hooks_library())
    finally:
        del os.environ["UVHTTP_WS_BATCHER_FAIL_EVERY"]
    pairs = [Pair(U, rng, reads=_conn_reads(rng)) for _ in range(10)]
    rcs = []
    while any(p.next < len(p.reads) for p in pairs):
        for p in pairs:
            if p.next < len(p.reads):
                p.feed(b, p.reads[p.next])
                p.next += 1
        rcs.append(b.flush())
    assert set(rcs) <= {0, -4} and -4 in rcs
    st = b.stats()
    assert st["device_errors"] > 0 and st["device_flushes"] == 0
    for p in pairs:
        p.check(b, L)
    b.close()


def test_numa_node_host_only_is_unknown():
    """uvhttp_ws_amd_batcher_numa_node: a host-only batcher has no GPU node (-1)"""
    import uvhttp_amd as U
    b = U.Batcher(device=-1)
    assert b.numa_node() == -1
    b.close()


@pytest.mark.gpu
def test_numa_node_of_the_device():
    """the device batcher reports its GPU's NUMA node from sysfs (or -1 where sysfs has none);
    the value matches the PCI device's numa_node file"""
    import glob
    import uvhttp_amd as U
    b = U.Batcher(device=0, min_device_bytes=0)
    node = b.numa_node()
    nodes = {int(open(f).read()) for f in glob.glob("/sys/class/drm/card*/device/numa_node")}
    assert node == -1 or node in nodes
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6])
def test_async_split_frames_stay_on_the_device(seed):
    """The live shape's async loop with a staging capacity of about one round: a flush cuts
    frames of the next round in two, and the connections' next reads are queued while that
    flush is still in flight.  Their recv-buffer prefix at staging time must be accounted from
    the in-flight reads too (prefix_bound), or the queue outgrows the device layout and falls
    back to the host decoder.  No fallback, and every transcript equals the oracle's."""
    import uvhttp_amd as U
    rng = random.Random(seed)
    pairs = []
    for _ in range(12):
        frames, _ = _frames(rng, 6, False, bad=False)  # complete, valid frames
        data = b"".join(frames)
        pairs.append(Pair(U, rng, mf=16 * 1024 * 1024, mm=64 * 1024 * 1024,
                          reads=[data[i:i + 4096] for i in range(0, len(data), 4096)]))
    per_round = sum(len(r) for p in pairs for r in p.reads) // 3
    b = U.Batcher(device=0, min_device_bytes=0, max_bytes=per_round + 64 * 1024)
    while any(p.next < len(p.reads) for p in pairs):
        for _ in range(len(pairs)):
            p = rng.choice(pairs)
            for _ in range(rng.randint(1, 6)):
                if p.next < len(p.reads):
                    p.feed(b, p.reads[p.next])
                    p.next += 1
            if b.in_flight() and rng.random() < 0.5:
                assert b.poll() in (0, 1)
        assert b.flush_async() == 0
    assert b.flush() == 0
    st = b.stats()
    assert st["fallback_flushes"] == 0 and st["host_flushes"] == 0, st
    assert st["device_flushes"] >= 2
    L = _oracle.load()
    for p in pairs:
        p.check(b, L)
    b.close()


@pytest.mark.parametrize("between", ["submit", "forget_other", "alloc_other"])
@pytest.mark.parametrize("device", DEVICES)
def test_commit_refused_after_another_queueing_call(device, between):
    """alloc_read(A), then another batcher call that queues (submit_read of B, a
    forget, a second alloc_read), then commit_read(A) must be refused — B's bytes would
    otherwise land in (device: share) the arena space A's socket read used — and both
    connections' payloads arrive intact once A's bytes are submitted again."""
    _need_device(device)
    import uvhttp_amd as U
    b = U.Batcher(device=device, min_device_bytes=0)
    key = b"\x01\x02\x03\x04"
    a = U.WsConnection(1, 16 << 20, 64 << 20, user_data=False)
    bb = U.WsConnection(1, 16 << 20, 64 << 20, user_data=False)
    other = U.WsConnection(1, 16 << 20, 64 << 20, user_data=False)
    fa = _frame(2, 1, bytes(range(200)) * 3, key, True, 0)
    fb = _frame(1, 1, b"B" * 333, key, True, 0)
    assert b.submit(other, _frame(1, 1, b"o", key, True, 0)) == 0
    rc, addr, n = b.alloc(a, len(fa))
    assert rc == 0 and n >= len(fa)
    C.memmove(addr, fa, len(fa))  # the socket read lands in the arena
    if between == "submit":
        assert b.submit(bb, fb) == 0
    elif between == "forget_other":
        b.forget(other)
    else:
        rc2, addr2, n2 = b.alloc(bb, len(fb))
        assert rc2 == 0
    assert b.commit(a, len(fa)) == -1  # UVHTTP_ERROR_INVALID_PARAM
    assert b.submit(a, fa) == 0
    if between != "submit":
        assert b.submit(bb, fb) == 0
    assert b.flush() == 0
    got_a = [(t, p) for t, _, p in a.events if t == "message"]
    got_b = [(t, p) for t, _, p in bb.events if t == "message"]
    assert got_a == [("message", bytes(range(200)) * 3)]
    assert got_b == [("message", b"B" * 333)]
    b.close()
    for c in (a, bb, other):
        c.close()


@pytest.mark.parametrize("device", DEVICES)
def test_alloc_read_hands_out_the_room_left(device):
    """with some room left in the accumulating queue, alloc_read hands out that room
    (shorter than libuv's 64 KiB suggestion) instead of handing the queue over and waiting; a
    bogus suggestion is bounded on the direct path (no exception through the C ABI)"""
    _need_device(device)
    import uvhttp_amd as U
    b = U.Batcher(device=device, min_device_bytes=0, max_bytes=48 * 1024)
    key = b"\x01\x02\x03\x04"
    c1 = U.WsConnection(1, 16 << 20, 64 << 20, user_data=False)
    assert b.submit(c1, _frame(2, 1, b"x" * 30000, key, True, 0)) == 0
    flushes = b.stats()["flushes"]
    rc, addr, n = b.alloc(c1, 65536)
    assert rc == 0 and 0 < n < 65536
    assert b.stats()["flushes"] == flushes  # no hand-over for a read that still has room
    assert b.commit(c1, 0) == 0
    # a huge suggestion on a queue with no room: the direct buffer stays bounded
    big = U.WsConnection(1, 16 << 20, 64 << 20, user_data=False)
    rc, addr, n = b.alloc(big, 1 << 62)
    assert rc == 0 and n <= 48 * 1024
    assert b.commit(big, 0) == 0
    assert b.flush() == 0
    assert [(t, p) for t, _, p in c1.events if t == "message"] == [("message", b"x" * 30000)]
    b.close()
    c1.close()
    big.close()
