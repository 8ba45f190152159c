"""The batcher group (uvhttp_ws_amd_batcher_group_*): the live path over several devices.

Every connection is pinned to one member for its life, so its reads keep the order the
reference's on_websocket_read gives them (process_data per read until one fails,
src/uvhttp_connection.c:1098-1175) while different connections flush through different members.
Each connection is checked against the oracle fed the same reads: callback transcript, failure,
recv-buffer and fragment state.  Host-decoder members (-1) run here on the CPU; groups with device
members (two members on GPU 0, or a GPU and a host member) are marked gpu."""
import random

import pytest

from test_batcher_transitions import Pair, _conn_reads

GROUPS = [[-1, -1, -1], [-1],
          pytest.param([0, 0], marks=pytest.mark.gpu, id="gpu0x2"),
          pytest.param([0, -1], marks=pytest.mark.gpu, id="gpu0+host")]


def _need(devices):
    if max(devices) >= 0:
        import torch
        if not torch.cuda.is_available():
            pytest.skip("no GPU")


def _drive(b, rng, pairs, forget_some=False):
    while any(p.next < len(p.reads) for p in pairs):
        for p in rng.sample(pairs, len(pairs)):
            if p.next >= len(p.reads) or rng.random() < 0.3:
                continue
            p.feed(b, p.reads[p.next])
            p.next += 1
            if forget_some and not p.dead and rng.random() < 0.01:
                b.forget(p.prod)
                p.dead = True
        act = rng.random()
        if act < 0.3:
            assert b.flush() == 0
        elif act < 0.6:
            assert b.flush_async() == 0
        elif act < 0.8:
            assert b.poll() >= 0
    assert b.flush() == 0
    assert not b.in_flight()


@pytest.mark.parametrize("zc", [False, True], ids=["submit", "zero_copy"])
@pytest.mark.parametrize("devices", GROUPS)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_group_matches_process_data(devices, seed, zc):
    _need(devices)
    import uvhttp_amd as U
    import _oracle
    rng = random.Random(600 + seed)
    b = U.BatcherGroup(devices, min_device_bytes=0, max_bytes=[64 << 10, 1 << 20, 8 << 20][seed - 1],
                       max_connections=64, max_reads=4000)
    assert b.size() == len(devices)
    pairs = [Pair(U, rng, reads=_conn_reads(rng, big=70000 if seed == 1 else 0), zc=zc) for _ in range(45)]
    _drive(b, rng, pairs, forget_some=seed == 3)
    L = _oracle.load()
    for p in pairs:
        p.check(b, L)
    # every member served connections, each connection stayed on its member
    members = [b.member(p.prod) for p in pairs if not p.dead]
    for m in range(len(devices)):
        assert members.count(m) >= 1
    st = b.stats()
    per = [b.member_stats(m)["flushes"] for m in range(len(devices))]
    assert st["flushes"] == sum(per)
    b.close()


def test_group_pinning_and_balance():
    """a connection's first read pins it to the least-loaded member (ties: round robin); it
    stays there across flushes; forget releases its place; member() is a query that never pins"""
    import uvhttp_amd as U
    b = U.BatcherGroup([-1, -1, -1, -1])
    conns = [U.WsConnection(1) for _ in range(10)]
    assert [b.member(c) for c in conns] == [-1] * 10  # asking does not pin
    frame = b"\x82\x85" + b"\x01\x02\x03\x04" + bytes(x ^ k for x, k in zip(b"hello", b"\x01\x02\x03\x04\x01"))
    for c in conns:
        assert b.submit(c, frame) == 0
    ms = [b.member(c) for c in conns]
    assert sorted(ms) == [0, 0, 0, 1, 1, 1, 2, 2, 3, 3]
    assert b.flush() == 0
    assert all([e[2] for e in c.events if e[0] == "message"] == [b"hello"] for c in conns)
    assert [b.member(c) for c in conns] == ms  # pinned across the flush
    b.forget(conns[3])  # its member drops to the fewest connections
    assert b.member(conns[3]) == -1
    fresh = U.WsConnection(1)
    assert b.member(fresh) == -1
    assert b.submit(fresh, frame) == 0 and b.member(fresh) == ms[3]
    assert b.flush() == 0
    b.close()


def test_group_tls_needs_a_device_member():
    """TLS records open only on a device member: in a host-only group set_tls pins nothing and
    returns ENODEV"""
    import uvhttp_amd as U
    b = U.BatcherGroup([-1, -1])
    c = U.WsConnection(1)
    assert b.set_tls(c, bytes(64), 0) == -2
    assert b.member(c) == -1
    b.close()


@pytest.mark.gpu
def test_group_tls_in_a_mixed_group():
    """in a [GPU, host] group every TLS connection goes to the device member — new
    ones, and ones already pinned to the host member that hold nothing there yet (their reads
    were delivered); a connection with reads still queued on the host member stays (ENODEV).
    Each TLS connection's records then decode against the oracle."""
    _need([0])
    import uvhttp_amd as U
    import _oracle as O
    from test_gpu_batcher_tls import _seal_stream
    from test_gpu_tls_ws_chain import _ws_frames
    rng = random.Random(77)
    b = U.BatcherGroup([0, -1], min_device_bytes=0, max_bytes=4 << 20)
    frame = b"\x82\x80" + rng.randbytes(4)
    conns = []
    for k in range(6):
        prod = U.WsConnection(1)
        if k % 2:  # first a plain read, delivered by whichever member it pinned to
            assert b.submit(prod, frame) == 0
            assert b.flush() == 0
        key = O.tls_key(rng.randbytes(16), rng.randbytes(12), O.TLS13, O.AES_GCM)
        assert b.set_tls(prod, key.tobytes(), 0) == 0, k
        assert b.member(prod) == 0
        frames = _ws_frames(rng, 6, small=True)
        cipher = _seal_stream(rng, key, 0, frames, rec=900)
        assert b.submit_tls(prod, cipher) == 0
        conns.append((prod, frames, k % 2))
    # a plain read queued on the host member: that connection cannot move
    busy = [U.WsConnection(1) for _ in range(2)]
    for c in busy:
        assert b.submit(c, frame) == 0
    stuck = [c for c in busy if b.member(c) == 1]
    assert stuck, [b.member(c) for c in busy]
    assert b.set_tls(stuck[0], bytes(64), 0) == -2 and b.member(stuck[0]) == 1
    assert b.flush() == 0
    for prod, frames, pre in conns:
        orc = O.OracleConn(1, record=1)
        if pre:
            assert orc.process_data(frame) == 0
        assert orc.process_data(frames) == 0
        pev = [e for e in prod.events if e[0] == "message"]
        oev = [e for e in orc.events() if e[0] == "message"]
        assert pev == oev and len(pev) >= 1
    b.close()


def test_group_rejects_bad_config():
    import uvhttp_amd as U
    with pytest.raises(U.GpuError):
        U.BatcherGroup([])
