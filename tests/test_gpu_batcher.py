"""The batcher on the device (include/uvhttp_ws_amd.h, uvhttp_ws_amd_batcher_*): live reads of
many connections reach the MI355X in one decode per flush, and every connection ends exactly
where the reference's process_data-per-read leaves it (src/uvhttp_connection.c:1098-1175).

* C1 harness (tests/c/c1_echo.c) with --batch 1 --device 0 --threshold 0: the libuv echo
  server's reads all go through device flushes; the echo streams equal the direct
  (process_data per read) run, and the batcher's counters prove the device decoded them.
* Python-level: random connections (fragments, control frames, partial frames buffered from
  earlier reads, header / fragment violations) fed as interleaved reads over several flushes;
  per connection: failure rc, transcript, recv-buffer bytes / size and fragment state vs the
  oracle fed the same reads.
"""
import ctypes as C
import json
import os
import random
import subprocess

import pytest

import _oracle
from test_gpu_streams import _frames

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _c1(*args):
    exe = os.path.join(REPO, "tests", "c", "_build", "c1_echo")
    p = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("async_", [0, 1])
@pytest.mark.parametrize("clients,frames,size,chunk", [(16, 40, 3000, 777), (4, 6, 70000, 5000),
                                                       (1, 1, 1024, 1032)])
def test_c1_echo_through_device_batcher(torch, clients, frames, size, chunk, async_):
    """async_ = 1: flush_async from uv_check, delivery from a uv_async_t that the batcher's
    on_ready (a HIP host callback) signals — the loop never waits for the device"""
    args = ("--clients", clients, "--frames", frames, "--size", size, "--chunk", chunk,
            "--seed", 11)
    direct = _c1(*args)
    dev = _c1(*args, "--batch", 1, "--device", 0, "--threshold", 0, "--async", async_)
    assert all(c["match"] for c in dev["clients"]) and dev["errors"] == 0
    assert [c["echo_fnv"] for c in dev["clients"]] == [c["echo_fnv"] for c in direct["clients"]]
    assert dev["device_flushes"] > 0 and dev["device_reads"] == dev["reads"]
    assert dev["host_reads"] == 0 and dev["device_frames"] >= clients * frames


@pytest.mark.parametrize("async_", [0, 1])
def test_batcher_random_connections_vs_oracle(torch, async_):
    import uvhttp_amd as U
    rng = random.Random(2024)
    b = U.Batcher(device=0, min_device_bytes=0)
    conns = []
    for k in range(120):
        mf = rng.choice([16 * 1024 * 1024, 65536, 4000])
        mm = rng.choice([64 * 1024 * 1024, 9000, 0])
        prod = U.WsConnection(1, mf, mm, user_data=False)
        orc = _oracle.OracleConn(1, mf, mm, record=1)
        frames, _ = _frames(rng, rng.randint(0, 14), False, bad=k % 3 == 0)
        data = b"".join(frames)
        reads, pos = [], 0
        while pos < len(data):
            n = rng.choice([1, 7, 300, 4096, 16384, rng.randint(1, 20000)])
            reads.append(data[pos:pos + n])
            pos += n
        conns.append([prod, orc, reads, 0, None])  # next read, oracle rc
    flushes = 0
    while any(c[3] < len(c[2]) for c in conns):
        # a loop iteration: some connections get a read each, in random order
        for c in rng.sample(conns, len(conns)):
            prod, orc, reads, nxt, _ = c
            if nxt >= len(reads) or rng.random() < 0.3:
                continue
            c[3] += 1
            if c[4] is not None:  # the reference closed it already
                continue
            rc = b.submit(prod, reads[nxt])
            if rc != 0:  # earlier reads failed (reported at a flush)
                c[4] = ("submit", rc)
                continue
            orc_rc = orc.process_data(reads[nxt])
            if orc_rc != 0:
                c[4] = ("oracle", orc_rc)
        if async_:
            assert b.poll() in (0, 1)
            assert b.flush_async() == 0
        else:
            assert b.flush() == 0
        flushes += 1
    assert b.flush() == 0
    st = b.stats()
    assert 0 < st["device_flushes"] == st["flushes"] <= flushes + 1  # (empty flushes do nothing)
    assert st["host_reads"] == 0 and st["device_reads"] > 0
    L = _oracle.load()
    for prod, orc, reads, _, end in conns:
        failed = C.addressof(prod.ptr.contents) in b.failures
        assert failed == (end is not None), end
        if failed:
            assert b.failures[C.addressof(prod.ptr.contents)] == -1
        pev = [(t, a, p) for t, a, p in prod.events if t in ("message", "close")]
        oev = [(t, a, p if t == "message" else None) for t, a, p in orc.events()
               if t in ("message", "close")]
        assert pev == oev
        s = prod.struct
        assert s.recv_buffer_pos == orc.recv_pos
        assert C.string_at(s.recv_buffer, s.recv_buffer_pos) == orc.recv_bytes()
        assert s.recv_buffer_size == orc.recv_size
        assert (s.fragmented_size if s.fragmented_message else 0) == L.oracle_conn_frag_size(orc.c)
        assert s.fragmented_opcode == orc.frag_opcode
    b.close()
