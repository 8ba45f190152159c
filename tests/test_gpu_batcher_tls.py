"""TLS connections through the batcher (uvhttp_ws_amd_batcher_set_tls / submit_tls_read): the
on_websocket_read TLS branch of the reference (src/uvhttp_connection.c:1122-1159:
mbedtls_ssl_read until WANT_READ, process_data on every decrypted chunk, close on errors)
for many connections at once, with libuv-sized ciphertext reads cut anywhere (records
straddle reads and flushes: the batcher keeps the unconsumed bytes).

Each connection's client WebSocket frames are cut into TLS records (TLS 1.3 / 1.2,
AES-128-GCM / AES-256-GCM / ChaCha20-Poly1305) sealed by the CPU oracle; some connections
already buffer a partial frame; some carry an alert record mid-stream (the batcher must hand
the rest of the ciphertext back for mbedtls, with the next sequence number), some a corrupted
record (bad MAC: the connection fails, as the reference closes it).  Expected outcome per
connection: the oracle opens the whole ciphertext stream (tls_oracle.c) and runs
process_data once per delivered record until a call fails.  Transcripts, failures, hand-back
bytes / sequence numbers and the recv-buffer / fragment state must match exactly."""
import ctypes as C
import random

import numpy as np
import pytest

import _oracle as O
from test_gpu_parity import _frame
from test_gpu_tls_ws_chain import _ws_frames

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


class TlsConn:
    def __init__(self, U, rng, kind):
        mf, mm = 16 * 1024 * 1024, 64 * 1024 * 1024
        self.prod = U.WsConnection(1, mf, mm, user_data=False)
        self.orc = O.OracleConn(1, mf, mm, record=1)
        kl, cipher = rng.choice([(16, O.AES_GCM), (32, O.AES_GCM), (32, O.CHACHA)])
        self.key = O.tls_key(rng.randbytes(kl), rng.randbytes(12), rng.choice([O.TLS13, O.TLS12]), cipher)
        self.seq0 = rng.randrange(1 << 40)
        if rng.random() < 0.3:  # a partial frame buffered by an earlier (plain) read
            tail = _frame(2, 1, rng.randbytes(rng.choice([10, 300, 3000])), b"\x01\x02\x03\x04")
            cut = rng.randint(1, len(tail) - 1)
            assert self.prod.process_data(tail[:cut]) == 0 == self.orc.process_data(tail[:cut])
            plain = tail[cut:] + _ws_frames(rng, rng.randint(1, 10))
        else:
            plain = _ws_frames(rng, rng.randint(0, 10))
        recs, pos, j = [], 0, 0
        while pos < len(plain):
            n = min(len(plain) - pos, rng.choice([1, 7, 500, 4096, 16384]))
            pad = rng.choice([0, 0, 40]) if self.key[0]["version"] == O.TLS13 else 0
            recs.append(O.tls_seal(self.key, self.seq0 + j, 23, plain[pos:pos + n], pad))
            pos += n
            j += 1
        if kind == "alert" and recs:  # close_notify-like alert record somewhere in the stream
            at = rng.randrange(len(recs) + 1)
            alert = O.tls_seal(self.key, self.seq0 + at, 21, b"\x01\x00")
            # records after it keep their own sequence numbers (they follow the alert)
            recs = recs[:at] + [alert] + [O.tls_seal(self.key, self.seq0 + at + 1 + k, 23, b"late" * 5)
                                          for k in range(2)]
        if kind == "corrupt" and recs:
            at = rng.randrange(len(recs))
            r = bytearray(recs[at])
            r[-1] ^= 0x40  # tag byte
            recs[at] = bytes(r)
        self.cipher = b"".join(recs)
        if kind == "cut" and self.cipher:
            self.cipher = self.cipher[:len(self.cipher) - rng.randint(1, min(30, len(self.cipher)))]
        reads, pos = [], 0
        while pos < len(self.cipher):
            n = rng.choice([1, 5, 300, 4096, 16384, rng.randint(1, 40000)])
            reads.append(self.cipher[pos:pos + n])
            pos += n
        self.reads, self.next = reads, 0
        self.kept = b""       # reads the batcher refused after a hand-back (the caller's mbedtls)
        self.refused = False

    def expected(self):
        st = np.zeros(1, O.TLS_STREAM_DT)
        st[0] = (0, len(self.cipher), self.seq0, 0, 0)
        w = np.frombuffer(self.cipher or b"\0", np.uint8)[:len(self.cipher)]
        recs, res, out = O.tls_open_batch(w, self.key, st, out_cap=max(16, w.size))
        r = res[0]
        reads = []
        for j in range(r["n_delivered"]):
            rec = recs[r["first_record"] + j]
            reads.append(out[rec["out_off"]:rec["out_off"] + rec["content_len"]].tobytes())
        ws_rc, _ = self.orc.process_reads(reads) if reads else (0, 0)
        return r, ws_rc


@pytest.mark.parametrize("seed", range(3))
def test_tls_connections_through_batcher(torch, seed):
    import uvhttp_amd as U
    rng = random.Random(7100 + seed)
    b = U.Batcher(device=0, min_device_bytes=1 << 20, max_bytes=[1 << 20, 8 << 20, 64 << 20][seed])
    kinds = ["ok"] * 6 + ["alert", "corrupt", "cut"]
    conns = [TlsConn(U, rng, rng.choice(kinds)) for _ in range(36)]
    for c in conns:
        assert b.set_tls(c.prod, c.key.tobytes(), c.seq0) == 0
    while any(c.next < len(c.reads) for c in conns):
        for c in rng.sample(conns, len(conns)):
            if c.next >= len(c.reads) or rng.random() < 0.3:
                continue
            data = c.reads[c.next]
            c.next += 1
            if c.refused:
                c.kept += data
                continue
            rc = b.submit_tls(c.prod, data)
            if rc != 0:  # handed back (or failed) at an earlier flush: the caller keeps it
                c.refused = True
                c.kept += data
        act = rng.random()
        if act < 0.3:
            assert b.flush() in (0,)
        elif act < 0.7:
            assert b.flush_async() == 0
        else:
            assert b.poll() in (0, 1)
    assert b.flush() == 0
    st = b.stats()
    assert st["tls_records"] > 0 and st["host_reads"] == 0
    L = O.load()
    for c in conns:
        key = C.addressof(c.prod.ptr.contents)
        r, ws_rc = c.expected()
        info = (r, ws_rc, len(c.cipher))
        if r["first_status"] == O.REC_CONTROL and ws_rc == 0:
            data, next_seq, status = b.handbacks[key]
            assert status == O.REC_CONTROL and next_seq == c.seq0 + int(r["n_delivered"]), info
            assert data + c.kept == c.cipher[int(r["consumed_bytes"]):], info
        else:
            assert key not in b.handbacks, info
        failed = key in b.failures
        assert failed == (ws_rc != 0 or int(r["status"]) != 0), info
        pev = [(k, a, p) for k, a, p in c.prod.events if k in ("message", "close")]
        oev = [(k, a, p if k == "message" else None) for k, a, p in c.orc.events()
               if k in ("message", "close")]
        assert pev == oev, info
        s_ = c.prod.struct
        assert s_.recv_buffer_pos == c.orc.recv_pos, info
        assert C.string_at(s_.recv_buffer, s_.recv_buffer_pos) == c.orc.recv_bytes(), info
        assert s_.recv_buffer_size == c.orc.recv_size, info
        frag = s_.fragmented_size if s_.fragmented_message else 0
        assert frag == L.oracle_conn_frag_size(c.orc.c), info
    b.close()


def test_tls_rules(torch):
    """host-only batchers refuse TLS; plain reads on a TLS connection are refused"""
    import uvhttp_amd as U
    host = U.Batcher(device=-1)
    c = U.WsConnection(1)
    key = O.tls_key(bytes(16), bytes(12), O.TLS13).tobytes()
    assert host.set_tls(c, key, 0) == -2  # ENODEV
    dev = U.Batcher(device=0, min_device_bytes=0)
    assert dev.set_tls(c, key, 0) == 0
    assert dev.submit(c, b"\x81\x80abcd") == -1
    d = U.WsConnection(1)
    assert dev.submit_tls(d, b"\x17\x03\x03") == -1  # not registered
    dev.close()
    host.close()


def _seal_stream(rng, key, seq0, plain, rec=16384):
    recs, pos, j = [], 0, 0
    while pos < len(plain):
        n = min(len(plain) - pos, rec)
        recs.append(O.tls_seal(key, seq0 + j, 23, plain[pos:pos + n]))
        pos += n
        j += 1
    return b"".join(recs)


@pytest.mark.parametrize("pattern", ["async", "sync"])
def test_tls_bulk_upload_larger_than_flushes(torch, pattern):
    """ONE TLS connection sending far more than a flush holds (a bulk upload, > 2 x max_bytes),
    in reads up to 1.5 x max_bytes, while earlier queues are still in flight: every read is
    taken (the in-flight queue's bytes made the staging bound refuse it before),
    and the connection sees exactly the oracle's process_data per record."""
    import uvhttp_amd as U
    rng = random.Random(4400 + len(pattern))
    mb = 1 << 20
    b = U.Batcher(device=0, min_device_bytes=0, max_bytes=mb)
    key = O.tls_key(rng.randbytes(16), rng.randbytes(12), O.TLS13, O.AES_GCM)
    seq0 = 77
    mf, mm = 16 * 1024 * 1024, 64 * 1024 * 1024
    prod = U.WsConnection(1, mf, mm)
    orc = O.OracleConn(1, mf, mm, record=1)
    sizes = [1000, 300000, 300000] * 4 + [60000, 300000]  # 14 frames, 2.76 MB
    plain = b"".join(_frame(2, 1, rng.randbytes(p), rng.randbytes(4)) for p in sizes)
    cipher = _seal_stream(rng, key, seq0, plain)
    assert len(cipher) > 2 * mb
    assert b.set_tls(prod, key.tobytes(), seq0) == 0
    pos = 0
    while pos < len(cipher):
        n = rng.choice([16384, 200000, mb // 2, mb + mb // 2])
        assert b.submit_tls(prod, cipher[pos:pos + n]) == 0, pos
        pos += n
        if pattern == "async":
            assert b.flush_async() == 0
            assert b.poll() in (0, 1)
    assert b.flush() == 0
    key_ = C.addressof(prod.ptr.contents)
    assert key_ not in b.failures and key_ not in b.handbacks
    st = np.zeros(1, O.TLS_STREAM_DT)
    st[0] = (0, len(cipher), seq0, 0, 0)
    recs, res, out = O.tls_open_batch(np.frombuffer(cipher, np.uint8), key, st, out_cap=len(cipher))
    reads = [out[r["out_off"]:r["out_off"] + r["content_len"]].tobytes()
             for r in recs[:int(res[0]["n_delivered"])]]
    assert orc.process_reads(reads)[0] == 0
    pev = [(k, a, p) for k, a, p in prod.events if k == "message"]
    oev = [(k, a, p) for k, a, p in orc.events() if k == "message"]
    assert len(pev) == 14 and pev == oev
    b.close()


def test_tls_device_error_hands_ciphertext_back(torch, monkeypatch):
    """A device or launch error on a queue holding TLS connections (injected: every launch
    fails) neither fails nor closes them: their ciphertext — all of it from the next record on
    — goes back to the caller for mbedtls (status UVHTTP_WS_BATCHER_HANDBACK_DEVICE = -100,
    ADVICE r03); plain connections of the same queue are decoded by the host decoder."""
    import uvhttp_amd as U
    monkeypatch.setenv("UVHTTP_WS_BATCHER_FAIL_EVERY", "1")
    rng = random.Random(4500)
    b = U.Batcher(device=0, min_device_bytes=0, max_bytes=4 << 20, library=U.test_hooks_library())
    monkeypatch.delenv("UVHTTP_WS_BATCHER_FAIL_EVERY")
    conns = []
    for k in range(5):
        key = O.tls_key(rng.randbytes(32), rng.randbytes(12), O.TLS12, O.CHACHA)
        prod = U.WsConnection(1)
        cipher = _seal_stream(rng, key, 1000 * k, _ws_frames(rng, 6), rec=700)
        assert b.set_tls(prod, key.tobytes(), 1000 * k) == 0
        conns.append((prod, cipher, 1000 * k))
    plain_conn = U.WsConnection(1)
    orc = O.OracleConn(1, record=1)
    pf = _ws_frames(rng, 5)
    for prod, cipher, _ in conns:
        cut = len(cipher) // 3
        assert b.submit_tls(prod, cipher[:cut]) == 0
        assert b.submit_tls(prod, cipher[cut:]) == 0
    assert b.submit(plain_conn, pf) == 0
    rc = b.flush()
    assert rc == -4  # ELAUNCH: the injected device error, reported
    assert orc.process_data(pf) == 0
    assert [e for e in plain_conn.events if e[0] == "message"] == \
        [e for e in orc.events() if e[0] == "message"]
    for prod, cipher, seq in conns:
        key_ = C.addressof(prod.ptr.contents)
        assert key_ not in b.failures
        data, next_seq, status = b.handbacks[key_]
        assert status == -100 and next_seq == seq and data == cipher
        assert not [e for e in prod.events if e[0] == "message"]
    st = b.stats()
    assert st["device_errors"] == 1 and st["tls_handbacks"] == 5
    b.close()


def test_set_tls_inside_callback_with_queued_plain_reads(torch):
    """set_tls from a batcher callback while the connection still has plain reads queued cannot
    flush them first: it is refused (EINVAL) instead of registering a TLS connection whose plain
    reads would then be unreachable; after the flush it succeeds."""
    import uvhttp_amd as U
    b = U.Batcher(device=0, min_device_bytes=0)
    a, c = U.WsConnection(1), U.WsConnection(1)
    key = O.tls_key(bytes(range(16)), bytes(12), O.TLS13).tobytes()
    seen = []

    def hook(conn, ev):
        if not seen:
            seen.append(b.set_tls(c, key, 5))

    a.hook = hook
    assert b.submit(a, _frame(2, 1, b"first", b"\x01\x02\x03\x04")) == 0
    assert b.submit(c, _frame(2, 1, b"second", b"\x05\x06\x07\x08")) == 0
    assert b.flush() == 0
    assert seen == [-1]
    assert [e[2] for e in c.events if e[0] == "message"] == [b"second"]
    assert b.set_tls(c, key, 5) == 0
    b.close()
