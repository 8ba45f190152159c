"""TLS connections end to end on the device: record open (include/uvhttp_tls_amd.h) feeding the
WebSocket stream decode (include/uvhttp_ws_amd.h) — the on_websocket_read TLS branch of the
reference (src/uvhttp_connection.c:1122-1159: mbedtls_ssl_read, then uvhttp_ws_process_data on
each decrypted chunk) for many connections in two device calls.

Each connection's client WebSocket frames are cut into TLS records at random points (frames
straddle records), sealed with the CPU oracle under its own key (TLS 1.3 and 1.2, AES-128-GCM,
AES-256-GCM and ChaCha20-Poly1305), and the ciphertext may end inside a record.  The device opens the records; each
connection's plaintext (contiguous at its out_off) is handed as that connection's wire stream
to uvhttp_ws_gpu_decode_streams; uvhttp_ws_deliver_stream replays the callbacks.  The oracle
side: tls_oracle.c opens the same records and oracle process_data decodes the plaintext.  Both
transcripts must match exactly."""
import ctypes as C
import random

import numpy as np
import pytest

import _oracle as O
from test_gpu_parity import _frame

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _ws_frames(rng, n):
    out, open_msg = [], False
    for _ in range(n):
        key = rng.randbytes(4)
        if rng.random() < 0.1:
            out.append(_frame(9, 1, rng.randbytes(rng.choice([0, 5, 125])), key, True, 0))
            continue
        payload = rng.randbytes(rng.choice([0, 1, 100, 125, 126, 3000, 20000, 70000]))
        op = 0 if open_msg else rng.choice([1, 2])
        fin = rng.random() < 0.6
        open_msg = not fin
        out.append(_frame(op, int(fin), payload, key, True, 0))
    return b"".join(out)


@pytest.mark.parametrize("seed", range(3))
def test_tls_then_websocket(torch, seed):
    import uvhttp_amd as U
    t = torch
    rng = random.Random(4242 + seed)
    n_conn = [6, 40, 120][seed]
    ciphers = [(16, O.AES_GCM), (32, O.AES_GCM), (32, O.CHACHA)]
    keys = np.concatenate([O.tls_key(rng.randbytes(kl), rng.randbytes(12), rng.choice([O.TLS13, O.TLS12]), c)
                           for kl, c in (rng.choice(ciphers) for _ in range(n_conn))])
    wire, st = bytearray(), np.zeros(n_conn, O.TLS_STREAM_DT)
    for c in range(n_conn):
        plain = _ws_frames(rng, rng.randint(0, 12))
        seq = rng.randrange(1 << 40)
        begin = len(wire)
        pos, j = 0, 0
        while pos < len(plain):
            n = min(len(plain) - pos, rng.choice([1, 7, 500, 4096, 16384]))
            pad = rng.choice([0, 0, 40]) if keys[c]["version"] == O.TLS13 else 0
            wire += O.tls_seal(keys[c:c + 1], seq + j, 23, plain[pos:pos + n], pad)
            pos += n
            j += 1
        if rng.random() < 0.3 and len(wire) > begin:
            wire = wire[:len(wire) - rng.randint(1, min(30, len(wire) - begin))]  # cut mid-record
        st[c] = (begin, len(wire) - begin, seq, c, 0)
    w = np.frombuffer(bytes(wire), np.uint8)

    # oracle: TLS open, then process_data on each connection's plaintext
    o_recs, o_res, o_out = O.tls_open_batch(w, keys, st)

    # device: TLS open ...
    eng_t = U.TlsEngine(0)
    dev = lambda a: t.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to("cuda")  # noqa: E731
    out = t.zeros(max(16, w.size + 64), dtype=t.uint8, device="cuda")
    recs, res = eng_t.open_records(dev(w) if w.size else t.zeros(16, dtype=t.uint8, device="cuda"),
                                   dev(keys), n_conn, dev(st), n_conn, max(1, w.size // 5 + 1),
                                   out[:max(16, w.size)], wire_len=w.size)
    t.cuda.synchronize()
    R = res.cpu().numpy().view(O.TLS_RESULT_DT)[:n_conn]
    assert R.tobytes() == o_res.tobytes()

    # ... then the WebSocket stream decode over the plaintext the TLS call left in `out`
    eng_w = U.GpuEngine(0)
    conns, streams = [], []
    for c in range(n_conn):
        prod = U.WsConnection(1, 16 * 1024 * 1024, 64 * 1024 * 1024, user_data=False)
        s = U.Stream()
        U.lib().uvhttp_ws_stream_init(prod.ptr, int(R[c]["out_off"]), int(R[c]["plain_len"]),
                                      C.byref(s))
        conns.append(prod)
        streams.append(s)
    sdev = t.from_numpy(np.frombuffer(b"".join(bytes(s) for s in streams), np.uint8).copy()).to("cuda")
    max_frames = 8192
    desc, wres = eng_w.decode_streams(out, sdev, n_conn, max_frames)
    t.cuda.synchronize()
    results = eng_w.read_stream_results(wres, n_conn)
    host_out, host_desc = out.cpu().numpy(), desc.cpu().numpy()
    hw = (C.c_uint8 * host_out.size).from_buffer(host_out)
    hd = (C.c_uint8 * host_desc.size).from_buffer(host_desc)
    for c in range(n_conn):
        rc = U.lib().uvhttp_ws_deliver_stream(conns[c].ptr, hw, hd, C.byref(streams[c]),
                                              C.byref(results[c]))
        orc = O.OracleConn(1, 16 * 1024 * 1024, 64 * 1024 * 1024, record=1)
        r = o_res[c]
        plain = o_out[r["out_off"]:r["out_off"] + r["plain_len"]].tobytes()
        assert rc == orc.process_data(plain), c
        pev = [(k, a, p) for k, a, p in conns[c].events if k in ("message", "close")]
        oev = [(k, a, p if k == "message" else None) for k, a, p in orc.events()
               if k in ("message", "close")]
        assert pev == oev, c
    eng_w.close()
    eng_t.close()
