"""TLS record open / seal on the MI355X against the CPU oracle
(oracle/tls_oracle.c): OpenSSL-written sessions, randomized multi-connection batches with every
stop rule of include/uvhttp_tls_amd.h, device seal vs oracle seal byte for byte, and a large
seal -> open round trip — AES-128/256-GCM and ChaCha20-Poly1305, TLS 1.3 and 1.2.  Bit-exact:
records, connection results and the delivered plaintext."""
import base64
import hashlib
import json
import os
import random

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def eng(torch):
    import uvhttp_amd as U
    e = U.TlsEngine(0)
    yield e
    e.close()


def _dev(torch, a):
    b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    if b.size == 0:
        b = np.zeros(16, np.uint8)
    return torch.from_numpy(b.copy()).to("cuda")


def _run(torch, eng, wire, keys, streams, max_records=None, out_cap=None):
    w = np.ascontiguousarray(wire, np.uint8)
    max_records = max(1, w.size // 5 + 1) if max_records is None else max_records
    out_cap = w.size if out_cap is None else out_cap
    out = torch.zeros(max(16, out_cap), dtype=torch.uint8, device="cuda")
    recs, res = eng.open_records(_dev(torch, w), _dev(torch, keys), len(keys),
                                 _dev(torch, streams), len(streams), max_records,
                                 out[:out_cap] if out_cap else out[:0], wire_len=w.size)
    torch.cuda.synchronize()
    R = res.cpu().numpy().view(O.TLS_RESULT_DT)[:len(streams)]
    n = int(R["n_records"].sum()) if len(R) else 0
    D = recs.cpu().numpy().view(O.TLS_RECORD_DT)[:n]
    return D, R, out.cpu().numpy()


def check(torch, eng, wire, keys, streams, max_records=None, out_cap=None):
    ro, so, oo = O.tls_open_batch(wire, keys, streams, max_records, out_cap)
    rd, sd, od = _run(torch, eng, wire, keys, streams, max_records, out_cap)
    assert so.tobytes() == sd.tobytes(), (so, sd)
    assert ro.tobytes() == rd.tobytes(), (ro, rd)
    for r in so:
        a, b = int(r["out_off"]), int(r["out_off"] + r["plain_len"])
        assert np.array_equal(oo[a:b], od[a:b])
    return ro, so, oo


def _sessions():
    with open(os.path.join(GOLD, "tls_openssl_records.json")) as f:
        return json.load(f)["sessions"]


def test_openssl_sessions(torch, eng):
    """Every OpenSSL session alone, then all seven in one batch (seven keys: both versions,
    AES-GCM and ChaCha20-Poly1305)."""
    wires, keys, sts = [], [], []
    base = 0
    for i, s in enumerate(_sessions()):
        w = np.frombuffer(base64.b64decode(s["wire_b64"]), np.uint8)
        k = O.tls_key(bytes.fromhex(s["key"]), bytes.fromhex(s["iv"]), s["version"],
                      s.get("cipher", 0))
        st = np.zeros(1, O.TLS_STREAM_DT)
        st[0]["len"], st[0]["seq"] = w.size, s["seq"]
        _, so, oo = check(torch, eng, w, k, st)
        r = so[0]
        assert hashlib.sha256(oo[r["out_off"]:r["out_off"] + r["plain_len"]].tobytes()).hexdigest() \
            == s["plaintext_sha256"]
        st[0]["begin"], st[0]["key"] = base, i
        wires.append(w)
        keys.append(k)
        sts.append(st)
        base += w.size
    check(torch, eng, np.concatenate(wires), np.concatenate(keys), np.concatenate(sts))


def _key_set(rng):
    """AES-128-GCM, AES-256-GCM, ChaCha20-Poly1305 x TLS 1.3, TLS 1.2"""
    return np.concatenate([O.tls_key(rng.randbytes(kl), rng.randbytes(12), v, c)
                           for kl, c in ((16, O.AES_GCM), (32, O.AES_GCM), (32, O.CHACHA))
                           for v in (O.TLS13, O.TLS12)])


def _random_batch(seed, n_streams, sizes, faults=True):
    rng = random.Random(seed)
    keys = _key_set(rng)
    wire, st = bytearray(), np.zeros(n_streams, O.TLS_STREAM_DT)
    for s in range(n_streams):
        k = rng.randrange(len(keys))
        kr = keys[k:k + 1]
        v = int(kr[0]["version"])
        seq = rng.randrange(1 << 48)
        begin = len(wire)
        for j in range(rng.randint(0, 5)):
            c = rng.randbytes(rng.choice(sizes))
            t = 23 if not faults or rng.random() < 0.9 else rng.choice([21, 22])
            pad = rng.choice([0, 0, 0, 1, 33, 300]) if v == O.TLS13 else 0
            if v == O.TLS13 and t != 23:
                pad = 0
            rec = bytearray(O.tls_seal(kr, seq + j, t, c, pad))
            if faults and rng.random() < 0.05:
                rec[rng.randrange(len(rec))] ^= 1 << rng.randrange(8)  # corrupt anywhere
            wire += rec
        if faults:
            wire += rng.choice([b"", b"", b"\x17", b"\x17\x03\x03", b"\x17\x03\x03\x00\x20abc"])
        st[s]["begin"], st[s]["len"], st[s]["seq"], st[s]["key"] = begin, len(wire) - begin, seq, k
    return np.frombuffer(bytes(wire), np.uint8), keys, st


@pytest.mark.parametrize("seed", range(6))
def test_random_batches(torch, eng, seed):
    sizes = [[0, 1, 15, 16, 17, 31, 33, 100, 255], [1000, 4095, 4096, 8191, 16383, 16384],
             [0, 7, 16384, 2000, 64]][seed % 3]
    wire, keys, st = _random_batch(seed, [1, 7, 64, 300, 33, 129][seed], sizes)
    check(torch, eng, wire, keys, st)


def test_key_and_capacity_errors(torch, eng):
    wire, keys, st = _random_batch(77, 20, [50, 500], faults=False)
    keys[1]["key_len"] = 24      # invalid key length
    keys[2]["version"] = 0x0302  # invalid version
    keys[5]["key_len"] = 16      # ChaCha20-Poly1305 with a 16-byte key
    keys[4]["cipher"] = 7        # unknown cipher
    st[3]["key"] = 99            # slot out of range
    check(torch, eng, wire, keys, st)
    n = int(O.tls_open_batch(wire, keys, st)[1]["n_records"].sum())
    check(torch, eng, wire, keys, st, max_records=max(1, n - 1))  # too many records
    check(torch, eng, wire, keys, st, out_cap=100)                # layout over capacity


def test_key_slot_cache(torch, eng):
    """k_tls_keys keeps a slot's schedule when the same key comes again: a repeated batch, a
    changed iv byte, a slot made invalid and then valid again, and keys moved between slots
    must all open exactly as the oracle does."""
    wire, keys, st = _random_batch(91, 40, [100, 3000, 16384], faults=False)
    check(torch, eng, wire, keys, st)
    check(torch, eng, wire, keys, st)                  # every slot cached
    k2 = keys.copy()
    k2[0]["iv"][5] ^= 1                                # same key bytes, other iv: rebuilt
    check(torch, eng, wire, k2, st)
    k3 = keys.copy()
    k3[3]["key_len"] = 24                              # invalid ...
    check(torch, eng, wire, k3, st)
    check(torch, eng, wire, keys, st)                  # ... and valid again
    perm = np.roll(np.arange(len(keys)), 1)            # keys moved between slots
    st2 = st.copy()
    st2["key"] = perm[st["key"]]
    k4 = keys.copy()
    k4[perm] = keys
    check(torch, eng, wire, k4, st2)


def _seal_dev(torch, eng, src, descs, keys, out_bytes):
    out = torch.zeros(out_bytes, dtype=torch.uint8, device="cuda")
    eng.seal_records(_dev(torch, src), _dev(torch, descs), len(descs), _dev(torch, keys),
                     len(keys), out)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_seal_matches_oracle(torch, eng):
    rng = random.Random(9)
    keys = _key_set(rng)
    src = np.frombuffer(rng.randbytes(1 << 18), np.uint8)
    sizes = [0, 1, 15, 16, 17, 100, 1023, 4096, 16383, 16384]
    n = 200
    descs = np.zeros(n, O.TLS_SEAL_DT)
    expect, off = [], 0
    for i in range(n):
        k = rng.randrange(len(keys))
        ln = rng.choice(sizes)
        so = rng.randrange(src.size - ln + 1)
        t = rng.choice([23, 23, 21, 22])
        seq = rng.randrange(1 << 62)
        rec = O.tls_seal(keys[k:k + 1], seq, t, src[so:so + ln].tobytes())
        descs[i] = (so, off, seq, ln, k, t, 0)
        expect.append((off, rec))
        off += len(rec) + rng.choice([0, 3, 16])
    got = _seal_dev(torch, eng, src, descs, keys, off + 64)
    for o, rec in expect:
        assert got[o:o + len(rec)].tobytes() == rec


def test_seal_open_roundtrip_large(torch, eng):
    """4096 connections x 4 full records sealed on the device, opened on the device: the
    delivered plaintext equals the source (size-independent round trip)."""
    t = torch
    rng = random.Random(21)
    n_conn, per = 4096, 4
    keys = np.concatenate([O.tls_key(rng.randbytes(16 if i % 2 and i % 5 else 32), rng.randbytes(12),
                                     O.TLS13 if i % 3 else O.TLS12,
                                     O.AES_GCM if i % 5 else O.CHACHA) for i in range(n_conn)])
    plen = 16384
    src = t.randint(0, 256, (n_conn * per * plen,), dtype=t.uint8, device="cuda")
    descs = np.zeros(n_conn * per, O.TLS_SEAL_DT)
    st = np.zeros(n_conn, O.TLS_STREAM_DT)
    off = 0
    for c in range(n_conn):
        v = int(keys[c]["version"])
        rl = 5 + plen + 16 + (1 if v == O.TLS13 else 8 if keys[c]["cipher"] == O.AES_GCM else 0)
        st[c] = (off, rl * per, 1000 + c, c, 0)
        for j in range(per):
            i = c * per + j
            descs[i] = (i * plen, off, 1000 + c + j, plen, c, 23, 0)
            off += rl
    wire = t.zeros(off, dtype=t.uint8, device="cuda")
    dk = _dev(t, keys)
    eng.seal_records(src, _dev(t, descs), len(descs), dk, n_conn, wire)
    out = t.zeros(off, dtype=t.uint8, device="cuda")
    recs, res = eng.open_records(wire, dk, n_conn, _dev(t, st), n_conn, n_conn * per, out)
    t.cuda.synchronize()
    R = res.cpu().numpy().view(O.TLS_RESULT_DT)
    assert (R["n_delivered"] == per).all() and (R["first_status"] == 0).all()
    assert (R["plain_len"] == per * plen).all()
    got = t.cat([out[int(r["out_off"]):int(r["out_off"]) + per * plen] for r in R])
    assert t.equal(got, src)
