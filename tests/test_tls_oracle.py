"""CPU checks of the TLS record-layer oracle (oracle/tls_oracle.c).

Pins the restatement: AES against FIPS-197 Appendix C, AES-GCM against the GCM
specification's test cases, ChaCha20 / Poly1305 / AEAD_CHACHA20_POLY1305 against RFC 8439's
vectors (tests/golden/tls_known_answers.json), and the TLS record layer (nonces, AAD, TLS 1.3
inner plaintext and padding, TLS 1.2 explicit / implicit nonces) against records a real TLS
stack wrote — OpenSSL 3.0.2 sessions (AES-GCM and ChaCha20-Poly1305, TLS 1.3 and 1.2) captured
by tests/golden/make_tls_vectors.py.
Then the batch contract of include/uvhttp_tls_amd.h case by case.
"""
import base64
import hashlib
import json
import os
import random

import numpy as np
import pytest

import _oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_aes_known_answers():
    ka = _json("tls_known_answers.json")
    for c in ka["aes"]:
        assert O.aes_encrypt_block(bytes.fromhex(c["key"]), bytes.fromhex(c["pt"])).hex() == c["ct"], c["id"]
    for x, y in ka["sbox"].items():
        assert O._tls_sigs(O.load()).oracle_aes_sbox(int(x, 16)) == int(y, 16)


def test_chacha_poly_known_answers():
    ka = _json("tls_known_answers.json")
    for c in ka["chacha20_block"]:
        assert O.chacha20_block(bytes.fromhex(c["key"]), c["counter"],
                                bytes.fromhex(c["nonce"])).hex() == c["out"], c["id"]
    for c in ka["poly1305"]:
        assert O.poly1305(bytes.fromhex(c["key"]), bytes.fromhex(c["msg"])).hex() == c["tag"], c["id"]
    for c in ka["chachapoly"]:
        k, n, aad = bytes.fromhex(c["key"]), bytes.fromhex(c["nonce"]), bytes.fromhex(c["aad"])
        ct, tag = O.chachapoly(k, n, aad, bytes.fromhex(c["pt"]))
        assert (ct.hex(), tag.hex()) == (c["ct"], c["tag"]), c["id"]
        rc, pt = O.chachapoly(k, n, aad, ct, tag, decrypt=True)
        assert rc == 0 and pt.hex() == c["pt"]
        assert O.chachapoly(k, n, aad, ct, bytes([tag[0] ^ 4]) + tag[1:], decrypt=True)[0] == -2


def test_gcm_known_answers():
    for c in _json("tls_known_answers.json")["gcm"]:
        k, iv, aad = bytes.fromhex(c["key"]), bytes.fromhex(c["iv"]), bytes.fromhex(c["aad"])
        ct, tag = O.gcm(k, iv, aad, bytes.fromhex(c["pt"]))
        assert (ct.hex(), tag.hex()) == (c["ct"], c["tag"]), c["id"]
        rc, pt = O.gcm(k, iv, aad, ct, tag, decrypt=True)
        assert rc == 0 and pt.hex() == c["pt"], c["id"]
        bad = bytes([tag[0] ^ 1]) + tag[1:]
        assert O.gcm(k, iv, aad, ct, bad, decrypt=True)[0] == -2, c["id"]


def _session_batch(s):
    wire = np.frombuffer(base64.b64decode(s["wire_b64"]), np.uint8)
    keys = O.tls_key(bytes.fromhex(s["key"]), bytes.fromhex(s["iv"]), s["version"],
                     s.get("cipher", 0))
    st = np.zeros(1, O.TLS_STREAM_DT)
    st[0]["len"], st[0]["seq"] = wire.size, s["seq"]
    return wire, keys, st


@pytest.mark.parametrize("idx", range(7))
def test_openssl_sessions(idx):
    """Records OpenSSL wrote open to exactly what OpenSSL's server read back, and the
    connection stops at the encrypted close_notify alert (CONTROL, type 21)."""
    s = _json("tls_openssl_records.json")["sessions"][idx]
    wire, keys, st = _session_batch(s)
    recs, res, out = O.tls_open_batch(wire, keys, st)
    r = res[0]
    assert r["status"] == 0 and r["first_status"] == O.REC_CONTROL
    assert r["n_records"] == len(recs) == r["n_delivered"] + 1
    assert recs[-1]["type"] == s["stop_type"] and recs[-1]["status"] == O.REC_CONTROL
    assert (recs["status"][:-1] == O.REC_OK).all() and (recs["type"][:-1] == 23).all()
    assert r["plain_len"] == s["plaintext_len"]
    got = out[r["out_off"]:r["out_off"] + r["plain_len"]].tobytes()
    assert hashlib.sha256(got).hexdigest() == s["plaintext_sha256"]
    assert r["consumed_bytes"] == recs[-1]["rec_off"]
    assert r["next_seq"] == s["seq"] + r["n_delivered"]
    if s["padding"]:
        # block padding: inner plaintexts are padded, contents shorter than the reservation
        assert any(int(x["content_len"]) < _cap(wire, x, s["version"], s.get("cipher", 0))
                   for x in recs[:-1])


def _cap(wire, rec, version, cipher=0):
    o = int(rec["rec_off"])
    ln = (int(wire[o + 3]) << 8) | int(wire[o + 4])
    return max(0, ln - _over(version, cipher) - (1 if version == O.TLS13 else 0))


def _mk_key(rng, version, klen=None, cipher=None):
    cipher = rng.choice([O.AES_GCM, O.CHACHA]) if cipher is None else cipher
    klen = 32 if cipher == O.CHACHA else (klen or rng.choice([16, 32]))
    return O.tls_key(rng.randbytes(klen), rng.randbytes(12), version, cipher)


def test_seal_open_roundtrip_many_streams():
    rng = random.Random(3)
    keys = np.concatenate([_mk_key(rng, v) for v in (O.TLS13, O.TLS12, O.TLS13, O.TLS12)])
    wire, streams, expect = b"", [], []
    for s in range(12):
        ks = s % len(keys)
        seq = rng.randrange(1 << 40)
        begin = len(wire)
        content = []
        for j in range(rng.randint(0, 6)):
            c = rng.randbytes(rng.choice([0, 1, 15, 16, 17, 300, 4096, 16384]))
            pad = rng.choice([0, 0, 0, 5, 200]) if keys[ks]["version"] == O.TLS13 else 0
            wire += O.tls_seal(keys[ks:ks + 1], seq + j, 23, c, pad)
            content.append(c)
        tail = rng.choice([b"", b"\x17\x03", b"\x17\x03\x03\x40\x00"])  # incomplete bytes
        wire += tail
        streams.append((begin, len(wire) - begin, seq, ks))
        expect.append(b"".join(content))
    st = np.zeros(len(streams), O.TLS_STREAM_DT)
    for i, (b, ln, sq, k) in enumerate(streams):
        st[i]["begin"], st[i]["len"], st[i]["seq"], st[i]["key"] = b, ln, sq, k
    w = np.frombuffer(wire, np.uint8)
    recs, res, out = O.tls_open_batch(w, keys, st)
    base = 0
    for i, r in enumerate(res):
        assert r["status"] == 0 and r["first_status"] == 0, i
        assert r["out_off"] == base
        assert out[r["out_off"]:r["out_off"] + r["plain_len"]].tobytes() == expect[i]
        mine = recs[recs["stream"] == i]
        kk = keys[streams[i][3]]
        base += sum(_cap(w, x, int(kk["version"]), int(kk["cipher"])) for x in mine)


def _one(version, build, klen=16, seq=7, max_records=None, out_cap=None, cipher=0):
    rng = random.Random(11)
    key = _mk_key(rng, version, klen, cipher)
    wire = build(key)
    st = np.zeros(1, O.TLS_STREAM_DT)
    st[0]["len"], st[0]["seq"] = len(wire), seq
    return O.tls_open_batch(np.frombuffer(wire, np.uint8), key, st, max_records, out_cap)


def _over(version, cipher):
    """AEAD overhead of a record: tag, + explicit nonce for TLS 1.2 AES-GCM"""
    return 16 + (8 if version == O.TLS12 and cipher == O.AES_GCM else 0)


@pytest.mark.parametrize("cipher", [O.AES_GCM, O.CHACHA])
@pytest.mark.parametrize("version", [O.TLS13, O.TLS12])
def test_contract_cases(version, cipher):
    seal = lambda k, j, t, c, pad=0: O.tls_seal(k, 7 + j, t, c, pad)  # noqa: E731
    one = lambda build, **kw: _one(version, build, cipher=cipher, **kw)  # noqa: E731
    ov = _over(version, cipher)
    # bad MAC on the second record: first delivered, second fails, third skipped
    def bad_mac(k):
        r1 = bytearray(seal(k, 1, 23, b"x" * 40))
        r1[-1] ^= 0x80
        return seal(k, 0, 23, b"a" * 10) + bytes(r1) + seal(k, 2, 23, b"b")
    recs, res, out = one(bad_mac)
    assert list(recs["status"]) == [0, O.REC_BAD_MAC, O.REC_SKIPPED]
    assert res[0]["n_delivered"] == 1 and res[0]["status"] == -1 and res[0]["plain_len"] == 10
    # wrong sequence number = authentication failure
    recs, res, _ = one(lambda k: seal(k, 1, 23, b"zz"))
    assert list(recs["status"]) == [O.REC_BAD_MAC]
    # header checks, in order: version, type, overflow, short
    def hdr(t, ver, ln):
        return bytes([t, ver >> 8, ver & 0xFF, ln >> 8, ln & 0xFF])
    over = 16384 + (1 if version == O.TLS13 else 0) + ov
    for h, st in [(hdr(23, 0x0301, 100), O.REC_VERSION), (hdr(20, 0x0303, 100), O.REC_BAD_TYPE),
                  (hdr(23, 0x0303, over + 1), O.REC_OVERFLOW),
                  (hdr(23, 0x0303, ov - 1), O.REC_BAD_MAC)]:
        recs, res, _ = one(lambda k: seal(k, 0, 23, b"ok") + h)
        assert list(recs["status"]) == [0, st], (h.hex(), recs["status"])
        assert res[0]["n_delivered"] == 1 and res[0]["first_status"] == st
    # maximum-size record opens; a header-only / partial record is incomplete (not counted)
    recs, res, _ = one(lambda k: seal(k, 0, 23, b"m" * 16384) + hdr(23, 0x0303, 40)[:3])
    assert list(recs["status"]) == [0] and res[0]["plain_len"] == 16384
    recs, res, _ = one(lambda k: seal(k, 0, 23, b"q" * 3) + seal(k, 1, 23, b"r" * 50)[:-1])
    assert len(recs) == 1
    assert res[0]["consumed_bytes"] == 5 + 3 + ov + (1 if version == O.TLS13 else 0)
    # alert / handshake records stop delivery without an error
    for t in (21, 22):
        recs, res, _ = one(lambda k: seal(k, 0, 23, b"d") + seal(k, 1, t, b"\x01\x00") + seal(k, 2, 23, b"e"))
        assert list(recs["status"]) == [0, O.REC_CONTROL, O.REC_SKIPPED]
        assert recs[1]["type"] == t and res[0]["status"] == 0 and res[0]["next_seq"] == 8
    # zero-length application data is delivered
    recs, res, _ = one(lambda k: seal(k, 0, 23, b"") + seal(k, 1, 23, b"Z"))
    assert list(recs["content_len"]) == [0, 1] and res[0]["plain_len"] == 1
    # capacity: too many records for the record array -> every stream ERR_CAPACITY
    recs, res, _ = one(lambda k: seal(k, 0, 23, b"1") + seal(k, 1, 23, b"2"), max_records=1)
    assert len(recs) == 0 and res[0]["first_status"] == O.REC_CAPACITY and res[0]["plain_len"] == 0


def test_tls13_inner_plaintext():
    # padding is stripped; an inner plaintext with no non-zero byte is ERR_EMPTY
    def build(k):
        return (O.tls_seal(k, 7, 23, b"abc", pad=100) + O.tls_seal(k, 8, 23, b"de")
                + O.tls_seal(k, 9, 0, b"", pad=3))
    for cipher in (O.AES_GCM, O.CHACHA):
        recs, res, out = _one(O.TLS13, build, cipher=cipher)
        assert list(recs["status"]) == [0, 0, O.REC_EMPTY]
        assert out[res[0]["out_off"]:res[0]["out_off"] + res[0]["plain_len"]].tobytes() == b"abcde"


def test_key_errors():
    rng = random.Random(5)
    keys = np.concatenate([_mk_key(rng, O.TLS13, cipher=O.AES_GCM) for _ in range(3)])
    keys[1]["key_len"] = 24                          # invalid AES key length
    keys[2]["cipher"], keys[2]["key_len"] = 1, 16   # ChaCha20-Poly1305 needs 32 bytes
    wire = O.tls_seal(keys[0:1], 0, 23, b"hello")
    st = np.zeros(4, O.TLS_STREAM_DT)
    st["len"] = len(wire)
    st["key"] = [0, 1, 2, 3]
    recs, res, out = O.tls_open_batch(np.frombuffer(wire, np.uint8), keys, st)
    assert list(res["first_status"]) == [0, O.REC_KEY, O.REC_KEY, O.REC_KEY]
    assert list(res["n_records"]) == [1, 0, 0, 0] and res[0]["plain_len"] == 5
