"""Generate tests/golden/tls_openssl_records.json: real TLS records from a real TLS stack.

Runs in the build container only (not on the GPU box, not by the tests): drives OpenSSL
3.0.2's libssl (system library, /usr/lib/x86_64-linux-gnu/libssl.so.3) through ctypes over
memory BIOs — a client and a server in one process, a throw-away self-signed P-256 certificate
made with the `openssl` CLI — and captures the client -> server bytes after the handshake:
application-data records of several sizes (a write over 2^14 bytes spans two records), and
the encrypted close_notify alert at the end — TLS 1.3 and TLS 1.2, AES-GCM and
ChaCha20-Poly1305.  The read keys are recovered from OpenSSL's key
log (TLS 1.3: CLIENT_TRAFFIC_SECRET_0 -> HKDF-Expand-Label "key"/"iv", RFC 8446 §7.1/7.3;
TLS 1.2: CLIENT_RANDOM master secret -> PRF "key expansion" key block, RFC 5246 §6.3), so the
fixture pins the record layer of tls_oracle.c (nonce, AAD, inner plaintext, padding) against
an independent implementation.  The plaintexts the server's SSL_read returned are stored as
the expected output.

    python3 tests/golden/make_tls_vectors.py        # rewrites the JSON
"""
import base64
import ctypes as C
import hashlib
import hmac
import json
import os
import random
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "tls_openssl_records.json")

ssl = C.CDLL("libssl.so.3")
crypto = C.CDLL("libcrypto.so.3")
vp, ip, cp = C.c_void_p, C.c_int, C.c_char_p
for name, res, args in [
    ("TLS_server_method", vp, []), ("TLS_client_method", vp, []),
    ("SSL_CTX_new", vp, [vp]), ("SSL_CTX_free", None, [vp]),
    ("SSL_CTX_ctrl", C.c_long, [vp, ip, C.c_long, vp]),
    ("SSL_CTX_use_certificate_file", ip, [vp, cp, ip]),
    ("SSL_CTX_use_PrivateKey_file", ip, [vp, cp, ip]),
    ("SSL_CTX_set_ciphersuites", ip, [vp, cp]), ("SSL_CTX_set_cipher_list", ip, [vp, cp]),
    ("SSL_CTX_set_keylog_callback", None, [vp, vp]),
    ("SSL_CTX_set_block_padding", ip, [vp, C.c_size_t]),
    ("SSL_new", vp, [vp]), ("SSL_free", None, [vp]), ("SSL_set_bio", None, [vp, vp, vp]),
    ("SSL_set_connect_state", None, [vp]), ("SSL_set_accept_state", None, [vp]),
    ("SSL_do_handshake", ip, [vp]), ("SSL_get_error", ip, [vp, ip]),
    ("SSL_write", ip, [vp, vp, ip]), ("SSL_read", ip, [vp, vp, ip]),
    ("SSL_shutdown", ip, [vp]),
    ("SSL_get_client_random", C.c_size_t, [vp, vp, C.c_size_t]),
    ("SSL_get_server_random", C.c_size_t, [vp, vp, C.c_size_t]),
    ("SSL_get_current_cipher", vp, [vp]), ("SSL_CIPHER_get_name", cp, [vp]),
    ("SSL_get_version", cp, [vp]),
]:
    fn = getattr(ssl, name)
    fn.restype, fn.argtypes = res, args
for name, res, args in [("BIO_new", vp, [vp]), ("BIO_s_mem", vp, []),
                        ("BIO_read", ip, [vp, vp, ip]), ("BIO_write", ip, [vp, vp, ip]),
                        ("BIO_ctrl", C.c_long, [vp, ip, C.c_long, vp])]:
    fn = getattr(crypto, name)
    fn.restype, fn.argtypes = res, args

SSL_CTRL_SET_MIN_PROTO_VERSION, SSL_CTRL_SET_MAX_PROTO_VERSION = 123, 124
SSL_FILETYPE_PEM = 1
BIO_CTRL_PENDING = 10
KEYLOG_CB = C.CFUNCTYPE(None, vp, cp)


def drain(bio):
    out = b""
    buf = C.create_string_buffer(1 << 16)
    while crypto.BIO_ctrl(bio, BIO_CTRL_PENDING, 0, None) > 0:
        n = crypto.BIO_read(bio, buf, len(buf))
        if n <= 0:
            break
        out += buf.raw[:n]
    return out


def hkdf_expand_label(secret, label, length, h):
    info = length.to_bytes(2, "big") + bytes([len(b"tls13 " + label)]) + b"tls13 " + label + b"\x00"
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac.new(secret, t + info + bytes([i]), h).digest()
        out += t
        i += 1
    return out[:length]


def prf(secret, label, seed, length, h):
    a, out = label + seed, b""
    while len(out) < length:
        a = hmac.new(secret, a, h).digest()
        out += hmac.new(secret, a + label + seed, h).digest()
    return out[:length]


def session(version, suite, klen, h, writes, padding=0, cipher=0):
    tmp = tempfile.mkdtemp()
    cert, key = os.path.join(tmp, "c.pem"), os.path.join(tmp, "k.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt",
                    "ec_paramgen_curve:P-256", "-nodes", "-subj", "/CN=uvhttp-amd-test",
                    "-days", "1", "-keyout", key, "-out", cert], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    lines = []
    cb = KEYLOG_CB(lambda s, line: lines.append(line.decode()))
    sctx = ssl.SSL_CTX_new(ssl.TLS_server_method())
    cctx = ssl.SSL_CTX_new(ssl.TLS_client_method())
    for ctx in (sctx, cctx):
        ssl.SSL_CTX_ctrl(ctx, SSL_CTRL_SET_MIN_PROTO_VERSION, version, None)
        ssl.SSL_CTX_ctrl(ctx, SSL_CTRL_SET_MAX_PROTO_VERSION, version, None)
        if version == 0x0304:
            assert ssl.SSL_CTX_set_ciphersuites(ctx, suite.encode()) == 1
        else:
            assert ssl.SSL_CTX_set_cipher_list(ctx, suite.encode()) == 1
    assert ssl.SSL_CTX_use_certificate_file(sctx, cert.encode(), SSL_FILETYPE_PEM) == 1
    assert ssl.SSL_CTX_use_PrivateKey_file(sctx, key.encode(), SSL_FILETYPE_PEM) == 1
    ssl.SSL_CTX_set_keylog_callback(cctx, C.cast(cb, vp))
    if padding:
        assert ssl.SSL_CTX_set_block_padding(cctx, padding) == 1
    cli, srv = ssl.SSL_new(cctx), ssl.SSL_new(sctx)
    c_in, c_out = crypto.BIO_new(crypto.BIO_s_mem()), crypto.BIO_new(crypto.BIO_s_mem())
    s_in, s_out = crypto.BIO_new(crypto.BIO_s_mem()), crypto.BIO_new(crypto.BIO_s_mem())
    ssl.SSL_set_bio(cli, c_in, c_out)
    ssl.SSL_set_bio(srv, s_in, s_out)
    ssl.SSL_set_connect_state(cli)
    ssl.SSL_set_accept_state(srv)
    done_c = done_s = False
    for _ in range(50):
        if not done_c:
            done_c = ssl.SSL_do_handshake(cli) == 1
        d = drain(c_out)
        if d:
            crypto.BIO_write(s_in, d, len(d))
        if not done_s:
            done_s = ssl.SSL_do_handshake(srv) == 1
        d = drain(s_out)
        if d:
            crypto.BIO_write(c_in, d, len(d))
        if done_c and done_s:
            break
    assert done_c and done_s, "handshake did not finish"
    # let the client consume post-handshake messages (TLS 1.3 session tickets)
    rb = C.create_string_buffer(1 << 15)
    ssl.SSL_read(cli, rb, 0)
    drain(c_out)
    suite_name = ssl.SSL_CIPHER_get_name(ssl.SSL_get_current_cipher(cli)).decode()
    cr, sr = C.create_string_buffer(32), C.create_string_buffer(32)
    ssl.SSL_get_client_random(cli, cr, 32)
    ssl.SSL_get_server_random(cli, sr, 32)

    rng = random.Random(version * 7 + klen)
    sent = []
    wire = b""
    for n in writes:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        assert ssl.SSL_write(cli, data, len(data)) == len(data)
        wire += drain(c_out)
        sent.append(data)
    ssl.SSL_shutdown(cli)  # encrypted close_notify alert
    wire += drain(c_out)
    # the server reads everything back: the expected application data
    crypto.BIO_write(s_in, wire, len(wire))
    got = b""
    while True:
        n = ssl.SSL_read(srv, rb, len(rb))
        if n <= 0:
            break
        got += rb.raw[:n]
    assert got == b"".join(sent), "server did not read back what the client wrote"

    kl = {ln.split()[0]: ln.split() for ln in lines}
    if version == 0x0304:
        secret = bytes.fromhex(kl["CLIENT_TRAFFIC_SECRET_0"][2])
        wkey, wiv = hkdf_expand_label(secret, b"key", klen, h), hkdf_expand_label(secret, b"iv", 12, h)
        seq0 = 0
    else:
        ms = bytes.fromhex(kl["CLIENT_RANDOM"][2])
        ivlen = 12 if cipher else 4  # ChaCha20-Poly1305: 12-byte fixed iv (RFC 7905)
        kb = prf(ms, b"key expansion", sr.raw + cr.raw, 2 * klen + 2 * ivlen, h)
        wkey, wiv = kb[:klen], (kb[2 * klen:2 * klen + ivlen] + bytes(12))[:12]
        seq0 = 1  # seq 0 was the client's Finished
    ssl.SSL_free(cli)  # frees its BIOs
    ssl.SSL_free(srv)
    ssl.SSL_CTX_free(sctx)
    ssl.SSL_CTX_free(cctx)
    return {
        "version": version, "suite": suite_name, "cipher": cipher,
        "key": wkey.hex(), "iv": wiv.hex(), "seq": seq0, "padding": padding,
        "writes": writes, "wire_b64": base64.b64encode(wire).decode(),
        "plaintext_len": len(got), "plaintext_sha256": hashlib.sha256(got).hexdigest(),
        "stop_type": 21,  # the close_notify alert after the data
    }


def main():
    writes = [1, 100, 1000, 16384, 17000, 0, 300]
    sessions = [
        session(0x0304, "TLS_AES_128_GCM_SHA256", 16, hashlib.sha256, writes),
        session(0x0304, "TLS_AES_256_GCM_SHA384", 32, hashlib.sha384, writes),
        session(0x0304, "TLS_AES_128_GCM_SHA256", 16, hashlib.sha256, writes, padding=256),
        session(0x0303, "ECDHE-ECDSA-AES128-GCM-SHA256", 16, hashlib.sha256, writes),
        session(0x0303, "ECDHE-ECDSA-AES256-GCM-SHA384", 32, hashlib.sha384, writes),
        session(0x0304, "TLS_CHACHA20_POLY1305_SHA256", 32, hashlib.sha256, writes, cipher=1),
        session(0x0303, "ECDHE-ECDSA-CHACHA20-POLY1305", 32, hashlib.sha256, writes, cipher=1),
    ]
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_tls_vectors.py",
                   "stack": "OpenSSL 3.0.2 libssl (system library of the build image)",
                   "sessions": sessions}, f, indent=1)
    print(OUT, len(sessions), "sessions")


if __name__ == "__main__":
    main()
