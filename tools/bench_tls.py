#!/usr/bin/env python3
"""TLS record open throughput on one MI355X (not the BASELINE metric).

Workload: `--conns` connections, each with `--records` application-data records of `--plen`
content bytes (default 65 536 x 4 x 16 KiB: 64 KiB of plaintext per connection, the C3 shape),
TLS 1.3 (or --version 12), AES-128-GCM (or --klen 32, or --cipher chacha: ChaCha20-Poly1305),
one key per connection.  The records
are sealed on the device (uvhttp_tls_gpu_seal_records), then each timed step opens all of them
(uvhttp_tls_gpu_open_records: key schedules, walk, crypto, finalize) with inputs resident in
HBM.  Prints one JSON line: plaintext GiB/s per step, the crypto kernel's time (HIP events),
its bytes moved (ciphertext read + plaintext written), and two single-core CPU baselines on a
bounded sample: the oracle restatement (byte-oriented C, the parity checker) and OpenSSL 3.0
EVP AES-GCM / ChaCha20-Poly1305 from the system libcrypto (AES-NI + PCLMUL / AVX2: what a
production CPU stack does).

    python tools/bench_tls.py [--conns N] [--records R] [--plen P] [--version 13|12] [--klen 16|32]
                              [--cipher aes|chacha] [--chain]

--chain: the TLS -> WebSocket chain the reference runs per read (src/uvhttp_connection.c:
1128-1158: mbedtls_ssl_read, then process_data on each decrypted chunk).  Each connection's
plaintext is one masked BINARY WebSocket frame filling its records (65 528-byte payload at the
default 4 x 16 KiB), and a step is open_records -> ws_streams (one process_data call per
record) -> decode_reads: ciphertext in HBM -> unmasked messages in HBM.  The rate is WebSocket
payload bytes per second.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
GIB = float(1 << 30)


def openssl_baseline(keyrec, seq, wire, n_rec, rlen, version, seconds, chacha=False):
    """OpenSSL EVP AEAD decrypt of the same records, 1 thread (libcrypto.so.3)."""
    try:
        L = C.CDLL("libcrypto.so.3")
    except OSError:
        return None
    vp, ip = C.c_void_p, C.c_int
    for name, res, args in [("EVP_CIPHER_CTX_new", vp, []), ("EVP_CIPHER_CTX_free", None, [vp]),
                            ("EVP_aes_128_gcm", vp, []), ("EVP_aes_256_gcm", vp, []),
                            ("EVP_chacha20_poly1305", vp, []),
                            ("EVP_DecryptInit_ex", ip, [vp, vp, vp, vp, vp]),
                            ("EVP_DecryptUpdate", ip, [vp, vp, C.POINTER(ip), vp, ip]),
                            ("EVP_DecryptFinal_ex", ip, [vp, vp, C.POINTER(ip)]),
                            ("EVP_CIPHER_CTX_ctrl", ip, [vp, ip, ip, vp])]:
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    klen = int(keyrec["key_len"])
    key = bytes(keyrec["key"][:klen])
    iv = bytes(keyrec["iv"])
    cipher = (L.EVP_chacha20_poly1305() if chacha else
              L.EVP_aes_128_gcm() if klen == 16 else L.EVP_aes_256_gcm())
    ctx = L.EVP_CIPHER_CTX_new()
    out = C.create_string_buffer(rlen)
    outl = ip(0)
    buf = wire.tobytes()
    done, t0, ok = 0, time.perf_counter(), True
    while time.perf_counter() - t0 < seconds:
        for j in range(n_rec):
            rec = buf[j * (5 + rlen):(j + 1) * (5 + rlen)]
            s = seq + j
            if version == 0x0304:
                nonce = bytes(a ^ b for a, b in zip(iv, bytes(4) + s.to_bytes(8, "big")))
                aad, ct = rec[:5], rec[5:5 + rlen - 16]
            elif chacha:  # RFC 7905: implicit nonce
                nonce = bytes(a ^ b for a, b in zip(iv, bytes(4) + s.to_bytes(8, "big")))
                ct = rec[5:5 + rlen - 16]
                aad = s.to_bytes(8, "big") + rec[:3] + len(ct).to_bytes(2, "big")
            else:
                nonce = iv[:4] + rec[5:13]
                ct = rec[13:5 + rlen - 16]
                aad = s.to_bytes(8, "big") + rec[:3] + len(ct).to_bytes(2, "big")
            tag = rec[5 + rlen - 16:5 + rlen]
            L.EVP_DecryptInit_ex(ctx, cipher, None, key, nonce)
            L.EVP_DecryptUpdate(ctx, None, C.byref(outl), aad, len(aad))
            L.EVP_DecryptUpdate(ctx, out, C.byref(outl), ct, len(ct))
            L.EVP_CIPHER_CTX_ctrl(ctx, 0x11, 16, tag)  # EVP_CTRL_GCM_SET_TAG
            ok &= L.EVP_DecryptFinal_ex(ctx, out, C.byref(outl)) == 1
            done += len(ct) - (1 if version == 0x0304 else 0)
    el = time.perf_counter() - t0
    L.EVP_CIPHER_CTX_free(ctx)
    return {"value": round(done / el / GIB, 3), "unit": "GiB/s", "cores": 1,
            "kind": "openssl-evp", "tags_ok": bool(ok),
            "sample": f"{n_rec} records x {rlen} B, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conns", type=int, default=65536)
    ap.add_argument("--records", type=int, default=4)
    ap.add_argument("--plen", type=int, default=16384)
    ap.add_argument("--version", type=int, default=13, choices=[12, 13])
    ap.add_argument("--klen", type=int, default=16, choices=[16, 32])
    ap.add_argument("--cipher", default="aes", choices=["aes", "chacha"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lib", default=None, help="another build of the library (A/B runs)")
    ap.add_argument("--chain", action="store_true", help="open_records -> ws_streams -> decode_reads")
    args = ap.parse_args()

    import torch
    import _oracle as O  # test infrastructure: key structs and the CPU baseline leg only
    import uvhttp_amd as U

    ver = 0x0304 if args.version == 13 else 0x0303
    n, per, plen = args.conns, args.records, args.plen
    rng = np.random.default_rng(7)
    # one key slot per connection up to 65 536 (the seal descriptor's slot is 16-bit); beyond
    # that connection i uses slot i % 65 536 (synthetic data: shared keys change no work)
    nk = min(n, 65536)
    keys = np.zeros(nk, O.TLS_KEY_DT)
    keys["key"] = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    keys["iv"] = rng.integers(0, 256, (nk, 12), dtype=np.uint8)
    chacha = args.cipher == "chacha"
    keys["key_len"], keys["version"] = (32 if chacha else args.klen), ver
    keys["cipher"] = O.CHACHA if chacha else O.AES_GCM
    # TLSCiphertext.length: content + tag + (TLS 1.3 type byte | TLS 1.2 AES-GCM explicit nonce)
    rlen = plen + 16 + (1 if ver == 0x0304 else 0 if chacha else 8)
    aead = "ChaCha20-Poly1305" if chacha else f"AES-{args.klen * 8}-GCM"
    stride = 5 + rlen
    idx = np.arange(n * per, dtype=np.uint64)
    seals = np.zeros(n * per, O.TLS_SEAL_DT)
    seals["src_off"] = idx * plen
    seals["out_off"] = idx * stride
    seals["seq"] = idx % per
    seals["plain_len"] = plen
    seals["key"] = ((idx // per) % nk).astype(np.uint16)
    seals["type"] = 23
    streams = np.zeros(n, O.TLS_STREAM_DT)
    streams["begin"] = np.arange(n, dtype=np.uint64) * per * stride
    streams["len"] = per * stride
    streams["key"] = np.arange(n) % nk
    dev = "cuda:0"
    t = torch
    src = t.randint(0, 256, (n * per * plen,), dtype=t.uint8, device=dev)
    weng = None
    if args.chain:
        # one masked BINARY frame per connection filling its per * plen plaintext bytes
        weng = U.GpuEngine(0)
        conn_bytes = per * plen
        fp = conn_bytes - 8 if conn_bytes - 8 < 65536 else conn_bytes - 14
        assert U.gen_frame_stride(fp) == conn_bytes, "pick --records * --plen >= 134"
        weng.gen_frames(src, n, fp, 11, opcode0=2)
    wire = t.empty(n * per * stride, dtype=t.uint8, device=dev)
    out = t.empty(wire.numel(), dtype=t.uint8, device=dev)
    dk = t.from_numpy(keys.view(np.uint8).reshape(-1).copy()).to(dev)
    ds = t.from_numpy(seals.view(np.uint8).reshape(-1).copy()).to(dev)
    dst = t.from_numpy(streams.view(np.uint8).reshape(-1).copy()).to(dev)
    eng = U.TlsEngine(0, library=U.load_library(args.lib) if args.lib else None)
    eng.seal_records(src, ds, n * per, dk, nk, wire)
    recs = t.empty(n * per * 32, dtype=t.uint8, device=dev)
    res = t.empty(n * 64, dtype=t.uint8, device=dev)

    if args.chain:
        ws0 = np.zeros(n, U.STREAM_DT)  # fresh server connections (uvhttp_ws_stream_init)
        ws0["recv_buffer_size"] = 65536
        ws0["max_frame_size"], ws0["max_message_size"], ws0["is_server"] = 16 << 20, 64 << 20, 1
        ws_dev = t.from_numpy(ws0.view(np.uint8).reshape(-1).copy()).to(dev)
        read_end = t.zeros(n * per, dtype=t.int64, device=dev)
        wdesc = t.empty(n * 32, dtype=t.uint8, device=dev)
        wres = t.empty(n * U.STREAM_RESULT_BYTES, dtype=t.uint8, device=dev)
        weng.reserve(n, out.numel(), 0)

    def step():
        eng.open_records(wire, dk, nk, dst, n, n * per, out, records=recs, results=res)
        if args.chain:
            eng.ws_streams(res, recs, n, dst, out, ws_dev, read_end)
            weng.decode_streams(out, ws_dev, n, n, desc=wdesc, results=wres, read_end=read_end,
                                n_reads=n * per)

    for _ in range(args.warmup):
        step()
    t.cuda.synchronize()
    R = res.cpu().numpy().view(O.TLS_RESULT_DT)
    assert (R["n_delivered"] == per).all() and (R["plain_len"] == per * plen).all(), "open failed"
    if args.chain:
        # every connection: one message of fp bytes, unmasked in place inside `out`
        wr = weng.read_stream_results(wres, n)
        assert all(r.status == 0 and r.n_delivered == 1 and r.calls == per for r in wr[:64]), wr[0].as_dict()
        assert sum(r.n_delivered for r in wr) == n
        weng.sync()
    else:
        got = out.view(-1)[: per * plen]
        assert t.equal(got, src[: per * plen]), "plaintext mismatch"
    eng.set_timing(True)
    eng.kernel_time()
    t.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t.cuda.synchronize()
    el = time.perf_counter() - t0
    kms, launches = eng.kernel_time()
    eng.set_timing(False)
    plain = n * per * plen
    kus = kms * 1e3 / max(1, launches)
    moved = n * per * (stride + plen)  # ciphertext records read + plaintext written
    if args.chain:
        plain = n * fp  # WebSocket payload delivered per step
    line = {
        "metric": ("TLS -> WebSocket chain GiB/s (ciphertext in HBM -> unmasked messages)"
                   if args.chain else "TLS record open GiB/s (device-resident)"),
        "value": round(plain * args.steps / el / GIB, 2),
        "unit": "GiB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
        "dtype": "u8/u32 (ChaCha20-Poly1305)" if chacha else "u8/u32 (AES-GCM)", "data": "synthetic (random plaintext sealed on the device)",
        "config": {"workload": f"{n} connections x {per} x {plen} B TLS 1.{args.version % 10} "
                               f"{aead} records", "conns": n, "records": per,
                   "plen": plen},
        "kernel": {"name": "k_tls_open", "avg_us": round(kus, 2),
                   "plaintext_gbs": round(plain / (kus * 1e-6) / 1e9, 1),
                   "hbm_gbs": round(moved / (kus * 1e-6) / 1e9, 1), "launches": launches},
    }
    if args.lib:
        line["lib"] = os.path.basename(args.lib)
    if args.chain:
        line["config"]["chain"] = ("open_records -> ws_streams (one process_data call per record) "
                                   f"-> decode_reads; one {fp}-byte masked BINARY frame per connection")
    if not args.no_cpu_baseline and not args.chain:
        m = per  # connection 0's records (one key, sequence numbers 0 .. per-1)
        sample = wire[: m * stride].cpu().numpy()
        ob = np.zeros(m * stride, np.uint8)
        t1 = time.perf_counter()
        done = 0
        while time.perf_counter() - t1 < args.cpu_seconds:
            done += O.tls_open_stream_bytes(keys[0:1], 0, sample, ob)
        el1 = time.perf_counter() - t1
        line["cpu_baseline"] = {
            "oracle": {"value": round(done / el1 / GIB, 4), "unit": "GiB/s", "cores": 1,
                       "kind": "port", "sample": f"{m} records of connection 0, {el1:.1f} s"},
            "openssl": openssl_baseline(keys[0], 0, sample, m, rlen, ver, args.cpu_seconds, chacha),
        }
    print(json.dumps(line))


if __name__ == "__main__":
    main()
