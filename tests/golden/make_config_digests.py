"""SHA-256 digests of the BASELINE configs' synthetic inputs and decoded outputs
("commit per-config SHA-256 digests of the unmasked payload stream computed by
the oracle from the committed generator seed; the GPU box reproduces the generator and
checks digests").

Generator: seed 0x5EED0001, key of frame i = low 32 bits of
splitmix64(seed ^ i), keys 0x00000000 / 0xFFFFFFFF forced at frames 0 and 1, payload byte b of
frame i = byte (b & 7) of splitmix64(seed + (i << 32) + (b >> 3)); restated in
oracle/ws_oracle.c (oracle_gen_frames).  Per config this records
  wire     sha256 of the masked wire as generated (frames packed at a fixed stride)
  payload  sha256 of the unmasked payload stream in frame order (what decode_compact's arena
           holds; for C4 the one reassembled 256 MiB message)
  decoded  sha256 of the whole wire after an in-place decode (headers and keys unchanged)
C5 (8 388 608 frames, 512 GiB) records, for one resident pass of 1 048 576 frames (68.7 GB of
wire; every rank's pass at N = 8 has this shape), the sha256 of the decoded wire of every
4096-frame chunk ("decoded_chunks", in order) and the sha256 of those digests concatenated
("decoded": a checksum of checksums), which tests/test_gpu_parity.py::test_config_c5_chunk
compares byte for byte through; and the payload digest of a sample of frames (every 4099th plus
the last), kept for the CPU test.

Run:  python tests/golden/make_config_digests.py   (rewrites config_digests.json here)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle  # noqa: E402

SEED = 0x5EED0001
CONFIGS = {  # name: (frames, payload bytes, fragmented)
    "c2": (65536, 4096, False),
    "c3": (65536, 65536, False),
    "c4": (1048576, 256, True),
}
C5 = (1048576, 65536)
CHUNK_BYTES = 256 << 20


def c5_sample():
    n = C5[0]
    return list(range(0, n, 4099)) + [n - 1]


def config_digests(n, plen, frag):
    L = _oracle.load()
    stride = int(L.oracle_gen_stride(plen))
    hs = stride - 4 - plen
    hw, hp, hd = hashlib.sha256(), hashlib.sha256(), hashlib.sha256()
    chunk = max(1, CHUNK_BYTES // stride)
    for first in range(0, n, chunk):
        cnt = min(chunk, n - first)
        ow, _ = _oracle.gen_frames(n, plen, SEED, fragmented=frag, force_keys=True,
                                   first=first, count=cnt, total=n)
        hw.update(ow)
        L.oracle_unmask_frames(_oracle._ptr(ow), cnt, stride)
        hd.update(ow)
        hp.update(ow.reshape(cnt, stride)[:, hs + 4:].tobytes())
    return {"frames": n, "payload_len": plen, "fragmented": frag, "stride": stride,
            "wire": hw.hexdigest(), "payload": hp.hexdigest(), "decoded": hd.hexdigest()}


def c5_digest():
    n, plen = C5
    L = _oracle.load()
    stride = int(L.oracle_gen_stride(plen))
    h = hashlib.sha256()
    for i in c5_sample():
        ow, _ = _oracle.gen_frames(n, plen, SEED, force_keys=True, first=i, count=1, total=n)
        L.oracle_unmask_frames(_oracle._ptr(ow), 1, stride)
        h.update(ow[stride - plen:].tobytes())
    return {"frames": n, "payload_len": plen, "sample": "range(0, 1048576, 4099) + [1048575]",
            "payload_sample": h.hexdigest()}


C5_CHUNK_FRAMES = 4096


def c5_chunk_digest(k):
    """sha256 of the oracle-decoded wire of C5 pass frames [4096 k, 4096 (k + 1))"""
    n, plen = C5
    L = _oracle.load()
    stride = int(L.oracle_gen_stride(plen))
    ow, _ = _oracle.gen_frames(n, plen, SEED, force_keys=True, first=k * C5_CHUNK_FRAMES,
                               count=C5_CHUNK_FRAMES, total=n)
    L.oracle_unmask_frames(_oracle._ptr(ow), C5_CHUNK_FRAMES, stride)
    return hashlib.sha256(ow).hexdigest()


def c5_chunk_digests(threads=8):
    """every chunk's digest, computed on `threads` threads (the oracle's C calls and sha256 run
    outside the GIL)"""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(c5_chunk_digest, range(C5[0] // C5_CHUNK_FRAMES)))


def main():
    out = {"seed": SEED, "generator": "oracle/ws_oracle.c oracle_gen_frames (force_keys=1)"}
    for name, (n, plen, frag) in CONFIGS.items():
        out[name] = config_digests(n, plen, frag)
        print(name, out[name], flush=True)
    out["c5_pass"] = c5_digest()
    chunks = c5_chunk_digests()
    out["c5_pass"].update({"chunk_frames": C5_CHUNK_FRAMES, "decoded_chunks": chunks,
                           "decoded": hashlib.sha256("".join(chunks).encode()).hexdigest()})
    with open(os.path.join(HERE, "config_digests.json"), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main()
