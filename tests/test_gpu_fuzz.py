"""Exhaustive and property-based GPU checks against the oracle (oracle/ws_oracle.c).

* Unmask sweep: payload lengths 0..130 and 65535 / 65536 / 70000, each at all 16 payload
  alignments (a PING of 0..15 payload bytes in front shifts the data frame), with masking keys
  0, 0xFFFFFFFF and random — decoded in place, compact, and as one connection's stream; bytes,
  statuses, summaries and the guard bytes around every buffer are checked (the partial-vector
  head and tail of each payload and the key rotation at every offset, src/uvhttp_websocket.c
  :931-937 / uvhttp_ws_apply_mask).
* Hypothesis fuzzer of uvhttp_ws_gpu_decode_streams / _decode_reads: connections with drawn
  limits, history (an open fragment, a partial frame buffered) and drawn frame lists (every
  opcode including reserved ones, RSV bits, unmasked frames, oversize control frames, 16/64-bit
  length forms used for small payloads) cut into drawn read sizes; the host delivery must leave
  each connection exactly where the oracle's process_data per read leaves it.
* The same for connections of EQUAL frames, the shape the speculative stream decode (k_sspec_*)
  takes: a drawn frame length (64 bytes up, around the 16 / 64-bit length forms and the 16 KiB
  tile), a drawn fragment pattern, an optional break (one frame of another length, a control
  frame, RSV bits, an unmasked frame, a CONT without a start) at a drawn index, a drawn trailing
  partial frame — so the speculation runs, is refused by the plan, or breaks in the pass or the
  state machine and is undone.
"""
import random

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import _oracle
from test_gpu_parity import _compare, _frame, _run_both
from test_gpu_streams import _run_cases, hooks  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

LENGTHS = list(range(131)) + [65535, 65536, 70000]
KEYS = [bytes(4), b"\xff\xff\xff\xff", None]  # None: a random key per frame


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def eng(torch):
    import uvhttp_amd as U
    e = U.GpuEngine(0)
    yield e
    e.close()


def _sweep_frames(lengths, rng):
    """[PING pad][data frame] pairs: every length at every payload alignment mod 16, each key"""
    frames, pos = [], 0
    for key in KEYS:
        for n in lengths:
            h = 2 if n < 126 else 4 if n < 65536 else 10
            for a in range(16):
                pad = (a - (pos + 6 + h + 4)) % 16
                ping = _frame(9, 1, rng.randbytes(pad), rng.randbytes(4))
                k = key if key is not None else rng.randbytes(4)
                data = _frame(rng.choice([1, 2]), 1, rng.randbytes(n), k)
                assert (pos + len(ping) + h + 4) % 16 == a
                frames += [ping, data]
                pos += len(ping) + len(data)
    return frames


@pytest.mark.parametrize("part", ["small", "large"])
@pytest.mark.parametrize("compact", [False, True])
def test_unmask_sweep_lengths_alignments_keys(torch, eng, part, compact):
    rng = random.Random(4242)
    lengths = LENGTHS[:131] if part == "small" else LENGTHS[131:]
    frames = _sweep_frames(lengths, rng)
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    ref, got = _run_both(torch, eng, wire, len(frames), offs=offs, compact=compact)
    assert ref["summary"]["status"] == 0 and ref["summary"]["n_delivered"] == len(frames)
    _compare(ref, got, compact)


@pytest.mark.parametrize("part", ["small", "large"])
def test_unmask_sweep_as_stream(torch, eng, hooks, part):  # noqa: F811
    """The same sweep as one connection's bytes, cut into 16 KiB reads (process_data per read)."""
    import uvhttp_amd as U
    rng = random.Random(4243)
    lengths = LENGTHS[:131] if part == "small" else LENGTHS[131:]
    data = b"".join(_sweep_frames(lengths, rng))
    prod = U.WsConnection(1, 16 * 1024 * 1024, 64 * 1024 * 1024, user_data=True)
    orc = _oracle.OracleConn(1, 16 * 1024 * 1024, 64 * 1024 * 1024, record=1, wrapper=True)
    reads = [data[k:k + 16384] for k in range(0, len(data), 16384)]
    res = _run_cases(torch, eng, U, [(prod, orc, reads)], rng, 2 * len(LENGTHS) * 48 + 16,
                     use_reads=True)
    assert res[0].status == 0


# ---- hypothesis fuzzer of the stream decode ----------------------------------------------

_OPS = st.sampled_from([0, 0, 1, 1, 2, 2, 3, 8, 9, 10, 0xB])
_PLEN = st.one_of(st.integers(0, 130), st.sampled_from([125, 126, 127, 300, 4000, 65535, 65536, 70000]))
_FRAME = st.tuples(_OPS, st.booleans(), _PLEN,
                   st.sampled_from([0] * 12 + [1, 2, 4, 7]),       # RSV bits (mostly clear)
                   st.sampled_from([True] * 12 + [False]),         # masked
                   st.sampled_from([None] * 6 + [16, 64]))         # length form


def _mk(rng, spec):
    op, fin, plen, rsv, masked, form = spec
    if form == 16 and plen >= 65536:
        form = None
    return _frame(op, fin, rng.randbytes(plen), rng.randbytes(4), masked, rsv, form)


_CONN = st.fixed_dictionaries({
    "mf": st.sampled_from([16 * 1024 * 1024, 65536, 4000, 130]),
    "mm": st.sampled_from([64 * 1024 * 1024, 9000, 0, 200]),
    "prefix_open": st.booleans(),            # a fragmented message open before the reads
    "partial": st.sampled_from([0, 0, 1, 5, 13, 200]),  # bytes of a frame already buffered
    "frames": st.lists(_FRAME, max_size=8),
    "reads": st.lists(st.sampled_from([0, 1, 2, 3, 7, 14, 100, 1000, 4096, 16384, 20000]),
                      min_size=1, max_size=12),
})


def _case(U, rng, c):
    prod = U.WsConnection(1, c["mf"], c["mm"], user_data=True)
    orc = _oracle.OracleConn(1, c["mf"], c["mm"], record=1, wrapper=True)
    prefix = b""
    if c["prefix_open"]:
        prefix += _frame(1, 0, rng.randbytes(20), rng.randbytes(4))
    new = b"".join(_mk(rng, f) for f in c["frames"])
    if c["partial"]:
        tail = _frame(2, 1, rng.randbytes(100), rng.randbytes(4))
        cut = min(c["partial"], len(tail) - 1)
        prefix += tail[:cut]
        new = tail[cut:] + new
    r1, r2 = prod.process_data(prefix), orc.process_data(prefix)
    assert r1 == r2
    if r1 != 0:
        return None
    reads, pos, k = [], 0, 0
    sizes = c["reads"]
    while pos < len(new):
        n = sizes[k % len(sizes)] or 1
        if sizes[k % len(sizes)] == 0:
            reads.append(b"")  # a zero-length read, then one byte
        reads.append(new[pos:pos + n])
        pos += n
        k += 1
    if not reads:
        reads = [b""]
    return prod, orc, reads


@settings(max_examples=60, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(conns=st.lists(_CONN, min_size=1, max_size=10), seed=st.integers(0, 2**32 - 1),
       per_read=st.booleans())
def test_hypothesis_streams_vs_oracle(torch, eng, hooks, conns, seed, per_read):  # noqa: F811
    import uvhttp_amd as U
    rng = random.Random(seed)
    cases = [c for c in (_case(U, rng, c) for c in conns) if c]
    if not cases:
        return
    _run_cases(torch, eng, U, cases, rng, 4096, use_reads=per_read)


_SPEC_CONN = st.fixed_dictionaries({
    "plen": st.sampled_from([58, 59, 60, 100, 121, 125, 126, 200, 250, 1000, 4090, 16378, 16390, 65530, 65536]),
    "n": st.integers(1, 40),
    "pattern": st.sampled_from(["whole", "frag", "mixed", "open_end"]),
    "op": st.sampled_from([1, 2]),
    "break_at": st.one_of(st.none(), st.integers(0, 39)),
    "break_kind": st.sampled_from(["len", "ping", "close", "rsv", "unmasked", "cont", "start"]),
    "tail": st.sampled_from([0, 0, 1, 3, 9, 100]),
    "pending": st.booleans(),
    "mm": st.sampled_from([0, 0, 64 * 1024 * 1024, 3000]),
    "reads": st.lists(st.sampled_from([0, 100, 1000, 4096, 16384, 20000, 1 << 20]), min_size=1, max_size=4),
})


def _spec_case(U, rng, c):
    plen, n, op = c["plen"], c["n"], c["op"]
    if plen > 16000:
        n = min(n, 6)  # (a few MB per connection at most: the oracle decodes it too)
    prod = U.WsConnection(1, 16 * 1024 * 1024, c["mm"], user_data=True)
    orc = _oracle.OracleConn(1, 16 * 1024 * 1024, c["mm"], record=1, wrapper=True)
    prefix = _frame(op, 0, rng.randbytes(20), rng.randbytes(4)) if c["pending"] else b""
    frames = []
    for i in range(n):
        if c["pattern"] == "whole":
            fop, fin = (0 if c["pending"] and i == 0 else op), 1
        elif c["pattern"] == "frag":  # one message over all frames
            fop, fin = (op if i == 0 and not c["pending"] else 0), int(i == n - 1)
        elif c["pattern"] == "mixed":  # messages of 3 frames
            fop, fin = (op if i % 3 == 0 and not (c["pending"] and i == 0) else 0), int(i % 3 == 2)
        else:  # every frame continues, the message stays open
            fop, fin = (op if i == 0 and not c["pending"] else 0), 0
        p, masked, rsv = plen, True, 0
        if c["break_at"] == i:
            k = c["break_kind"]
            if k == "len":
                p = plen + 1 if plen < 65536 else plen - 1
            elif k in ("ping", "close"):
                fop, fin, p = (9 if k == "ping" else 8), 1, min(plen, 125)
            elif k == "rsv":
                rsv = 4
            elif k == "unmasked":
                masked = False
            elif k == "cont":
                fop = 0
            else:
                fop = op
        frames.append(_frame(fop, fin, rng.randbytes(p), rng.randbytes(4), masked, rsv))
    new = b"".join(frames)
    if c["tail"]:
        t = _frame(0, 1, rng.randbytes(plen), rng.randbytes(4))
        new += t[:min(c["tail"], len(t) - 1)]
    r1, r2 = prod.process_data(prefix), orc.process_data(prefix)
    assert r1 == r2
    if r1 != 0:
        return None
    reads, pos, k = [], 0, 0
    while pos < len(new):
        sz = c["reads"][k % len(c["reads"])] or len(new)
        reads.append(new[pos:pos + sz])
        pos += sz
        k += 1
    return prod, orc, reads or [b""]


@settings(max_examples=60, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(conns=st.lists(_SPEC_CONN, min_size=1, max_size=12), seed=st.integers(0, 2**32 - 1),
       per_read=st.booleans())
def test_hypothesis_equal_frame_streams_vs_oracle(torch, eng, hooks, conns, seed, per_read):  # noqa: F811
    import uvhttp_amd as U
    rng = random.Random(seed)
    cases = [c for c in (_spec_case(U, rng, c) for c in conns) if c]
    if not cases:
        return
    # a frame capacity of at least 8 per connection: the speculative decode is tried
    _run_cases(torch, eng, U, cases, rng, max(8 * len(cases), 64 * len(cases)), use_reads=per_read)
