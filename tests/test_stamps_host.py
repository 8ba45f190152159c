"""Device-stamp ring reduction on the host (no GPU): a pass launched as several dispatch pieces
reads as ONE record spanning every piece (VERDICT r05 "What's weak" 1: the C5 pass's five
pieces each restarted blockIdx.x at 0, so the slot kept only the last piece and a 68.7 GB pass
read as 6.7 us).  The ring is written by uvhttp_ws_gpu_stamp_simulate, which uses the kernels'
own slot mapping (ws_gpu.hip stamp_sampled / stamp_end_word), and reduced by the same function
read_stamps runs on the copied device ring."""
import ctypes as C

import numpy as np
import pytest

import uvhttp_amd as U

KHZ = 100000  # gfx9 wall clock: 100 MHz -> 10 ns per tick
PAYLOAD = 5   # UVHTTP_WS_STAMP_PAYLOAD
PIECE = 1 << 24


@pytest.fixture(scope="module")
def L():
    return U.lib()


def _ring(L):
    return np.zeros(int(L.uvhttp_ws_gpu_stamp_ring_words()), dtype=np.uint64)


def _reduce(L, ring, epoch):
    out = (U.GpuStamp * 256)()
    n = C.c_uint32(0)
    assert L.uvhttp_ws_gpu_stamps_reduce(ring.ctypes.data, epoch, KHZ, out, 256, C.byref(n)) == 0
    return [(r.call, r.kernel, r.begin_ns, r.end_ns) for r in out[:n.value]]


def _pass(L, ring, epoch, total_blocks, t0, ticks, dur, restart_block_index=False):
    """One pass of total_blocks workgroups launched as pieces of <= 2^24, back to back in time"""
    base = 0
    while base < total_blocks:
        blocks = min(PIECE, total_blocks - base)
        tb = t0 + ticks * base // total_blocks
        te = t0 + ticks * (base + blocks) // total_blocks
        b = 0 if restart_block_index else base
        assert L.uvhttp_ws_gpu_stamp_simulate(ring.ctypes.data, epoch, PAYLOAD, b, blocks, 1,
                                              tb, te, dur) == 0
        base += blocks


def test_multi_piece_pass_is_one_record(L):
    # a C5 pass on one rank: 1 048 576 x 64 KiB frames in 1 KiB tiles = 67.1 M workgroups
    total = 1048576 * 65540 // 1024
    assert total > 4 * PIECE
    ring = _ring(L)
    t0, ticks, dur = 1_000_000, 1_020_000, 20  # 10.2 ms, 200 ns per workgroup
    _pass(L, ring, 7, total, t0, ticks, dur)
    recs = _reduce(L, ring, 7)
    assert len(recs) == 1
    call, kern, b, e = recs[0]
    assert kern == PAYLOAD
    assert b == t0 * 10
    # the last sampled workgroup is within 1024 of the pass's end
    assert (t0 + ticks + dur) * 10 >= e >= (t0 + ticks - ticks * 1024 // total) * 10
    # the span covers the whole pass, not one piece
    assert (e - b) >= 0.99 * ticks * 10


def test_restarting_block_index_would_keep_one_piece(L):
    """the round-5 behaviour, reproduced through the same mapping with base = 0 in every piece:
    the begin words are the last piece's, so the 'kernel' is one piece long"""
    total = 5 * PIECE - 123
    ring = _ring(L)
    t0, ticks = 0, 1_000_000
    _pass(L, ring, 3, total, t0, ticks, 5, restart_block_index=True)
    (_, _, b, e), = _reduce(L, ring, 3)
    assert (e - b) < 0.25 * ticks * 10
    ring[:] = 0
    _pass(L, ring, 3, total, t0, ticks, 5)
    (_, _, b, e), = _reduce(L, ring, 3)
    assert (e - b) > 0.99 * ticks * 10


def test_single_piece_and_call_order(L):
    ring = _ring(L)
    # two calls (epochs 10, 11), each a plan-like small kernel and a payload kernel
    for ep, t in ((10, 0), (11, 50_000)):
        assert L.uvhttp_ws_gpu_stamp_simulate(ring.ctypes.data, ep, 6, 0, 64, 4, t, t + 100, 30) == 0
        _pass(L, ring, ep, 4096, t + 200, 40_000, 7)
    recs = _reduce(L, ring, 11)
    assert [(c, k) for c, k, _, _ in recs] == [(11, 6), (11, 5), (12, 6), (12, 5)]
    for c, k, b, e in recs:
        assert e > b
    # payload of call 10: begins at 200 ticks, ends at most dur after the pass
    assert recs[1][2] == 200 * 10 and recs[1][3] <= (200 + 40_000 + 7) * 10


def test_simulate_rejects_bad_arguments(L):
    ring = _ring(L)
    assert L.uvhttp_ws_gpu_stamp_simulate(ring.ctypes.data, 1, 99, 0, 1, 1, 0, 1, 0) != 0
    assert L.uvhttp_ws_gpu_stamp_simulate(ring.ctypes.data, 1, 5, 0, 0, 1, 0, 1, 0) != 0
    assert L.uvhttp_ws_gpu_stamp_simulate(ring.ctypes.data, 1, 5, 0, 1, 1, 5, 1, 0) != 0
