"""BASELINE config C1 — examples/05_websocket echo of one 1 KiB masked binary frame — on a
real libuv loop (CPU; tests/c/c1_echo.c), plus the sanitizer builds of the host decoder.

The harness is the reference's L2 path around the product's drop-in surface: a loopback TCP
server whose read callback hands every libuv read (<= 16 KiB, the reference's read_buffer,
src/uvhttp_connection.c:128-158) to uvhttp_ws_process_data (:1163-1164), and whose on_message
echoes the payload as an unmasked TEXT frame (websocket_echo_server.c:12-23 ->
uvhttp_server_ws_send).  The echo each client receives is checked here against the ORACLE's
decode of the bytes the client sent (oracle/ws_oracle.c, process_data per read-sized cut).

The ASan/UBSan builds (tests/c/Makefile) run the same harness with ws_host.c compiled in, and a
differential fuzzer of ws_host.c against the oracle (tests/c/sanitize_drive.c); a sanitizer
report fails the run.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import _oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "tests", "c", "_build")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-C", os.path.join(REPO, "tests", "c")], check=True,
                   stdout=subprocess.DEVNULL)
    return BUILD


def _run(prog, *args, timeout=120, dump=None):
    cmd = [os.path.join(BUILD, prog)] + [str(a) for a in args]
    if dump:
        cmd += ["--dump", dump]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    return json.loads(p.stdout.strip().splitlines()[-1])


def _oracle_echo(tx: bytes):
    """What the echo server must send back for the frames in tx: the oracle decodes them
    (process_data per 16 KiB cut, the live read size) and each message comes back as one
    unmasked FIN|TEXT frame (the reference's build_frame, src/uvhttp_websocket.c:204-285)."""
    orc = _oracle.OracleConn(1, 16 * 1024 * 1024, 64 * 1024 * 1024, record=1)
    for k in range(0, len(tx), 16384):
        assert orc.process_data(tx[k:k + 16384]) == 0
    out = bytearray()
    for kind, _op, payload in orc.events():
        assert kind == "message"
        rc, frame = _oracle.build_frame(payload, 0x1, 0, 1)
        assert rc == len(frame)
        out += frame
    return bytes(out)


def test_c1_one_1kib_frame(built, tmp_path):
    """The BASELINE C1 case itself: one client, one 1 KiB masked BINARY frame, echoed."""
    out = _run("c1_echo", dump=str(tmp_path / "c1"))
    cl = out["clients"][0]
    assert cl["match"] == 1 and cl["sent"] == 1024 + 4 + 4 and cl["echoed"] == 1024 + 4
    assert out["messages"] == 1 and out["errors"] == 0
    assert 0 < out["max_read"] <= 16384
    tx = (tmp_path / "c1.tx.0").read_bytes()
    rx = (tmp_path / "c1.rx.0").read_bytes()
    assert rx == _oracle_echo(tx)
    # the payload really was unmasked: the echo differs from the masked bytes on the wire
    assert rx[4:] != tx[8:]


@pytest.mark.parametrize("clients,frames,size,chunk", [(16, 40, 3000, 777), (4, 6, 70000, 5000),
                                                       (32, 200, 120, 1)])
def test_c1_concurrent_clients(built, tmp_path, clients, frames, size, chunk):
    """N clients on one loop, frames cut into `chunk`-byte writes (frames straddle reads),
    7/16/64-bit length forms; every echo stream equals the oracle's."""
    out = _run("c1_echo", "--clients", clients, "--frames", frames, "--size", size,
               "--chunk", chunk, "--seed", 7, dump=str(tmp_path / "c"))
    assert all(c["match"] for c in out["clients"]) and out["errors"] == 0
    assert out["max_read"] <= 16384 and out["messages"] == clients * frames
    for k in range(clients):
        tx = (tmp_path / f"c.tx.{k}").read_bytes()
        rx = (tmp_path / f"c.rx.{k}").read_bytes()
        assert rx == _oracle_echo(tx)


def test_c1_batcher_host_mode_matches(built):
    """The batcher (uvhttp_ws_amd_batcher_*) with no device: reads queued on the loop and
    decoded at the check-phase flush give the same echo streams as process_data per read."""
    args = ("--clients", 12, "--frames", 30, "--size", 2000, "--chunk", 900, "--seed", 3)
    direct = _run("c1_echo", *args)
    batched = _run("c1_echo", *args, "--batch", 1, "--device", -1)
    assert [c["echo_fnv"] for c in batched["clients"]] == [c["echo_fnv"] for c in direct["clients"]]
    assert all(c["match"] for c in batched["clients"]) and batched["host_reads"] > 0


@pytest.mark.parametrize("args", [(), ("--clients", 8, "--frames", 50, "--size", 3000, "--chunk", 777),
                                  ("--clients", 3, "--frames", 4, "--size", 70000, "--chunk", 4096)])
def test_c1_echo_under_asan_ubsan(built, args):
    """The host decoder (ws_host.c) compiled into the harness under -fsanitize=address,undefined:
    a heap overflow, use-after-free, leak or UB anywhere on the live path aborts the run."""
    out = _run("c1_echo_asan", *args)
    assert all(c["match"] for c in out["clients"]) and out["errors"] == 0


@pytest.mark.parametrize("seed", [1, 2])
def test_host_decoder_fuzz_under_asan_ubsan(built, seed):
    """tests/c/sanitize_drive.c: ws_host.c vs oracle/ws_oracle.c on random frame streams with
    header violations, random limits and random read cuts (state compared after every call),
    parse/mask on random bytes and alignments, TLS oracle seal -> open — all under
    ASan/UBSan."""
    p = subprocess.run([os.path.join(BUILD, "sanitize_drive"), "1500", str(seed)],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "clean" in p.stdout


@pytest.mark.parametrize("sse2", ["0", "1"])
def test_batcher_read_copy_under_asan_ubsan(built, sse2):
    """the batcher's read copy into its pinned arena (ws_host.c uvhttp_ws_amd_copy_stream: AVX2
    or SSE2 streaming stores, one fence per upload) equals memcpy at every length / alignment
    tried and writes nothing outside the destination (tests/c/copy_check.c)"""
    exe = os.path.join(BUILD, "copy_check")
    p = subprocess.run([exe], env=dict(os.environ, UVHTTP_WS_COPY_SSE2=sse2),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.startswith("ok")
