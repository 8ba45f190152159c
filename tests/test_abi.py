"""The C-ABI library loads and exports every function include/*.h declares; the device
surface refuses cleanly (ENODEV) where there is no MI355X.  No compute on a GPU here."""
import ctypes as C
import glob
import os
import re

import pytest

import uvhttp_amd as U

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(uvhttp_\w+)\s*\(", src, flags=re.M):
            if "typedef" in src[src.rfind("\n", 0, m.start()) + 1:m.end()]:
                continue
            names.add(m.group(1))
    return sorted(names)


def test_every_declared_symbol_is_exported():
    names = _declared_functions()
    assert len(names) >= 19, names
    L = C.CDLL(U.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_version_string():
    assert b"gfx950" in U.lib().uvhttp_ws_amd_version()


def test_gfx950_code_object_present():
    """The library carries a gfx950 code object (offload bundle)."""
    blob = open(U.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_gpu_means_enodev():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    assert U.lib().uvhttp_ws_gpu_engine_create(0, C.byref(h)) == -2
    assert U.lib().uvhttp_tls_gpu_engine_create(0, C.byref(h)) == -2
    with pytest.raises(U.GpuError):
        U.GpuEngine(0)
    with pytest.raises(U.GpuError):
        U.TlsEngine(0)


def test_product_does_not_reference_oracle():
    """The product library and package never load the oracle (no CPU fallback path)."""
    for p in glob.glob(os.path.join(REPO, "uvhttp_amd", "**", "*"), recursive=True):
        if os.path.isfile(p) and p.endswith((".py", ".c", ".hip", ".h")):
            txt = open(p).read()
            assert "libws_oracle" not in txt and "import _oracle" not in txt, p
    blob = open(U.LIB_PATH, "rb").read()
    assert b"libws_oracle" not in blob and b"oracle_" not in blob


def test_fault_injection_only_in_the_test_build():
    """The batcher's fault-injection variable is read only by the test build
    (libuvhttp_ws_amd_testhooks.so, -DUVWS_TEST_HOOKS); the product library has no such hook."""
    assert b"UVHTTP_WS_BATCHER_FAIL_EVERY" not in open(U.LIB_PATH, "rb").read()
    assert b"UVHTTP_WS_BATCHER_FAIL_EVERY" in open(U.TESTHOOKS_LIB_PATH, "rb").read()


def test_product_library_reads_no_environment():
    """the A/B switches — among them UVHTTP_WS_PLAN_TICKET=0 and
    UVHTTP_WS_WALK_FUSE=1, whose workgroup orderings rely on in-order dispatch — are compiled
    only into the experiment build (-DUVWS_EXPERIMENTS); the product library names none of them
    and imports no getenv at all.  The Python mirror routes an engine created while a switch is
    set to the experiment build."""
    prod = open(U.LIB_PATH, "rb").read()
    exp = open(U.TESTHOOKS_LIB_PATH, "rb").read()
    for k in U.EXPERIMENT_KNOBS:
        assert k.encode() not in prod, k
    for k in ("UVHTTP_WS_PLAN_TICKET", "UVHTTP_WS_WALK_FUSE", "UVHTTP_WS_COMPACT", "UVHTTP_TLS_CRYPT_GRID"):
        assert k.encode() in exp, k
    import subprocess
    syms = subprocess.run(["nm", "-D", "--undefined-only", U.LIB_PATH], capture_output=True,
                          text=True).stdout
    assert " getenv" not in syms and "secure_getenv" not in syms


def test_knob_routes_to_experiment_build(monkeypatch):
    monkeypatch.delenv("UVHTTP_WS_COMPACT", raising=False)
    for k in U.EXPERIMENT_KNOBS:
        monkeypatch.delenv(k, raising=False)
    assert U.default_library() is U.lib()
    monkeypatch.setenv("UVHTTP_WS_WALK", "lane")
    assert U.default_library() is U.test_hooks_library()
