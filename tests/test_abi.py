"""CPU tests of the C-ABI library: it loads, exports every symbol include/picp_c.h declares,
and fails cleanly (status code, no crash) when no HIP device is present.  No compute calls.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "picp_c.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(picp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import picp_amd
    L = picp_amd.lib()
    names = _declared()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert sorted(picp_amd.EXPORTED) == names
    out = subprocess.run(["nm", "-D", "--defined-only", picp_amd.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(r"\bT %s\b" % n, out), n


def test_abi_version_and_defaults():
    import picp_amd
    assert picp_amd.lib().picp_abi_version() == 3  # 3: picp_match_batch_form, picp_shard_pad/unpack
    p = picp_amd.default_params()
    assert (p.threshold, p.damping, p.min_inliers, p.keep_outliers, p.max_rounds) == (1000.0, 1.0, 0, 0, 50)
    assert abs(p.conv_eps - 1e-5) < 1e-12


def test_library_has_gfx950_code_object():
    import picp_amd
    blob = open(picp_amd.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # offload bundle target id


def test_shipped_environment_switches_are_the_documented_ones():
    """Every PICP_* variable the shipped library can read is a row of INTEGRATION.md §4, and none
    of the diagnostic (result-changing) ones is among them (diagnostics live in
    diagnostic builds only)."""
    import picp_amd
    blob = open(picp_amd.LIB_PATH, "rb").read()
    names = set(re.findall(rb"\x00(PICP_[A-Z0-9_]+)\x00", blob))
    names = {n.decode() for n in names}
    assert "PICP_MODE" in names
    for diag in ("PICP_VO_DIAG_SKIP", "PICP_MATCH_ACCEPT_ONLY", "PICP_MATCH_EXACT"):
        assert diag not in names, diag
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 4."):doc.index("## 5.")]
    missing = sorted(n for n in names if "`%s" % n not in sec)
    assert not missing, missing
    # and the other way: every switch the table documents is one the library still reads (a
    # variant removed from the library leaves no row behind)
    documented = set()
    for row in sec.splitlines():
        if row.startswith("| `PICP_"):
            documented |= set(re.findall(r"`(PICP_[A-Z0-9_]+)", row.split(" | ")[0]))
    read = {n.decode() for n in re.findall(rb"PICP_[A-Z0-9_]+", blob)}  # any string, merged or not
    stale = sorted(documented - read)
    assert not stale, stale


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"), reason="no llvm-objdump")
def test_shipped_device_code_has_no_packed_fp32_and_no_calls():
    """every kernel of the shipped library is built without packed-FP32 VALU code
    (lane-dependent results beside MFMA work on MI355X) and with everything inlined (a per-kernel
    target attribute once left HIP's header functions as real calls, C2 -18 %, C5 -80 %)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import codeobj
    import picp_amd
    c = codeobj.census(picp_amd.LIB_PATH)
    assert len(c) >= 30
    bad = {s: n for s, n in c.items() if n["pk_f32"] or n["calls"]}
    assert not bad, bad


def test_null_arguments_are_rejected_without_device():
    import picp_amd
    L = picp_amd.lib()
    assert L.picp_device_count(None) == picp_amd.ERR_ARG
    assert L.picp_create(None, 0, 480, 640, None) == picp_amd.ERR_ARG
    assert L.picp_batch_create(None, 0, 1, None, 480, 640, None) == picp_amd.ERR_ARG
    assert L.picp_projection_matrix(None, None, None) == picp_amd.ERR_ARG
    assert L.picp_destroy(None) == 0 and L.picp_batch_destroy(None) == 0
    assert L.picp_last_error()  # a message was recorded


def test_no_device_fails_loudly_not_silently():
    """On a host without a GPU the compute entry points return an error code (no fallback)."""
    import picp_amd
    n = ctypes.c_int(-1)
    rc = picp_amd.lib().picp_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    with pytest.raises(picp_amd.PicpError):
        picp_amd.PICPSolver()
    with pytest.raises(picp_amd.PicpError):
        picp_amd.triangulate(np.eye(3, 4), np.eye(3, 4), np.zeros((1, 2)), np.zeros((1, 2)))


def test_projection_matrix_host_helper(oracle):
    import picp_amd
    from picp_amd import synth
    K = picp_amd.K_REF
    T = synth.rigid_inverse(synth.world_in_camera((1.0, -2.0, 0.3))).astype(np.float32)
    np.testing.assert_array_equal(picp_amd.projection_matrix(K, T), oracle.projection_matrix(K, T))
