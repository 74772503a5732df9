"""librtx.so loads and exports every entry point include/rtx.h declares (no GPU calls)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT, PKG


def declared():
    text = open(os.path.join(ROOT, "include", "rtx.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rtx_[a-z_0-9]+)\s*\(", text)))


def test_header_and_binding_agree(rtx_mod):
    assert declared() == sorted(rtx_mod.EXPORTS)


def test_every_declared_symbol_is_exported(rtx_mod):
    L = C.CDLL(rtx_mod.LIB_PATH)
    for name in declared():
        assert hasattr(L, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", rtx_mod.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared():
        assert re.search(rf"\bT {name}\b", nm), name


def test_abi_version(rtx_mod):
    assert rtx_mod.lib().rtx_abi_version() == 4


def test_library_is_a_gfx950_code_object(rtx_mod):
    """The HIP kernels are compiled for gfx950 (and only gfx950)."""
    data = open(rtx_mod.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}


def test_no_cpu_fallback_without_device(rtx_mod):
    """Without a HIP device the C ABI fails loudly instead of computing on the CPU."""
    if rtx_mod.device_count() > 0:
        pytest.skip("a GPU is present")
    hs = rtx_mod.HostScene.load(os.path.join(ROOT, "tests", "golden", "scenes", "three.rtxs"))
    with pytest.raises(rtx_mod.RtxError):
        rtx_mod.DeviceScene(hs)


def test_invalid_descriptors_rejected_before_launch(rtx_mod):
    """Bad material/child indices are caught on the host (kernels never read out of bounds)."""
    d = rtx_mod.SceneDesc()
    prims = (rtx_mod.Prim * 1)()
    prims[0].kind, prims[0].material = 0, 3  # material out of range
    d.prims, d.n_prims = prims, 1
    h = C.c_void_p()
    rc = rtx_mod.lib().rtx_scene_create(0, C.byref(d), C.byref(h))
    assert rc == -1 and b"material out of range" in rtx_mod.lib().rtx_last_error()
