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
    assert rtx_mod.lib().rtx_abi_version() == 9


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


@pytest.mark.parametrize("park", [0, 1, 2, 8, 9, 10])
def test_persistent_lds_regions_are_disjoint(rtx_mod, park):
    """The persistent kernel's LDS regions (traversal stacks, throughput, hit point, leaf queue)
    are each lane-interleaved with their own element size, so a byte shared by two regions
    belongs to DIFFERENT lanes in the two — lanes of other waves that run concurrently.  Round 2's
    6-word leaf queue laid over the hit-point words faulted exactly that way (ledger,
    cmp_spec6_fault.txt).  The layout the kernel and the launch share (persist_lds, exported as a
    host-only test hook) must keep every region inside the block's LDS and apart from the others,
    for every stack size the host can choose (the lean walk's exact bound + 1, up to 65), with and
    without a block-wide region after them: an adaptive phase launch's chunk words (park + 8)."""
    f = rtx_mod.lib().rtx_internal_lds_layout
    f.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_uint32)]
    out = (C.c_uint32 * 11)()
    spec, tiles = (park & 3) == 2, bool(park & 8)
    for slots in range(1, 66):
        assert f(slots, park, out) == 0
        stack, thr, hitp, leafq, tl, end, *per_lane = list(out)
        assert (per_lane[3] != 0) == spec and per_lane[0] == slots * (2 if spec else 4)
        assert (per_lane[4] != 0) == tiles
        regions = [(o, o + 256 * b) for o, b in zip((stack, thr, hitp, leafq), per_lane[:4]) if b]
        if tiles:
            regions.append((tl, tl + per_lane[4]))
        regions.sort()
        assert regions[0][0] == 0 and regions[-1][1] == end, (slots, regions, end)
        for (a0, a1), (b0, b1) in zip(regions, regions[1:]):
            assert a1 <= b0, (slots, regions)
        assert thr % 8 == 0 and hitp % 8 == 0 and tl % 8 == 0, (slots, thr, hitp, tl)
        assert end <= 160 * 1024, (slots, end)  # a workgroup may take all 160 KiB


def test_launch_constant_division_is_exact(rtx_mod):
    """FastDiv (rtx_kernels.h): the kernels divide slot and pixel indices by launch constants (the
    group's samples per pixel, the row length, the stripe height) with a multiply-high and two
    shifts; it must equal the integer division for every 32-bit dividend.  Checked on the host
    (the same inline code the kernels run) for divisors 1..4096, powers of two and their
    neighbours to 2^31, and random divisors, against random and boundary dividends."""
    import ctypes as C

    import numpy as np

    f = rtx_mod.lib().rtx_internal_fastdiv
    f.argtypes = [C.c_uint32, C.c_void_p, C.c_int64, C.c_void_p]
    f.restype = C.c_int
    rng = np.random.default_rng(7)
    ds = list(range(1, 4097)) + [(1 << k) + e for k in range(12, 32) for e in (-1, 0, 1)]
    ds += [int(x) for x in rng.integers(4097, 1 << 32, 300)]
    top = np.uint64((1 << 32) - 1)
    for d in ds:
        d = int(min(d, (1 << 32) - 1))
        n = np.concatenate([rng.integers(0, 1 << 32, 512, dtype=np.uint64),
                            np.array([0, 1, d - 1, d, d + 1, 2 * d - 1, 2 * d], dtype=np.uint64),
                            top - np.arange(4, dtype=np.uint64),
                            (top // np.uint64(d)) * np.uint64(d) - np.arange(2, dtype=np.uint64)])
        n = np.clip(n, 0, top).astype(np.uint32)
        out = np.zeros_like(n)
        assert f(d, n.ctypes.data, len(n), out.ctypes.data) == 0
        assert np.array_equal(out, n // np.uint32(d)), d
