"""Device-side P3 PPM output (SURVEY §8f "on-GPU resolve + PPM output"): the bytes the GPU
formats equal write_color's (core/color.h:18-33 via the oracle's restatement, which the
reference harness pins byte for byte in tests/test_oracle_golden.py)."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu


def _hip():
    """The HIP runtime that librtx.so itself uses, for raw device buffers in the tests."""
    return C.CDLL("libamdhip64.so")


class DevBuf:
    def __init__(self, nbytes):
        self.hip = _hip()
        self.p = C.c_void_p()
        assert self.hip.hipMalloc(C.byref(self.p), C.c_size_t(max(1, nbytes))) == 0
        self.n = nbytes

    def put(self, arr):
        arr = np.ascontiguousarray(arr)
        assert self.hip.hipMemcpy(self.p, arr.ctypes.data_as(C.c_void_p), C.c_size_t(arr.nbytes), 1) == 0

    def get(self, nbytes):
        out = np.zeros(nbytes, np.uint8)
        assert self.hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), self.p, C.c_size_t(nbytes), 2) == 0
        return out.tobytes()

    def __del__(self):
        self.hip.hipFree(self.p)


def test_render_p3_equals_host_writer_and_oracle(rtx_mod, orc, gpu, tmp_path):
    dev = rtx_mod.DeviceScene(rtx_mod.HostScene.load(scene_path("final")))
    cam = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=96))
    W, H = cam.image_width, cam.image_height
    p3, _ = dev.render_p3(cam, 4, 8, seed=5, adaptive=False, mode="persistent", precision="fast")
    rgb, _, _ = dev.render(cam, 4, 8, seed=5, adaptive=False, mode="persistent", precision="fast")
    path = str(tmp_path / "host.ppm")
    rtx_mod.write_ppm(path, rgb, W, H)
    assert p3 == open(path, "rb").read()
    assert p3 == orc.ppm_bytes(rgb.reshape(H, W, 3))
    assert p3.startswith(b"P3\n%d %d\n255\n" % (W, H))


def test_render_p3_tile_header(rtx_mod, gpu):
    dev = rtx_mod.DeviceScene(rtx_mod.HostScene.load(scene_path("three")))
    cam = rtx_mod.camera(rtx_mod.camera_config("c1_three", width=64))
    p3, _ = dev.render_p3(cam, 2, 4, adaptive=False, tile=(5, 3, 17, 9))
    assert p3.startswith(b"P3\n17 9\n255\n") and p3.count(b"\n") == 3 + 17 * 9


def test_encode_p3_device_edge_values(rtx_mod, orc, gpu):
    """Channel values at every byte boundary, negatives, zero, NaN, inf, denormals, >1."""
    b = np.arange(256, dtype=np.float64)
    edges = np.concatenate([(b / 256) ** 2, np.nextafter((b / 256) ** 2, -1), np.nextafter((b / 256) ** 2, 2),
                            [-1.0, -0.0, 0.0, np.nan, np.inf, -np.inf, 5e-324, 1e-300, 0.998001, 0.999 ** 2,
                             np.nextafter(0.999 ** 2, 2), 1.0, 7.5, 1e300]])
    rng = np.random.default_rng(3)
    W, H = 61, 29
    fb = rng.choice(edges, size=(H, W, 3))
    fb[0, :, :] = np.resize(edges, (W, 3))
    dev = rtx_mod.DeviceScene(rtx_mod.HostScene.load(scene_path("three")))
    cap = rtx_mod.lib().rtx_p3_max_bytes(W, H)
    d_rgb, d_out = DevBuf(fb.nbytes), DevBuf(cap)
    d_rgb.put(fb)
    n = dev.encode_p3_device(d_rgb.p.value, W, H, d_out.p.value, cap)
    assert d_out.get(n) == orc.ppm_bytes(fb)


def test_encode_p3_rejects_small_buffer(rtx_mod, gpu):
    dev = rtx_mod.DeviceScene(rtx_mod.HostScene.load(scene_path("three")))
    d_rgb, d_out = DevBuf(8 * 3 * 4), DevBuf(16)
    with pytest.raises(rtx_mod.RtxError):
        dev.encode_p3_device(d_rgb.p.value, 2, 2, d_out.p.value, 16)


def test_encode_p3_large_frame_property(rtx_mod, gpu):
    """4K frame: line count, byte budget, and a sampled set of lines against write_color."""
    W, H = 3840, 2160
    rng = np.random.default_rng(9)
    fb = rng.random((H, W, 3)) ** 3
    dev = rtx_mod.DeviceScene(rtx_mod.HostScene.load(scene_path("three")))
    cap = rtx_mod.lib().rtx_p3_max_bytes(W, H)
    d_rgb, d_out = DevBuf(fb.nbytes), DevBuf(cap)
    d_rgb.put(fb)
    n = dev.encode_p3_device(d_rgb.p.value, W, H, d_out.p.value, cap)
    data = d_out.get(n)
    lines = data.split(b"\n")
    assert lines[:3] == [b"P3", b"%d %d" % (W, H), b"255"] and len(lines) == 3 + W * H + 1 and lines[-1] == b""
    idx = rng.integers(0, W * H, 2000)
    flat = fb.reshape(-1, 3)
    g = np.where(flat[idx] > 0, np.sqrt(flat[idx]), 0.0)
    v = (256 * np.clip(g, 0.0, 0.999)).astype(int)
    for k, i in enumerate(idx):
        assert lines[3 + i] == b"%d %d %d" % tuple(v[k])


def test_cli_output_equals_library_p3(rtx_mod, gpu):
    """The drop-in CLI (main.cc:158-197 surface) prints the device-encoded P3 bytes."""
    import subprocess

    from conftest import ROOT, PKG

    exe = os.path.join(PKG, "raytracer")
    cams = os.path.join(ROOT, "configs", "cameras.json")
    out = subprocess.run([exe, "c1_three", "--scene", "three", "--cameras", cams, "--spp", "2", "--depth", "4",
                          "--fixed", "--seed", "77"], capture_output=True, timeout=120)
    assert out.returncode == 0, out.stderr.decode()
    dev = rtx_mod.DeviceScene(rtx_mod.HostScene.recipe("three"))
    cam = rtx_mod.camera(rtx_mod.camera_config("c1_three", cameras=cams))
    p3, _ = dev.render_p3(cam, 2, 4, seed=77, adaptive=False, mode="wavefront", precision="parity")
    assert out.stdout == p3
