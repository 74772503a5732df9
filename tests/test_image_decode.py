"""Image decode (rt/image.h via rtx_image_load) against the reference's own stb_image.

Image::Load (scene/image.cc:16-73) reads textures with stb_image v2.30's stbi_loadf: an 8-bit
decode, then the gamma-2.2 float conversion and Image::FloatToByte.  The fixtures under
tests/golden/images/ (Pillow-written JPEG / PNM: baseline and progressive, 4:4:4 / 4:2:2 /
4:2:0 chroma, grayscale, CMYK, restart markers, optimised Huffman tables, odd sizes, every
byte value through the gamma step) were decoded by the reference's compiled stb
(oracle/gen_image_golden.py): both the 8-bit decode and the texels must match byte for byte,
and so must the earthmap texture the C5 scene samples (tests/golden/textures/earthmap.ppm).
CPU only (no device is needed for image decode).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, PKG

IMAGES = os.path.join(GOLDEN, "images")
Z = np.load(os.path.join(GOLDEN, "images.npz"))
NAMES = sorted({k.split(":")[0] for k in Z.files})


@pytest.mark.parametrize("name", NAMES)
def test_decode_matches_reference_stb(rtx_mod, name):
    path = os.path.join(IMAGES, name)
    got8 = rtx_mod.image_load(path, linear8=True)
    assert np.array_equal(got8, Z[f"{name}:image8"]), (name, int(np.abs(got8.astype(int) - Z[f"{name}:image8"]).max()))
    tex = rtx_mod.image_load(path)
    assert np.array_equal(tex, Z[f"{name}:imagebytes"]), name


def test_every_byte_value_through_the_gamma_step(rtx_mod):
    """The 256-value ramp covers stb's (float)pow(b / 255.0f, 2.2f) and FloatToByte for
    every possible input byte."""
    z = Z["ramp_256x1.ppm:imagebytes"][0]
    got = rtx_mod.image_load(os.path.join(IMAGES, "ramp_256x1.ppm"))[0]
    assert np.array_equal(got, z)
    assert set(range(256)) == set(Z["ramp_256x1.ppm:image8"][0, :, 0].tolist())


def test_earthmap_texels_equal_the_reference_decode(rtx_mod):
    got = rtx_mod.image_load(os.path.join(PKG, "assets", "earthmap.jpg"))
    data = open(os.path.join(GOLDEN, "textures", "earthmap.ppm"), "rb").read()
    head = b"P6\n1024 512\n255\n"
    assert data.startswith(head)
    ref = np.frombuffer(data[len(head):], dtype=np.uint8).reshape(512, 1024, 3)
    assert np.array_equal(got, ref)


def test_mixed_scene_uses_the_decoded_texture(rtx_mod):
    """The C5 recipe's ImageTexture("earthmap.jpg") is decoded from the shipped JPEG."""
    hs = rtx_mod.HostScene.recipe("mixed", 1234)
    d = hs.desc()
    assert d.n_images == 1
    im = d.images[0]
    assert (im.width, im.height) == (1024, 512)
    buf = (rtx_mod.C.c_uint8 * (1024 * 512 * 3)).from_address(im.texels)
    ref = open(os.path.join(GOLDEN, "textures", "earthmap.ppm"), "rb").read()[len(b"P6\n1024 512\n255\n"):]
    assert bytes(buf) == ref


def test_unsupported_and_corrupt_files_fail_cleanly(rtx_mod, tmp_path):
    p = tmp_path / "x.png"
    p.write_bytes(b"\x89PNG\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(rtx_mod.RtxError, match="unknown image type"):
        rtx_mod.image_load(str(p))
    q = tmp_path / "trunc.jpg"
    q.write_bytes(open(os.path.join(IMAGES, NAMES[0]), "rb").read()[:20])
    with pytest.raises(rtx_mod.RtxError):
        rtx_mod.image_load(str(q))
    with pytest.raises(rtx_mod.RtxError):
        rtx_mod.image_load(str(tmp_path / "missing.jpg"))
