#!/usr/bin/env python3
"""oracle/gen_image_golden.py — TEST INFRASTRUCTURE: image-decode fixtures (tests/golden/images/).

Generates small JPEG / PNM files with Pillow (baseline and progressive, 4:4:4 / 4:2:2 / 4:2:0 /
4:1:1 chroma, grayscale, CMYK, restart markers, optimised Huffman tables, 1x1 and odd sizes,
qualities 5..100), decodes each with the reference's own stb_image through
oracle/_ref/ref_harness (`image8`: stbi_load's 8-bit RGB; `imagebytes`: scene::Image's texels
after stbi_loadf + FloatToByte) and writes the files plus tests/golden/images.npz.  The
product's decoder (rt/image.h, rtx_image_load) must reproduce both byte for byte
(tests/test_image_decode.py).  Needs /root/reference (build container only).
"""
import io
import os
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
OUT = os.path.join(ROOT, "tests", "golden", "images")


def picture(w, h, seed):
    """Smooth gradients + edges + noise: exercises every IDCT frequency and chroma upsampling."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    a = np.stack([(x * 255.0 / max(1, w - 1)), (y * 255.0 / max(1, h - 1)), ((x + y) % 32) * 8.0], -1)
    a += rng.normal(0, 18, a.shape)
    a[(x // 5 + y // 7) % 3 == 0] = [250, 20, 40]
    return np.clip(a, 0, 255).astype(np.uint8)


def cases():
    """(name, bytes) of every fixture file."""
    out = []

    def jpg(name, arr, mode="RGB", **kw):
        b = io.BytesIO()
        im = Image.fromarray(arr) if mode in ("RGB", "L") else Image.fromarray(arr).convert(mode)
        im.save(b, "JPEG", **kw)
        out.append((name + ".jpg", b.getvalue()))

    p = picture(37, 23, 1)
    for q in (5, 50, 95, 100):
        for ss, tag in ((0, "444"), (1, "422"), (2, "420")):
            jpg(f"rgb_{tag}_q{q}_37x23", p, quality=q, subsampling=ss)
    big = picture(129, 67, 2)
    jpg("rgb_420_129x67", big, quality=85, subsampling=2)
    jpg("rgb_422_129x67_opt", big, quality=85, subsampling=1, optimize=True)
    jpg("rgb_444_129x67_prog", big, quality=85, subsampling=0, progressive=True)
    jpg("rgb_420_129x67_prog", big, quality=75, subsampling=2, progressive=True)
    jpg("rgb_420_129x67_prog_opt", big, quality=60, subsampling=2, progressive=True, optimize=True)
    jpg("gray_61x17", np.asarray(Image.fromarray(picture(61, 17, 3)).convert("L")), mode="L", quality=80)
    jpg("gray_61x17_prog", np.asarray(Image.fromarray(picture(61, 17, 3)).convert("L")), mode="L", quality=80,
        progressive=True)
    jpg("cmyk_40x24", picture(40, 24, 4), mode="CMYK", quality=90)
    jpg("rgb_1x1", picture(1, 1, 5), quality=90)
    jpg("rgb_2x1_420", picture(2, 1, 6), quality=90, subsampling=2)
    jpg("rgb_17x9_420", picture(17, 9, 7), quality=90, subsampling=2)
    for kw, tag in (({"restart_marker_blocks": 3}, "rst_blocks3"), ({"restart_marker_rows": 1}, "rst_rows1")):
        try:
            jpg(f"rgb_420_129x67_{tag}", big, quality=85, subsampling=2, **kw)
        except TypeError:
            pass
    # binary PNM: a 256-value ramp (stb's gamma step on every byte value), P5 and P6
    ramp = np.arange(256, dtype=np.uint8)
    rgb = np.stack([ramp, ramp[::-1], ((ramp.astype(np.int32) * 7) % 256).astype(np.uint8)], -1).reshape(1, 256, 3)
    out.append(("ramp_256x1.ppm", b"P6\n# ramp\n256 1\n255\n" + rgb.tobytes()))
    out.append(("ramp_16x16.pgm", b"P5\n16 16\n255\n" + ramp.tobytes()))
    return [c for c in out if c is not None]


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the harness first: make -C oracle _ref/ref_harness")
    os.makedirs(OUT, exist_ok=True)
    for f in os.listdir(OUT):
        os.remove(os.path.join(OUT, f))
    z = {}
    with tempfile.TemporaryDirectory() as td:
        for name, data in cases():
            path = os.path.join(OUT, name)
            open(path, "wb").write(data)
            for cmd in ("image8", "imagebytes"):
                o = os.path.join(td, "o.bin")
                subprocess.run([HARNESS, cmd, path, o], check=True)
                raw = np.fromfile(o, dtype=np.uint8)
                w, h = np.frombuffer(raw[:8].tobytes(), dtype=np.int32)
                assert w > 0 and h > 0, (name, cmd)
                z[f"{name}:{cmd}"] = raw[8:].reshape(h, w, 3)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "images.npz"), **z)
    print(f"{len(z) // 2} image fixtures")


if __name__ == "__main__":
    main()
