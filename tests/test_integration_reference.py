"""INTEGRATION.md's reference-side files compile against the reference and flatten its scenes
exactly as the product does (CPU only; needs /root/reference, i.e. the build container).

A scratch copy of the reference's src/ gets the read accessors of integration/accessors.txt
(inserted after each class's `public:`); integration/rtx_flatten.h + gpu_ray_integrator.h are
compiled against it together with the reference's material.cc / image.cc and linked with
librtx.so.  The reference's own classes build each scene (the harness loader, main.cc
recipes' data) and its own Bvh; the flattened C-ABI arrays must equal the product's
(rtx_host_scene_desc of the same file): nodes and leaf-order primitives byte for byte, and
every primitive's material/texture parameters.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT, scene_path

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="needs /root/reference")


def patch_headers(src_root):
    for line in open(os.path.join(ROOT, "integration", "accessors.txt")):
        if not line.strip() or line.startswith("#"):
            continue
        header, cls, code = [x.strip() for x in line.split("|", 2)]
        path = os.path.join(src_root, header)
        text = open(path).read()
        key = f"class {cls} "
        i = text.index(key)
        j = text.index("public:", i) + len("public:")
        open(path, "w").write(text[:j] + "\n    " + code + "\n" + text[j:])


@pytest.fixture(scope="module")
def flatten_check(tmp_path_factory, rtx_mod):
    d = tmp_path_factory.mktemp("refint")
    src = d / "src"
    shutil.copytree(os.path.join(REF, "src"), src)
    patch_headers(str(src))
    inc = [f"-I{src}"] + [f"-I{src}/{s}" for s in ("core", "geom", "integrator", "material", "renderer", "scene",
                                                    "third-party")]
    exe = d / "flatten_check"
    cmd = ["g++", "-std=c++20", "-O1", "-fopenmp", "-w", f'-DIMAGE_DIR="{REF}/textures"', *inc,
           f"-I{ROOT}/include", f"-I{ROOT}/integration", f"-I{ROOT}/oracle", "-o", str(exe),
           os.path.join(ROOT, "oracle", "flatten_check.cc"), str(src / "material" / "material.cc"),
           str(src / "scene" / "image.cc"), f"-L{PKG}", "-lrtx", f"-Wl,-rpath,{PKG}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe, d


def resolve(mats, texs, m, texels_by_image):
    """Material m's parameters with its textures inlined (ids differ between flatteners)."""
    mat = mats[m]
    out = [int(mat["kind"])]

    def tex(t):
        x = texs[t]
        k = int(x["kind"])
        if k == 0:
            return ("solid", *x["color"].tolist())
        if k == 1:
            return ("checker", float(x["inv_scale"]), tex(int(x["even"])), tex(int(x["odd"])))
        return ("image", texels_by_image(int(x["image"])))

    if mat["kind"] in (0, 3):
        out.append(tex(int(mat["texture"])))
    elif mat["kind"] == 1:
        out += [*mat["albedo"].tolist(), float(mat["fuzz"])]
    else:
        out.append(float(mat["ref_idx"]))
    return tuple(out)


@pytest.mark.parametrize("scene", ["three", "cornell", "final", "bunny", "rects", "one_triangle", "mixed"])
def test_reference_flatten_equals_product(flatten_check, rtx_mod, tmp_path, scene):
    exe, _ = flatten_check
    path = scene_path(scene)
    if scene == "mixed":
        path = str(tmp_path / "mixed.rtxs")
        rtx_mod.HostScene.recipe("mixed", 1234).write(path)
    prefix = str(tmp_path / scene)
    r = subprocess.run([str(exe), path, os.path.join(REF, "models"), prefix], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr
    ref = {k: np.fromfile(f"{prefix}.{k}", dtype=dt) for k, dt in
           (("prims", rtx_mod.PRIM_DTYPE), ("nodes", rtx_mod.NODE_DTYPE), ("mats", rtx_mod.MAT_DTYPE),
            ("texs", rtx_mod.TEX_DTYPE))}
    dims = np.fromfile(f"{prefix}.imgdims", dtype=np.int32).reshape(-1, 2)
    texels = np.fromfile(f"{prefix}.texels", dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(dims[:, 0] * dims[:, 1] * 3)])
    hs = rtx_mod.HostScene.load(path)
    a = hs.arrays()
    assert ref["nodes"].tobytes() == a["nodes"].tobytes()
    assert np.array_equal(ref["prims"]["kind"], a["prims"]["kind"])
    assert ref["prims"]["g"].tobytes() == a["prims"]["g"].tobytes()
    d = hs.desc()
    prod_imgs = [d.images[i] for i in range(d.n_images)]

    def ref_img(i):
        return (int(dims[i, 0]), int(dims[i, 1]), texels[offs[i]:offs[i + 1]].tobytes()) if i >= 0 else None

    def prod_img(i):
        if i < 0:
            return None
        im = prod_imgs[i]
        buf = (rtx_mod.C.c_uint8 * (im.width * im.height * 3)).from_address(im.texels)
        return (im.width, im.height, bytes(buf))

    cache_r, cache_p = {}, {}
    for pr, pp in zip(ref["prims"]["material"], a["prims"]["material"]):
        if pr not in cache_r:
            cache_r[pr] = resolve(ref["mats"], ref["texs"], int(pr), ref_img)
        if pp not in cache_p:
            cache_p[pp] = resolve(a["materials"], a["textures"], int(pp), prod_img)
        assert cache_r[pr] == cache_p[pp]
