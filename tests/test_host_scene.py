"""Product host side (librtx.so C++ API behind the C ABI) — no GPU needed: scene files,
recipes, SAH BVH layout, cameras.json, Camera::Initialize."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, scene_path

BVH = json.load(open(os.path.join(GOLDEN, "bvh_hashes.json")))
REF = "/root/reference"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bvh_arrays(hs):
    n = hs.arrays()["nodes"]
    boxes = np.stack([n["lo"][:, 0], n["hi"][:, 0], n["lo"][:, 1], n["hi"][:, 1], n["lo"][:, 2], n["hi"][:, 2]], 1)
    links = np.stack([n["left_first"], n["right_count"], n["is_leaf"]], 1).astype(np.uint32)
    return boxes, links, hs.prim_indices()


def content(hs):
    """Per-primitive geometry + resolved material/texture content (ids may differ)."""
    a = hs.arrays()
    t, m = a["textures"], a["materials"]

    def tex(i):
        x = t[i]
        if x["kind"] == 1:
            return (1, float(x["inv_scale"]), tex(x["even"]), tex(x["odd"]))
        return (int(x["kind"]), tuple(x["color"]), int(x["image"]) >= 0)

    out = []
    for q in a["prims"]:
        mm = m[q["material"]]
        mc = (int(mm["kind"]), tuple(mm["albedo"]), float(mm["fuzz"]), float(mm["ref_idx"]),
              tex(mm["texture"]) if mm["kind"] in (0, 3) else None)
        out.append((int(q["kind"]), tuple(q["g"]), mc))
    return out


@pytest.mark.parametrize("scene", ["cornell", "final", "bunny"])
def test_bvh_matches_reference(rtx_mod, scene):
    boxes, links, prims = bvh_arrays(rtx_mod.HostScene.load(scene_path(scene)))
    ref = BVH[scene]
    assert len(links) == ref["nodes"]
    assert (sha(boxes), sha(links), sha(prims)) == (ref["boxes_sha256"], ref["links_sha256"], ref["prims_sha256"])


def test_bvh_matches_reference_mixed(rtx_mod):
    boxes, links, prims = bvh_arrays(rtx_mod.HostScene.recipe("mixed", 1234))
    ref = BVH["mixed"]
    assert (sha(boxes), sha(links), sha(prims)) == (ref["boxes_sha256"], ref["links_sha256"], ref["prims_sha256"])


@pytest.mark.parametrize("scene", ["three", "cornell", "final", "bunny"])
def test_recipes_match_reference_scene_files(rtx_mod, scene):
    a = rtx_mod.HostScene.load(scene_path(scene))
    b = rtx_mod.HostScene.recipe(scene, 1234)
    assert content(a) == content(b)
    assert np.array_equal(a.arrays()["nodes"], b.arrays()["nodes"])


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_harness")),
                    reason="reference harness only exists in the build container")
def test_mixed_recipe_matches_reference_harness(rtx_mod, tmp_path):
    p = str(tmp_path / "mixed.rtxs")
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_harness"), "recipe", "mixed", p], check=True)
    assert content(rtx_mod.HostScene.load(p)) == content(rtx_mod.HostScene.recipe("mixed", 1234))


@pytest.mark.parametrize("scene", ["three", "cornell", "final", "bunny"])
def test_scene_file_round_trip(rtx_mod, tmp_path, scene):
    a = rtx_mod.HostScene.load(scene_path(scene))
    p = str(tmp_path / "x.rtxs")
    a.write(p)
    b = rtx_mod.HostScene.load(p)
    assert content(a) == content(b)
    assert np.array_equal(a.arrays()["nodes"], b.arrays()["nodes"])


def test_leaf_order_prims(rtx_mod):
    """Prims are shipped in leaf order: prims[k] is primitive prim_indices[k] (bvh.h:97-105)."""
    hs = rtx_mod.HostScene.load(scene_path("final"))
    a = hs.arrays()
    pi = hs.prim_indices()
    # list order from the scene file
    lines = [l.split() for l in open(scene_path("final")) if l.startswith("sphere")]
    for k in range(0, len(pi), 37):
        g = [float(x) for x in lines[pi[k]][1:5]]
        assert list(a["prims"][k]["g"][:4]) == g
    leaves = a["nodes"][a["nodes"]["is_leaf"] == 1]
    covered = np.zeros(len(pi), int)
    for n in leaves:
        covered[n["left_first"]:n["left_first"] + n["right_count"]] += 1
    assert np.all(covered == 1)


def test_bad_scene_file_reports_error(rtx_mod, tmp_path):
    p = tmp_path / "bad.rtxs"
    p.write_text("rtxscene 1\nbvh 1\nsphere 0 0 0 1 7\n")
    with pytest.raises(rtx_mod.RtxError, match="material id out of range"):
        rtx_mod.HostScene.load(str(p))
    with pytest.raises(rtx_mod.RtxError, match="cannot open"):
        rtx_mod.HostScene.load(str(tmp_path / "missing.rtxs"))
    with pytest.raises(rtx_mod.RtxError, match="unknown scene recipe"):
        rtx_mod.HostScene.recipe("nope")


def test_empty_and_flat_scenes(rtx_mod, tmp_path):
    p = tmp_path / "empty.rtxs"
    p.write_text("rtxscene 1\nbvh 1\n")
    a = rtx_mod.HostScene.load(str(p)).arrays()
    assert len(a["prims"]) == 0 and len(a["nodes"]) == 0
    flat = rtx_mod.HostScene.load(scene_path("three")).arrays()
    assert len(flat["nodes"]) == 0 and len(flat["prims"]) == 3


PRESETS = ["default", "cornell", "cornell_wide", "wide", "c1_three", "c2_final", "c3_bunny", "c4_bunny4k", "c5_mixed"]


@pytest.mark.parametrize("preset", PRESETS)
def test_camera_matches_oracle(rtx_mod, orc, preset):
    """cameras.json parsing (camera.h:40-67) + Camera::Initialize (camera.h:100-131)."""
    cfg = rtx_mod.camera_config(preset)
    raw = json.load(open(os.path.join(ROOT, "configs", "cameras.json")))[preset]
    assert cfg.image_width == raw["imageWidth"] and cfg.vfov == raw["vfov"]
    assert cfg.samples_per_pixel == raw["samplesPerPixel"] and cfg.max_depth == raw["maxDepth"]
    assert cfg.focus_dist == raw.get("focusDist", 10.0) and cfg.defocus_angle == raw.get("defocusAngle", 0.0)
    cam = rtx_mod.camera(cfg)
    oc = orc.make_camera(raw)
    assert cam.image_height == oc.height
    basis = np.zeros(21)
    import ctypes as C
    orc.lib().orc_camera_init(C.byref(oc), basis.ctypes.data_as(C.c_void_p))
    mine = np.array([*cam.center, *cam.pixel00, *cam.pixel_delta_u, *cam.pixel_delta_v, *cam.u, *cam.v, *cam.w])
    assert np.array_equal(mine, basis)


def test_reference_cameras_json_parses(rtx_mod):
    """The reference's own cameras.json (copied values in configs/) parses identically."""
    if not os.path.exists(os.path.join(REF, "cameras.json")):
        pytest.skip("reference not present")
    for name in ("default", "cornell", "cornell_wide", "wide"):
        a = rtx_mod.camera_config(name, cameras=os.path.join(REF, "cameras.json"))
        b = rtx_mod.camera_config(name)
        assert bytes(a) == bytes(b)


def test_camera_errors(rtx_mod, tmp_path):
    with pytest.raises(rtx_mod.RtxError, match="preset not found"):
        rtx_mod.camera_config("no_such_preset")
    p = tmp_path / "c.json"
    p.write_text('{"x": {"imageWidth": 10}}')
    with pytest.raises(rtx_mod.RtxError, match="missing lookfrom"):
        rtx_mod.camera_config("x", cameras=str(p))
    cfg = rtx_mod.camera_config("c1_three", width=0)
    with pytest.raises(rtx_mod.RtxError):
        rtx_mod.camera(cfg)


def test_image_height_rule(rtx_mod):
    """H = max(1, int(W / aspect)) (camera.h:102-103)."""
    for w, h in ((1200, 675), (1000, 562), (3840, 2160), (400, 225), (1, 1)):
        assert rtx_mod.camera(rtx_mod.camera_config("c2_final", width=w)).image_height == h
