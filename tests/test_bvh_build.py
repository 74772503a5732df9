"""BVH build (SURVEY §8f "GPU BVH build"): rtx_bvh_build (device) and rtx_bvh_build_host
produce the reference's node array and prim_indices byte for byte.  The host builder is
pinned to the reference's own Bvh::Build by tests/golden (test_oracle_golden.py BVH dumps
and hashes); here the raw-box entry points are checked against the scenes' BVHs, and the
device build against the host build on the scenes and on adversarial box sets."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, scene_path

BVH_SCENES = ["cornell", "final", "bunny", "mixed"]


def original_order_bounds(rtx_mod, host):
    """Primitive boxes in the order the builder saw them (before the leaf permutation)."""
    a = host.arrays()
    idx = host.prim_indices()
    leaf_bounds = rtx_mod.prim_bounds(a["prims"])
    b = np.zeros_like(leaf_bounds)
    b[idx] = leaf_bounds
    return b, a["nodes"], idx


def host_scene(rtx_mod, name, mixed_scene_file):
    return rtx_mod.HostScene.load(mixed_scene_file if name == "mixed" else scene_path(name))


@pytest.mark.parametrize("scene", BVH_SCENES)
def test_host_raw_box_build_reproduces_scene_bvh(rtx_mod, mixed_scene_file, scene):
    host = host_scene(rtx_mod, scene, mixed_scene_file)
    bounds, nodes, idx = original_order_bounds(rtx_mod, host)
    n2, i2 = rtx_mod.bvh_build(bounds, on="host")
    assert n2.tobytes() == nodes.tobytes()
    assert np.array_equal(i2.astype(np.int64), idx.astype(np.int64))


def test_host_build_matches_reference_hashes(rtx_mod, mixed_scene_file):
    """Ties the raw-box builder to the reference's own dumps (bvh_hashes.json)."""
    ref = json.load(open(os.path.join(GOLDEN, "bvh_hashes.json")))

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    for scene in BVH_SCENES:
        host = host_scene(rtx_mod, scene, mixed_scene_file)
        bounds, _, _ = original_order_bounds(rtx_mod, host)
        n, idx = rtx_mod.bvh_build(bounds, on="host")
        boxes = np.stack([n["lo"][:, 0], n["hi"][:, 0], n["lo"][:, 1], n["hi"][:, 1], n["lo"][:, 2], n["hi"][:, 2]], 1)
        links = np.stack([n["left_first"], n["right_count"], n["is_leaf"]], 1).astype(np.uint32)
        r = ref[scene]
        assert len(n) == r["nodes"]
        assert (sha(boxes), sha(links), sha(idx.astype(np.int32))) == (r["boxes_sha256"], r["links_sha256"],
                                                                        r["prims_sha256"])


def adversarial_boxes(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        c = rng.random((n, 3)) * 100 - 50
        e = rng.random((n, 3))
    elif kind == "clustered":
        c = rng.normal(size=(n, 3)) * np.array([1, 10, 100]) + rng.integers(0, 4, (n, 1)) * 37.0
        e = rng.random((n, 3)) * 0.1
    elif kind == "duplicates":  # many identical boxes: zero centroid extent
        c = np.repeat(rng.random((max(1, n // 50), 3)), 50, axis=0)[:n]
        e = np.full((n, 3), 0.25)
    elif kind == "signed_zero":  # coordinates that are exactly +-0 in unions
        c = rng.integers(-2, 3, (n, 3)).astype(np.float64)
        e = rng.integers(0, 2, (n, 3)).astype(np.float64)
        lo, hi = c - e, c + e
        lo[rng.random((n, 3)) < 0.3] = -0.0
        hi[rng.random((n, 3)) < 0.3] = 0.0
        return np.concatenate([np.minimum(lo, hi), np.maximum(lo, hi)], axis=1)
    else:  # flat: a plane of boxes (one axis degenerate)
        c = np.concatenate([rng.random((n, 2)) * 10, np.zeros((n, 1))], axis=1)
        e = np.concatenate([rng.random((n, 2)) * 0.2, np.zeros((n, 1))], axis=1)
    return np.concatenate([c - e, c + e], axis=1)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", BVH_SCENES)
def test_device_build_equals_host_on_scenes(rtx_mod, gpu, mixed_scene_file, scene):
    host = host_scene(rtx_mod, scene, mixed_scene_file)
    bounds, nodes, idx = original_order_bounds(rtx_mod, host)
    dn, di = rtx_mod.bvh_build(bounds, on="gpu")
    assert dn.tobytes() == nodes.tobytes()
    assert np.array_equal(di.astype(np.int64), idx.astype(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["uniform", "clustered", "duplicates", "signed_zero", "flat"])
@pytest.mark.parametrize("n", [1, 4, 5, 17, 1000, 40000])
def test_device_build_equals_host_adversarial(rtx_mod, gpu, kind, n):
    b = adversarial_boxes(kind, n, seed=n)
    hn, hi = rtx_mod.bvh_build(b, on="host")
    dn, di = rtx_mod.bvh_build(b, on="gpu")
    assert dn.tobytes() == hn.tobytes()
    assert np.array_equal(di, hi)


@pytest.mark.gpu
def test_device_build_empty_and_errors(rtx_mod, gpu):
    n, i = rtx_mod.bvh_build(np.zeros((0, 6)), on="gpu")
    assert len(n) == 0 and len(i) == 0
