"""GPU parity of the code the benchmark times, and of the multi-device frame.

The persistent fast kernel comes in per-scene builds (rtx_stats.build: sphere/triangle leaf
tests, Lambertian-only shading, no texture lookups, no thin-lens sampling, PARK schedule).
Every build the BASELINE configurations select is compared here with the CPU oracle at the
same Philox seed, on crops of the configurations' own cameras and image sizes:
  * C2 final_scene 1200x675 depth 50 (sphere tree, no textures, no defocus; plain)
  * C3/C4 bunny 1000x562 depth 20 / 3840x2160 depth 50 (triangle tree, Lambertian, no
    textures; PARK)
  * C5 mixed 3840x2160 depth 50 (sphere tree, textures, all three BSDFs; plain and PARK)
  * thin-lens cameras (defocusAngle > 0: the builds with camera disk sampling), every mode
and the generic build must give the same pixels as the specialised ones, bit for bit.

Tolerance: RMS <= 1e-4 on the linear framebuffer; with fixed spp the segment
counts are identical.  Multi-device frames (rtx_render_multi) must be bit-identical to the
single-device frame, however many scenes share the work.
"""
import os

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu
RMS_TOL = 1e-4
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def scenes(rtx_mod, gpu, mixed_scene_file):
    cache = {}

    def get(name):
        if name not in cache:
            path = mixed_scene_file if name == "mixed" else scene_path(name)
            cache[name] = (path, rtx_mod.DeviceScene(rtx_mod.HostScene.load(path)))
        return cache[name]

    return get


def oracle(orc, path, preset, width, spp, depth, seed, tile, adaptive=0, mode="per_pixel", **cam):
    cfg = orc.camera_preset(preset, **cam)
    return orc.Scene(path).render(cfg, width, spp, depth, seed, adaptive=adaptive, rng="philox", mode=mode,
                                  tile=tile, threads=THREADS)


def centre_tile(cam, w, h, dx=0, dy=0):
    return ((cam.image_width - w) // 2 + dx, (cam.image_height - h) // 2 + dy, w, h)


# scene, preset, full width, spp, depth, build of the plain / the PARK schedule
SPH = {"sphere_tree", "no_textures", "no_defocus"}
TRI = {"triangle_tree", "lambertian", "no_textures", "park"}
BENCH_CASES = [
    ("final", "c2_final", 1200, 8, 50, SPH, {"park"}),
    ("bunny", "c3_bunny", 1000, 6, 20, set(), TRI),
    ("bunny", "c4_bunny4k", 3840, 4, 50, set(), TRI),
    ("mixed", "c5_mixed", 3840, 4, 50, {"sphere_tree"}, {"park"}),
]
SPECIALISED = {"sphere_tree", "triangle_tree", "lambertian", "no_textures", "no_defocus", "park", "speculative"}


def want_build(schedule, st, plain_build, park_build):
    """The build a schedule runs: the PARK one walks speculatively on these trees (all under
    65536 BVH4 nodes) unless the leaf-step walk is asked for."""
    if schedule == "park_step":
        return park_build
    if schedule == "plain" or (schedule == "auto" and not st["parked"]):
        return plain_build
    return park_build | {"speculative"}


@pytest.mark.parametrize("schedule", ["plain", "park", "park_step", "auto"])
@pytest.mark.parametrize("case", BENCH_CASES, ids=[c[1] for c in BENCH_CASES])
def test_timed_kernel_builds_match_oracle(rtx_mod, orc, scenes, case, schedule):
    scene, preset, width, spp, depth, plain_build, park_build = case
    path, d = scenes(scene)
    cam = rtx_mod.camera(rtx_mod.camera_config(preset, width=width))
    tile = centre_tile(cam, 40, 24)
    ref, _, ref_st = oracle(orc, path, preset, width, spp, depth, 77, tile)
    rgb, sp, st = d.render(cam, spp, depth, seed=77, adaptive=False, mode="persistent", precision="fast", tile=tile,
                           schedule=schedule)
    names = set(rtx_mod.build_names(st["build"])) & SPECIALISED
    want = want_build(schedule, st, plain_build, park_build)
    assert names == want, (names, want)
    rms = np.sqrt(np.mean((rgb - ref.reshape(-1, 3)) ** 2))
    assert rms <= RMS_TOL, rms
    assert np.all(sp == spp) and st["rays_total"] == ref_st["rays"]


# Whole frames at the configurations' own cameras and sizes against the oracle: C2 and C3 at
# their full budgets (the benchmark's frames themselves), C4 and C5 at reduced spp (the oracle
# finishes each in seconds on the box's host cores).  The benchmark's own schedule (auto).
WHOLE_FRAME_CASES = [  # bench case index, spp
    (0, 100),
    (1, 200),
    (2, 4),
    (3, 2),
]


@pytest.mark.parametrize("wcase", WHOLE_FRAME_CASES, ids=[f"{BENCH_CASES[c[0]][1]}_{c[1]}spp" for c in WHOLE_FRAME_CASES])
def test_whole_frame_matches_oracle(rtx_mod, orc, scenes, wcase):
    ci, spp = wcase
    scene, preset, width, _, depth, _, _ = BENCH_CASES[ci]
    path, d = scenes(scene)
    cam = rtx_mod.camera(rtx_mod.camera_config(preset, width=width))
    ref, ref_spp, ref_st = oracle(orc, path, preset, width, spp, depth, 1234, None)
    rgb, sp, st = d.render(cam, spp, depth, seed=1234, adaptive=False, mode="persistent", precision="fast",
                           schedule="auto")
    assert st["rays_total"] == ref_st["rays"], (st["rays_total"], ref_st["rays"])
    assert np.all(sp == spp) and np.array_equal(sp, ref_spp.ravel())
    rms = np.sqrt(np.mean((rgb - ref.reshape(-1, 3)) ** 2))
    assert rms <= RMS_TOL, rms


# The reference's default sampling (WavefrontRenderer::Render is always adaptive:
# wavefront.cc:42-43 kRelThresh 0.05f / kMinSamples 16, converged pixels skipped at :68-69,
# IsConverged at :125-127), on the timed builds at the configurations' own cameras and
# widths: full-width row bands, with the configurations' sample budgets where the oracle
# finishes in seconds (C2 100, C3 200 spp) and 64 spp for the 4K ones.
ADAPTIVE_CASES = [  # bench case index, spp, band rows
    (0, 100, 2),
    (1, 200, 2),
    (2, 64, 1),
    (3, 64, 1),
]
ADAPTIVE_MIN, ADAPTIVE_REL = 16, float(np.float32(0.05))


@pytest.mark.parametrize("schedule", ["plain", "park", "park_step", "auto"])
@pytest.mark.parametrize("acase", ADAPTIVE_CASES, ids=[BENCH_CASES[c[0]][1] for c in ADAPTIVE_CASES])
def test_timed_kernel_builds_adaptive_match_oracle(rtx_mod, orc, scenes, acase, schedule):
    """Per-pixel sample counts equal the oracle's exactly, pixels within RMS_TOL: whatever
    the group schedule traces past a pixel's convergence is discarded, never recorded."""
    ci, spp, rows = acase
    scene, preset, width, _, depth, plain_build, park_build = BENCH_CASES[ci]
    path, d = scenes(scene)
    cam = rtx_mod.camera(rtx_mod.camera_config(preset, width=width))
    tile = (0, cam.image_height // 2 - rows, cam.image_width, rows)
    ref, ref_spp, ref_st = oracle(orc, path, preset, width, spp, depth, 515, tile, adaptive=1)
    rgb, sp, st = d.render(cam, spp, depth, seed=515, adaptive=True, mode="persistent", precision="fast", tile=tile,
                           schedule=schedule, min_spp=ADAPTIVE_MIN, rel_threshold=ADAPTIVE_REL)
    names = set(rtx_mod.build_names(st["build"])) & SPECIALISED
    want = want_build(schedule, st, plain_build, park_build)
    assert names == want, (names, want)
    ref_spp = ref_spp.ravel()
    assert np.array_equal(sp, ref_spp), (np.nonzero(sp != ref_spp)[0][:5], sp[sp != ref_spp][:5])
    assert ref_spp.min() >= ADAPTIVE_MIN and ref_spp.max() <= spp
    assert st["rays_total"] >= ref_st["rays"] and st["rays_primary"] >= ref_st["primaries"]
    rms = np.sqrt(np.mean((rgb - ref.reshape(-1, 3)) ** 2))
    assert rms <= RMS_TOL, rms


@pytest.mark.parametrize("rows", [2, 70])
@pytest.mark.parametrize("acase", ADAPTIVE_CASES[:2], ids=[BENCH_CASES[c[0]][1] for c in ADAPTIVE_CASES[:2]])
def test_adaptive_recorded_segments_equal_oracle(rtx_mod, orc, scenes, acase, rows):
    """The counting build's rays_recorded (the segments of the samples the pixels record; the
    adaptive bench line's value counts only these) equals the oracle's segment count exactly, and
    the samples traced past convergence are the difference to rays_total (2 and 70 full-width
    rows: a few to thousands of tiles)."""
    ci, spp, _ = acase
    scene, preset, width, _, depth, _, _ = BENCH_CASES[ci]
    path, d = scenes(scene)
    cam = rtx_mod.camera(rtx_mod.camera_config(preset, width=width))
    tile = (0, cam.image_height // 2 - rows // 2, cam.image_width, rows)
    ref, ref_spp, ref_st = oracle(orc, path, preset, width, spp, depth, 515, tile, adaptive=1)
    rgb, sp, st = d.render(cam, spp, depth, seed=515, adaptive=True, mode="persistent", precision="fast", tile=tile,
                           count=True, min_spp=ADAPTIVE_MIN, rel_threshold=ADAPTIVE_REL)
    assert np.array_equal(sp, ref_spp.ravel())
    assert st["rays_recorded"] == ref_st["rays"], (st["rays_recorded"], ref_st["rays"], st["rays_total"])
    assert st["rays_total"] >= st["rays_recorded"]
    _, _, fst = d.render(cam, 4, depth, seed=515, adaptive=False, mode="persistent", precision="fast", tile=tile,
                         count=True)
    assert fst["rays_recorded"] == fst["rays_total"] > 0  # fixed spp: every sample is recorded


# The configurations' own budgets through FORCED small workspaces (rtx_internal_adapt_tune):
# the paths only a large frame at a large budget reaches on its own — a pixel's batches capped
# (phase kcap / workspace), the phase floor few remaining pixels get, many phases — compared
# with the oracle on sample counts, recorded segments and pixels.
FULL_BUDGET_CASES = [(1, 200, 0.7), (3, 2048, 0.5)]  # bench case index, spp, band row (fraction of H)
TUNES = {"phases": {}, "phases_small": dict(phase_slots=4096, phase_kcap=8),
         "phases_kcap4": dict(phase_slots=64, phase_kcap=4), "phases_first_uniform": dict(first_map=0),
         "phases_floor_2e23": dict(phase_slots=1 << 23),
         "phases_unpooled": dict(margin1=1.0, pool_w=0.0)}


@pytest.mark.parametrize("tune", sorted(TUNES))
@pytest.mark.parametrize("fcase", FULL_BUDGET_CASES, ids=[f"{BENCH_CASES[c[0]][1]}_{c[1]}spp" for c in FULL_BUDGET_CASES])
def test_adaptive_full_budget_small_workspace_matches_oracle(rtx_mod, orc, scenes, fcase, tune):
    """One full-width row at the configuration's whole budget (C3 200 spp, C5 2048 spp), with
    the workspace and floors forced small: identical per-pixel sample counts, recorded segments
    equal to the oracle's, RMS <= RMS_TOL."""
    ci, spp, yfrac = fcase
    scene, preset, width, _, depth, _, _ = BENCH_CASES[ci]
    path, d = scenes(scene)
    cam = rtx_mod.camera(rtx_mod.camera_config(preset, width=width))
    tile = (0, int(cam.image_height * yfrac), cam.image_width, 1)
    ref, ref_spp, ref_st = oracle(orc, path, preset, width, spp, depth, 616, tile, adaptive=1)
    knobs = TUNES[tune]
    try:
        rtx_mod.adapt_tune(**knobs)
        rgb, sp, st = d.render(cam, spp, depth, seed=616, adaptive=True, mode="persistent", precision="fast",
                               tile=tile, count=True, min_spp=ADAPTIVE_MIN, rel_threshold=ADAPTIVE_REL)
    finally:
        rtx_mod.adapt_tune()
    ref_spp = ref_spp.ravel()
    assert ref_spp.max() > 64  # the row reaches deep into the budget
    assert np.array_equal(sp, ref_spp), (np.nonzero(sp != ref_spp)[0][:5], sp[sp != ref_spp][:5])
    assert st["rays_recorded"] == ref_st["rays"], (st["rays_recorded"], ref_st["rays"], st["rays_total"])
    rms = np.sqrt(np.mean((rgb - ref.reshape(-1, 3)) ** 2))
    assert rms <= RMS_TOL, rms


@pytest.mark.parametrize("case", BENCH_CASES, ids=[c[1] for c in BENCH_CASES])
def test_generic_build_equals_specialised(rtx_mod, scenes, case):
    """Specialisation compiles out unreachable code only: identical pixels and counts."""
    scene, preset, width, spp, depth, _, _ = case
    _, d = scenes(scene)
    cam = rtx_mod.camera(rtx_mod.camera_config(preset, width=width))
    tile = centre_tile(cam, 64, 32, dy=5)
    a, sa, sta = d.render(cam, spp, depth, seed=3, adaptive=False, mode="persistent", precision="fast", tile=tile)
    b, sb, stb = d.render(cam, spp, depth, seed=3, adaptive=False, mode="persistent", precision="fast", tile=tile,
                          generic=True)
    spec = set(rtx_mod.build_names(stb["build"])) & (SPECIALISED - {"park", "speculative"})
    assert not spec, spec
    assert sta["parked"] == stb["parked"]  # the generic flag keeps the scene's schedule
    assert np.array_equal(a, b) and np.array_equal(sa, sb) and sta["rays_total"] == stb["rays_total"]


def test_c4_full_width_rows_match_oracle(rtx_mod, orc, scenes):
    """C4 (bunny 3840x2160, depth 50): two full-width row bands, far apart, on the timed
    kernel (automatic schedule), against the oracle."""
    path, d = scenes("bunny")
    cam = rtx_mod.camera(rtx_mod.camera_config("c4_bunny4k", width=3840))
    assert (cam.image_width, cam.image_height) == (3840, 2160)
    for y0 in (1000, 1700):
        tile = (0, y0, 3840, 2)
        ref, _, ref_st = oracle(orc, path, "c4_bunny4k", 3840, 2, 50, 4096, tile)
        rgb, _, st = d.render(cam, 2, 50, seed=4096, adaptive=False, mode="persistent", precision="fast", tile=tile)
        rms = np.sqrt(np.mean((rgb - ref.reshape(-1, 3)) ** 2))
        assert rms <= RMS_TOL, (y0, rms)
        assert st["rays_total"] == ref_st["rays"]


DOF = {"defocusAngle": 0.6, "focusDist": 10.0}
DOF_CASES = [  # scene, preset, width, spp, depth, adaptive
    ("final", "c2_final", 48, 6, 50, 1),
    ("bunny", "c3_bunny", 40, 4, 20, 0),
    ("mixed", "c5_mixed", 40, 4, 50, 0),
    ("cornell", "cornell", 30, 8, 20, 1),
]


@pytest.mark.parametrize("precision", ["parity", "fast"])
@pytest.mark.parametrize("mode", ["wavefront", "persistent"])
@pytest.mark.parametrize("case", DOF_CASES, ids=[c[0] for c in DOF_CASES])
def test_defocus_camera_matches_oracle(rtx_mod, orc, scenes, case, mode, precision):
    """Thin-lens cameras (camera.h:134-144 defocus_disk_sample, math_utils.h:83-88
    RandomInUnitDisk rejection loop): the builds that keep camera disk sampling."""
    scene, preset, w, spp, depth, adaptive = case
    path, d = scenes(scene)
    ref, ref_spp, ref_st = oracle(orc, path, preset, w, spp, depth, 606, None, adaptive=adaptive, **DOF)
    cam = rtx_mod.camera(rtx_mod.camera_config(preset, width=w, defocus=DOF["defocusAngle"], focus=DOF["focusDist"]))
    assert cam.defocus_angle > 0
    scheds = ["plain", "park"] if (mode, precision) == ("persistent", "fast") else [None]
    for sched in scheds:
        rgb, sp, st = d.render(cam, spp, depth, seed=606, adaptive=adaptive, mode=mode, precision=precision,
                               schedule=sched)
        assert "no_defocus" not in rtx_mod.build_names(st["build"])
        rms = np.sqrt(np.mean((rgb - ref.reshape(-1, 3)) ** 2))
        assert rms <= RMS_TOL, (sched, rms)
        assert np.array_equal(sp, ref_spp.ravel())
        if not adaptive:
            assert st["rays_total"] == ref_st["rays"]
        if precision == "parity":
            assert np.all(rgb == ref.reshape(-1, 3), 1).mean() >= 0.95


def test_defocus_megakernel_matches_oracle(rtx_mod, orc, scenes):
    path, d = scenes("final")
    ref, _, ref_st = oracle(orc, path, "c2_final", 32, 3, 50, 91, None, mode="megakernel", **DOF)
    cam = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=32, defocus=0.6, focus=10.0))
    for precision in ("parity", "fast"):
        rgb, _, st = d.render(cam, 3, 50, seed=91, adaptive=False, mode="megakernel", precision=precision)
        assert np.sqrt(np.mean((rgb - ref.reshape(-1, 3)) ** 2)) <= RMS_TOL
        assert st["rays_total"] == ref_st["rays"]


def test_defocus_changes_the_image(rtx_mod, scenes):
    """Guard: the thin-lens path is really taken (a pinhole render differs)."""
    _, d = scenes("final")
    cam0 = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=48))
    cam1 = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=48, defocus=0.6, focus=10.0))
    a, _, _ = d.render(cam0, 4, 50, seed=1, adaptive=False, mode="persistent", precision="fast")
    b, _, _ = d.render(cam1, 4, 50, seed=1, adaptive=False, mode="persistent", precision="fast")
    assert not np.array_equal(a, b)


# ---- multi-device frame (rtx_render_multi) -------------------------------------------------

def test_render_multi_same_device_twice_is_bit_identical(rtx_mod, scenes):
    """Two (and three) scenes on device 0, each with its own host thread and stream, split
    the frame into interleaved stripes; the gathered frame equals the one-device frame."""
    path, d = scenes("final")
    cam = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=96))
    full, fsp, fst = d.render(cam, 5, 50, seed=12, adaptive=False, mode="persistent", precision="fast")
    extra = [rtx_mod.DeviceScene(rtx_mod.HostScene.load(path)) for _ in range(2)]
    for group in ([d, extra[0]], [d, extra[0], extra[1]]):
        for rows in (8, 3):
            rgb, sp, st, per = rtx_mod.render_multi(group, cam, 5, 50, seed=12, adaptive=False, stripe_rows=rows)
            assert np.array_equal(rgb, full) and np.array_equal(sp, fsp), (len(group), rows)
            assert st["rays_total"] == fst["rays_total"] and sum(p["rays_total"] for p in per) == st["rays_total"]
            assert all(p["rays_total"] > 0 for p in per)


def test_render_multi_adaptive_and_parity(rtx_mod, scenes):
    path, d = scenes("cornell")
    cam = rtx_mod.camera(rtx_mod.camera_config("cornell", width=40))
    other = rtx_mod.DeviceScene(rtx_mod.HostScene.load(path))
    full, fsp, _ = d.render(cam, 24, 20, seed=5, adaptive=True, mode="wavefront", precision="parity")
    rgb, sp, _, _ = rtx_mod.render_multi([d, other], cam, 24, 20, seed=5, adaptive=True, mode="wavefront",
                                         precision="parity")
    assert np.array_equal(rgb, full) and np.array_equal(sp, fsp)


def test_render_multi_partial_stripes_write_only_their_rows(rtx_mod, scenes):
    """A process that owns stripes 1 and 2 of 4 writes exactly those rows of the shared
    frame (the bench's multi-process gather)."""
    path, d = scenes("final")
    cam = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=64))
    H, W = cam.image_height, cam.image_width
    full, _, _ = d.render(cam, 3, 50, seed=8, adaptive=False, mode="persistent", precision="fast")
    other = rtx_mod.DeviceScene(rtx_mod.HostScene.load(path))
    sentinel = -7.0
    out = np.full((H * W, 3), sentinel)
    rtx_mod.render_multi([d, other], cam, 3, 50, seed=8, adaptive=False, stripe_rows=4, stripe_index=1,
                         stripe_count=4, out=out)
    mine = set(rtx_mod.stripe_rows_of(H, 4, 1, 4)) | set(rtx_mod.stripe_rows_of(H, 4, 2, 4))
    o, f = out.reshape(H, W, 3), full.reshape(H, W, 3)
    for y in range(H):
        if y in mine:
            assert np.array_equal(o[y], f[y]), y
        else:
            assert np.all(o[y] == sentinel), y


def test_render_multi_into_pinned_buffer(rtx_mod, scenes):
    """A pinned caller framebuffer receives the stripes by strided DMA: same bytes."""
    import torch

    path, d = scenes("final")
    cam = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=80))
    full, _, _ = d.render(cam, 2, 50, seed=4, adaptive=False, mode="persistent", precision="fast")
    other = rtx_mod.DeviceScene(rtx_mod.HostScene.load(path))
    pinned = torch.zeros((cam.image_width * cam.image_height, 3), dtype=torch.float64).pin_memory()
    out = pinned.numpy()
    rtx_mod.render_multi([d, other], cam, 2, 50, seed=4, adaptive=False, out=out)
    assert np.array_equal(out, full)


def test_render_multi_banded_output_one_device(rtx_mod, scenes):
    """The benchmark's path: one device, a pinned whole-frame buffer, the last sample group's
    accumulate in bands whose device-to-host copies overlap the next band (BandSink), the
    output resolved by the accumulate itself.  Against rtx_render (one copy at the end), for
    one and several sample groups, a frame height that is no multiple of the stripe height,
    and the three modes' fixed-spp sums."""
    import torch

    path, d = scenes("final")
    cam = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=76))  # 42 rows
    npix = cam.image_width * cam.image_height
    for mode, precision in (("persistent", "fast"), ("wavefront", "parity"), ("megakernel", "fast")):
        for group in (0, 2):
            full, fsp, fst = d.render(cam, 5, 50, seed=21, adaptive=False, mode=mode, precision=precision,
                                      samples_per_group=group)
            pinned = torch.full((npix, 3), -1.0, dtype=torch.float64).pin_memory()
            out = pinned.numpy()
            rgb, sp, st, _ = rtx_mod.render_multi([d], cam, 5, 50, seed=21, adaptive=False, mode=mode,
                                                  precision=precision, out=out, samples_per_group=group)
            assert np.array_equal(out, full) and np.array_equal(sp, fsp), (mode, group)
            assert st["rays_total"] == fst["rays_total"]


def test_render_multi_adaptive_early_output_into_pinned_buffer(rtx_mod, scenes):
    """The benchmark's adaptive path: once a phase holds at most npix / 32 pixels (kEarlyOutDiv),
    the output goes to the pinned caller framebuffer early (copy stream) and the device writes the
    remaining pixels' final values into it at the end (k_patch_host).  Against rtx_render (no
    sink, one resolve at the end): same bytes and sample counts, for one device and for two
    (interleaved stripes), with the default phases and with forced small ones; at the bench's
    frame size the early output must have fired, with pixels patched, on every device."""
    import torch

    path, d = scenes("bunny")
    other = rtx_mod.DeviceScene(rtx_mod.HostScene.load(path))
    for width, knobs in ((120, {}), (120, dict(phase_slots=64, phase_kcap=8)), (1000, {})):
        try:
            rtx_mod.adapt_tune(**knobs)
            cam = rtx_mod.camera(rtx_mod.camera_config("c3_bunny", width=width))
            npix = cam.image_width * cam.image_height
            full, fsp, _ = d.render(cam, 200, 20, seed=33, adaptive=True, mode="persistent", precision="fast")
            for group in ([d], [d, other]):
                n0, p0 = rtx_mod.early_output_stats()
                pinned = torch.full((npix, 3), -1.0, dtype=torch.float64).pin_memory()
                out = pinned.numpy()
                rgb, sp, st, _ = rtx_mod.render_multi(group, cam, 200, 20, seed=33, adaptive=True, mode="persistent",
                                                      precision="fast", out=out)
                assert np.array_equal(out, full) and np.array_equal(sp, fsp), (knobs, len(group))
                assert (fsp < 200).any() and (fsp > 16).any()  # phases past the first ran
                n1, p1 = rtx_mod.early_output_stats()
                # the bench's frame (C3, 1000 wide): a late phase holds <= npix / 32 pixels, so the
                # output goes early and the device patches those pixels (at 120 wide the pixels at
                # the budget end together, in one phase: no early output)
                if width == 1000:
                    assert n1 - n0 == len(group) and p1 > p0, (n0, n1, p0, p1)
        finally:
            rtx_mod.adapt_tune()


def test_render_multi_rejects_bad_arguments(rtx_mod, scenes):
    _, d = scenes("final")
    cam = rtx_mod.camera(rtx_mod.camera_config("c2_final", width=16))
    with pytest.raises(rtx_mod.RtxError, match="twice"):
        rtx_mod.render_multi([d, d], cam, 1, 5)
    with pytest.raises(rtx_mod.RtxError, match="stripe_count"):
        rtx_mod.render_multi([d], cam, 1, 5, stripe_index=2, stripe_count=2)


def test_encode_p3_matches_device_render_p3(rtx_mod, scenes):
    _, d = scenes("cornell")
    cam = rtx_mod.camera(rtx_mod.camera_config("cornell", width=30))
    p3, _ = d.render_p3(cam, 4, 10, seed=2, adaptive=False, mode="persistent")
    rgb, _, _ = d.render(cam, 4, 10, seed=2, adaptive=False, mode="persistent")
    assert rtx_mod.encode_p3(d, rgb, cam.image_width, cam.image_height) == p3


def test_schedule_timing_is_ordered_after_user_stream_work(rtx_mod, scenes):
    """The first fast persistent render of a scene times its two schedules on scratch
    buffers shared with every render: on the caller's stream, so a render still queued there
    is not overwritten."""
    import torch

    path, _ = scenes("bunny")
    cam = rtx_mod.camera(rtx_mod.camera_config("c3_bunny", width=160))
    ref_dev = rtx_mod.DeviceScene(rtx_mod.HostScene.load(path))
    want_a, _, _ = ref_dev.render(cam, 6, 20, seed=21, adaptive=False, mode="wavefront", precision="parity")
    want_b, _, _ = ref_dev.render(cam, 6, 20, seed=22, adaptive=False, mode="persistent", precision="fast")
    fresh = rtx_mod.DeviceScene(rtx_mod.HostScene.load(path))  # schedule not yet timed
    npix = cam.image_width * cam.image_height
    a = torch.empty((npix, 3), dtype=torch.float64, device="cuda:0")
    b = torch.empty((npix, 3), dtype=torch.float64, device="cuda:0")
    s = torch.cuda.Stream()
    pa, pb = rtx_mod.RenderParams(), rtx_mod.RenderParams()
    for p, seed, mode, prec in ((pa, 21, 0, 0), (pb, 22, 1, 1)):
        p.spp, p.max_depth, p.adaptive, p.seed, p.mode, p.precision = 6, 20, 0, seed, mode, prec
    # no stats: the first call returns with its render still queued on s
    fresh.render_device(cam, pa, a.data_ptr(), 0, stream=s.cuda_stream, stats=False)
    fresh.render_device(cam, pb, b.data_ptr(), 0, stream=s.cuda_stream, stats=False)  # times the schedules first
    s.synchronize()
    assert np.array_equal(a.cpu().numpy(), want_a)
    assert np.array_equal(b.cpu().numpy(), want_b)


def test_restated_sincos_is_the_library_bit_for_bit(rtx_mod, gpu):
    """The plain kernel's Lambertian cos/sin of 2*pi*r1 come from a restatement of the device
    library's small-argument path (rtx_device.h sincos_small, one reduction each, no
    Payne-Hanek branch): on 2^24 random draws r1 (the reference's 53-bit uniforms) and around
    0, 1/4, 1/2, 3/4 and the largest draw, both must equal the library's cos() and sin() bit
    for bit."""
    import ctypes as C

    f = rtx_mod.lib().rtx_internal_check_sincos
    f.argtypes = [C.c_int, C.c_int64, C.c_uint64, C.POINTER(C.c_int64), C.POINTER(C.c_double)]
    f.restype = C.c_int
    bad, first = C.c_int64(-1), C.c_double(0.0)
    for seed in (1, 0x5EED):
        assert f(0, 1 << 24, seed, C.byref(bad), C.byref(first)) == 0, rtx_mod.lib().rtx_last_error()
        assert bad.value == 0, f"{bad.value} mismatches, first at u = {first.value!r}"
