#!/usr/bin/env python3
"""Bit-for-bit comparison of two librtx builds (A/B kernel variants) on small renders.

    python scripts/cmp_libs.py A.so B.so      (run on the GPU box)

Each library renders the same scenes in a child process (RTX_LIB selects the build); the
linear framebuffers, per-pixel sample counts and segment counts must be identical for a
variant that claims to be a pure scheduling / code-motion change.
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [  # scene recipe, camera preset, width, spp, depth, mode, precision, adaptive
    ("final", "c2_final", 96, 16, 50, "persistent", "fast", False),
    ("final", "c2_final", 96, 16, 50, "persistent", "parity", True),
    ("mixed", "c5_mixed", 96, 8, 50, "persistent", "fast", False),
    ("bunny", "c3_bunny", 96, 8, 20, "persistent", "fast", False),
    ("cornell", "cornell", 64, 16, 50, "persistent", "fast", False),
    ("final", "c2_final", 64, 8, 50, "wavefront", "fast", False),
    ("final", "c2_final", 48, 100, 50, "persistent", "fast", False),  # many accumulate chunks
    ("bunny", "c3_bunny", 48, 37, 20, "persistent", "fast", False),  # odd K: unaligned runs
    ("bunny", "c3_bunny", 160, 16, 20, "persistent", "fast", False, "park"),  # the PARK kernel, forced
    ("mixed", "c5_mixed", 96, 8, 50, "persistent", "fast", False, "park"),
    ("cornell", "cornell", 64, 16, 50, "persistent", "fast", False, "park"),
    ("bunny", "c3_bunny", 160, 16, 20, "persistent", "fast", False, "park_step"),  # PARK, leaf-step walk
    ("bunny", "c3_bunny", 400, 64, 20, "persistent", "fast", True),  # adaptive, two sub-renders
    ("final", "c2_final", 400, 48, 50, "persistent", "fast", True),
]


def child(out):
    sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))
    import torch  # noqa: F401  (HIP runtime before librtx, as bench.py)

    import rtx

    res = {}
    for i, (scene, preset, w, spp, depth, mode, prec, adaptive, *sched) in enumerate(CASES):
        dev = rtx.DeviceScene(rtx.HostScene.recipe(scene, 1234), device=0)
        cam = rtx.camera(rtx.camera_config(preset, width=w))
        rgb, n, st = dev.render(cam, spp, depth, seed=1234, adaptive=adaptive, mode=mode, precision=prec,
                                **({"schedule": sched[0]} if sched else {}))
        res[f"rgb{i}"], res[f"spp{i}"] = rgb, n
        res[f"rays{i}"] = np.array([st["rays_total"]])
    np.savez(out, **res)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    a, b = sys.argv[1:3]
    outs = []
    for k, lib in enumerate((a, b)):
        out = os.path.join(ROOT, "gpurun_out", f"cmp_{k}.npz")
        env = dict(os.environ, RTX_LIB=os.path.abspath(lib) if lib != "default" else "")
        subprocess.run([sys.executable, __file__, "--child", out], env=env, check=True)
        outs.append(np.load(out))
    report = {}
    ok = True
    for i, case in enumerate(CASES):
        ra, rb = outs[0][f"rgb{i}"], outs[1][f"rgb{i}"]
        same = np.array_equal(ra.view(np.uint64), rb.view(np.uint64))
        frac = float(np.mean(np.all(ra.view(np.uint64) == rb.view(np.uint64), axis=-1)))
        spp_same = np.array_equal(outs[0][f"spp{i}"], outs[1][f"spp{i}"])
        rays_same = int(outs[0][f"rays{i}"][0]) == int(outs[1][f"rays{i}"][0])
        report[" ".join(map(str, case))] = {"bit_identical": bool(same), "pixels_identical": frac,
                                            "spp_identical": bool(spp_same), "rays_identical": bool(rays_same)}
        # adaptive renders trace whole batches, so the segments traced (not the result) depend on
        # the batch schedule
        ok &= same and spp_same and (rays_same or case[7])
    print(json.dumps(report, indent=1))
    print("ALL BIT-IDENTICAL" if ok else "DIFFERENCES FOUND")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
