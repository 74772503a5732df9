#!/usr/bin/env python3
"""Fixed cost of one persistent launch: hot-kernel time (HIP events, rtx_stats.hot_kernel_ms)
of small renders, by scene, schedule, width and spp.  Run on the GPU box:
    python scripts/launch_cost.py > gpurun_out/launch_cost.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))
import rtx  # noqa: E402

CASES = [("bunny", "c3_bunny", 20), ("final", "c2_final", 50)]
for scene, preset, depth in CASES:
    d = rtx.DeviceScene(rtx.HostScene.recipe(scene, 1234))
    for width in (1000, 250, 64):
        cam = rtx.camera(rtx.camera_config(preset, width=width))
        for sched in ("park", "plain"):
            for spp in (1, 4, 16):
                ts = []
                for _ in range(6):
                    _, _, st = d.render(cam, spp, depth, seed=1, adaptive=False, mode="persistent", precision="fast",
                                        schedule=sched)
                    ts.append(st["hot_kernel_ms"])
                ts = sorted(ts[1:])
                print(f"{scene:6s} w={width:5d} {sched:5s} spp={spp:3d} segs={st['rays_total']:10d} "
                      f"hot_ms min {ts[0]:.3f} med {ts[len(ts) // 2]:.3f}", flush=True)
