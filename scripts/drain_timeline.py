#!/usr/bin/env python3
"""Launch timelines of the counting build (when the slot counters run dry, when the waves end),
for fixed-spp frames at several spp and for an adaptive frame's phases.  Run on the GPU box:
  RTX_DEBUG_DRAIN=1 RTX_DEBUG_ADAPT=1 python3 scripts/drain_timeline.py
The library prints the timelines on stderr (rtx_capi.hip)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3360-ray-tracer_amd"))
import rtx  # noqa: E402

CASES = [("bunny", "c3_bunny", 1000, 20, "park"), ("final", "c2_final", 1200, 50, "plain")]
for recipe, preset, width, depth, sched in CASES:
    d = rtx.DeviceScene(rtx.HostScene.recipe(recipe, 1234))
    cam = rtx.camera(rtx.camera_config(preset, width=width))
    for spp in (1, 16, 64, 200):
        print(f"== {preset} {spp} spp fixed", file=sys.stderr, flush=True)
        d.render(cam, spp, depth, seed=7, adaptive=False, mode="persistent", precision="fast", count=True,
                 schedule=sched)
    if recipe == "bunny":
        print(f"== {preset} 200 spp adaptive", file=sys.stderr, flush=True)
        d.render(cam, 200, depth, seed=7, adaptive=True, mode="persistent", precision="fast", count=True,
                 schedule=sched)
