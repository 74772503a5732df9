#!/usr/bin/env python3
"""Per-rank load of the N-GPU split, measured on ONE GPU.

`bench.py --gpus N` renders one frame split into interleaved row stripes, stripe k -> rank k mod
N, every rank on its own GPU.  A rank's time is that of its own stripe set rendered alone, so
each rank's share is rendered here, one after the other on the single GPU, at the workload's
full size and budget, through the same call the bench makes (rtx_render_multi with the rank's
stripe_index / stripe_count).  Per rank: wall time of the frame (best of `--reps`), the hot
kernel's time, and its segments.  The predicted imbalance of an N-GPU frame is max / mean of the
ranks' times (the bench's value is the whole frame's segments / the slowest rank's time, so the
predicted N-GPU value is segments / max).

usage: python scripts/rank_balance.py [--workload c4_bunny4k] [--ranks 2,4,8] [--stripe-rows 8]
Prints one JSON line per (stripe height, N).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4_bunny4k", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--stripe-rows", default="8")
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--adaptive", action="store_true")
    args = ap.parse_args()
    import torch

    torch.cuda.init()
    import rtx

    scene_name, preset, width, spp, depth = bench.WORKLOADS[args.workload]
    spp = args.spp or spp
    host = rtx.HostScene.recipe(scene_name, 1234)
    dev = rtx.DeviceScene(host, device=0)
    cam = rtx.camera(rtx.camera_config(preset, width=width))
    W, H = cam.image_width, cam.image_height
    fb = torch.empty((W * H, 3), dtype=torch.float64).pin_memory().numpy()
    scenes = (rtx.C.c_void_p * 1)(dev.h.value)

    def frame(srows, idx, count):
        p = rtx.RenderParams()
        p.spp, p.max_depth, p.seed = spp, depth, 1234
        p.adaptive, p.min_spp, p.rel_threshold = int(args.adaptive), bench.ADAPTIVE_MIN_SPP, bench.ADAPTIVE_REL
        p.mode, p.precision = rtx.MODES["persistent"], rtx.PRECISIONS["fast"]
        p.stripe_rows, p.stripe_index, p.stripe_count = srows, idx, count
        st = rtx.Stats()
        t = time.perf_counter()
        rtx._check(rtx.lib().rtx_render_multi(scenes, 1, rtx.C.byref(cam), rtx.C.byref(p), fb.ctypes.data, None,
                                              rtx.C.byref(st), None), "rtx_render_multi")
        return time.perf_counter() - t, st.as_dict()

    frame(8, 0, 8)  # schedule timing and buffers outside the measurements
    for srows in [int(x) for x in args.stripe_rows.split(",")]:
        for n in [int(x) for x in args.ranks.split(",")]:
            per = []
            for k in range(n):
                best = None
                for _ in range(args.reps):
                    t, st = frame(srows, k, n)
                    if best is None or t < best[0]:
                        best = (t, st)
                t, st = best
                per.append({"rank": k, "rows": len(rtx.stripe_rows_of(H, srows, k, n, width=W)), "ms": t * 1e3,
                            "hot_ms": st["hot_kernel_ms"], "segments": st["rays_total"]})
            ms = np.array([r["ms"] for r in per])
            seg = np.array([r["segments"] for r in per], dtype=np.float64)
            print(json.dumps({"workload": args.workload, "spp": spp, "adaptive": args.adaptive, "stripe_rows": srows,
                              "n": n, "imbalance_time": float(ms.max() / ms.mean()),
                              "imbalance_segments": float(seg.max() / seg.mean()),
                              "predicted_value_Mrays": float(seg.sum() / (ms.max() / 1e3) / 1e6),
                              "one_gpu_equiv_Mrays": float(seg.sum() / (ms.sum() / 1e3) / 1e6),
                              "ranks": per}), flush=True)


if __name__ == "__main__":
    main()
