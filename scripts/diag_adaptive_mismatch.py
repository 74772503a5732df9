#!/usr/bin/env python3
"""Which pixels of an adaptive render differ between the GPU and the CPU oracle, and why.
Renders a band of the workload's frame adaptively on the GPU (fast precision, as the bench) and
on the oracle (philox), lists the pixels whose sample counts or values differ, then renders each
of them alone on the GPU in parity precision: a pixel that parity precision reproduces differs
in fast precision only (an exact-t tie between primitives resolved by the other walk order,
DESIGN.md §1), one that it does not is a bug.
  python3 scripts/diag_adaptive_mismatch.py --workload c4_bunny4k --rows 529 1631"""
import argparse
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))
import bench  # noqa: E402  (WORKLOADS, adaptive constants)
import oracle_ctypes as orc  # noqa: E402
import rtx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4_bunny4k")
    ap.add_argument("--rows", type=int, nargs=2, default=None)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    scene_name, preset, width, spp, depth = bench.WORKLOADS[a.workload]
    host = rtx.HostScene.recipe(scene_name, 1234)
    dev = rtx.DeviceScene(host, device=0)
    cam = rtx.camera(rtx.camera_config(preset, width=width))
    W, H = cam.image_width, cam.image_height
    r0, r1 = a.rows or (0, H)
    tile = (0, r0, W, r1 - r0)
    kw = dict(adaptive=True, mode="persistent", min_spp=bench.ADAPTIVE_MIN_SPP, rel_threshold=bench.ADAPTIVE_REL)
    gpu, gspp, _ = dev.render(cam, spp, depth, seed=a.seed, tile=tile, precision="fast", **kw)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "scene.rtxs")
        host.write(path)
        s = orc.Scene(path)
        t = time.time()
        ref, rspp, _ = s.render(orc.camera_preset(preset), W, spp, depth, a.seed, adaptive=1, rng="philox",
                                mode="per_pixel", tile=tile, threads=a.threads)
        print(f"oracle band {W}x{r1 - r0} in {time.time() - t:.1f}s", flush=True)
    ref, rspp = ref.reshape(-1, 3), rspp.ravel()
    bad = np.nonzero((gspp != rspp) | np.any(gpu != ref, axis=1))[0]
    big = np.nonzero((gspp != rspp) | np.any(np.abs(gpu - ref) > 1e-12 * np.maximum(1.0, np.abs(ref)), axis=1))[0]
    print(f"{len(bad)} pixels differ at all, {len(big)} beyond 1e-12 relative or in sample count", flush=True)
    for i in big[:20]:
        x, y = int(i % W), int(r0 + i // W)
        par, pspp, _ = dev.render(cam, spp, depth, seed=a.seed, tile=(x, y, 1, 1), precision="parity", **kw)
        fas, fspp, _ = dev.render(cam, spp, depth, seed=a.seed, tile=(x, y, 1, 1), precision="fast", **kw)
        print(f"pixel ({x},{y}): spp gpu fast {gspp[i]} (alone {int(fspp[0])}), gpu parity {int(pspp[0])}, cpu {rspp[i]}; "
              f"rgb fast {gpu[i]}, parity {par[0]}, cpu {ref[i]}; parity == cpu: "
              f"{bool(int(pspp[0]) == rspp[i] and np.allclose(par[0], ref[i], rtol=1e-12, atol=0))}", flush=True)


if __name__ == "__main__":
    main()
