#!/usr/bin/env python3
"""scripts/calibrate_cpu.py — TEST INFRASTRUCTURE (needs oracle/_ref/ref_harness, built in the build
container from the reference's sources by oracle/Makefile; it travels to the GPU box with the tree).

Times the reference's own renderer (oracle/_ref/ref_harness: the reference's CPURayIntegrator,
materials and PixelState driven by the Render() glue of wavefront.cc:40-242; its OpenMP
IntersectBatch and, as the reference runs it, its OpenMP shading loop on REF_THREADS threads) and the CPU restatement used as bench.py's
cpu_baseline (oracle/librtx_oracle.so, per-pixel Philox mode, OpenMP) on identical
configurations and the same number of threads, fixed spp.  The ratio port/reference
calibrates bench.py's cpu_baseline against the reference.

Writes profiles/cpu_calibration.json, or --out.  Usage:
    python scripts/calibrate_cpu.py [--threads 8] [--out F] [--host "text"]
The models directory is the reference's when it is present, else the package's assets (the
same stanford-bunny.obj), so the same harness can run on the GPU box's host cores.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
MODELS = "/root/reference/models" if os.path.isdir("/root/reference/models") else \
    os.path.join(ROOT, "3360-ray-tracer_amd", "assets")
# name, scene, preset, width, spp, depth (fixed spp; C2-C5 at reduced spp, the rate is per segment)
CASES = [
    ("c1_three", "three", "c1_three", 400, 4, 4),
    ("c2_final", "final", "c2_final", 1200, 2, 50),
    ("c3_bunny", "bunny", "c3_bunny", 1000, 4, 20),
    ("c5_mixed", "mixed", "c5_mixed", 3840, 1, 50),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_calibration.json"))
    ap.add_argument("--host", default=f"build container, {os.cpu_count()} CPUs")
    ap.add_argument("--serial-shading", action="store_true",
                    help="run the reference's shading loop serially (round 3's calibration); by default it runs "
                         "in parallel as wavefront.cc:105-217 does (omp parallel for schedule(dynamic), thread-local "
                         "child queues merged in thread order)")
    args = ap.parse_args()
    import gen_golden
    import oracle_ctypes as orc
    import rtx

    out = {"threads": args.threads, "host": args.host, "cases": {},
           "reference_parallel": ("IntersectBatch (cpu_ray_integrator.h:24) only" if args.serial_shading else
                                  "IntersectBatch (cpu_ray_integrator.h:24) and the shading loop (wavefront.cc:105-217, "
                                  "schedule(dynamic), thread-local child queues)"),
           "reference_serial": "primary generation (wavefront.cc:62-79), batch copies and queue merges, as in the "
                               "reference"}
    with tempfile.TemporaryDirectory() as td:
        for name, scene, preset, width, spp, depth in CASES:
            if args.only and name not in args.only.split(","):
                continue
            path = os.path.join(td, scene + ".rtxs")
            rtx.HostScene.recipe(scene, 1234).write(path)
            cfg = orc.camera_preset(preset)
            env = dict(os.environ, REF_THREADS=str(args.threads), REF_PAR_SHADE="0" if args.serial_shading else "1")
            prefix = os.path.join(td, name)
            subprocess.run([str(a) for a in [HARNESS, "render", path, MODELS, *gen_golden.cam_args(cfg, width), depth, spp, 0, 1234,
                            prefix]], check=True, env=env, cwd=MODELS)  # (image textures by file name)
            st = dict(l.split() for l in open(prefix + ".stats"))
            ref_rays, ref_s = int(st["rays"]), float(st["loop_seconds"])
            assert int(st.get("parallel_shading", "0")) == (0 if args.serial_shading else 1)
            s = orc.Scene(path)
            t0 = time.perf_counter()
            _, _, pst = s.render(cfg, width, spp, depth, 1234, adaptive=0, rng="philox", mode="per_pixel",
                                 threads=args.threads)
            port_s = time.perf_counter() - t0
            ref_rate, port_rate = ref_rays / ref_s / 1e6, pst["rays"] / port_s / 1e6
            out["cases"][name] = {
                "config": f"{scene} {width}w, {spp} spp, depth {depth}, fixed spp",
                "reference": {"mrays_s": ref_rate, "segments": ref_rays, "loop_seconds": ref_s,
                              "render_seconds_incl_p3": float(st["render_seconds"])},
                "port": {"mrays_s": port_rate, "segments": pst["rays"], "seconds": port_s},
                "ratio_port_over_reference": port_rate / ref_rate,
            }
            print(name, json.dumps(out["cases"][name]), flush=True)
    dst = args.out
    prev = json.load(open(dst)) if os.path.exists(dst) and args.only else {}
    if prev:
        prev["cases"].update(out["cases"])
        out = prev
    json.dump(out, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
