#!/usr/bin/env python3
"""bench.py — Mrays/s of the MI355X path-tracing hot path (BASELINE.json metric).

A "step" is one complete frame of the workload (every sample of every pixel of this rank's
shard) rendered through the C ABI (rtx_render_device into device-resident buffers, scene
already in HBM).  Default workload = BASELINE configs[1]: C2 final_scene, 1200x675,
100 spp, depth 50, fixed spp (adaptive sampling off).

N GPUs (one process per GPU, launched by torch.distributed.run): the image's rows are
split into interleaved 8-row stripes (stripe k -> rank k mod N) and the sample
count is N x spp, so every rank traces the same amount of work as the 1-GPU run ("weak"
scaling); no collective touches the data path (RCCL only carries the timing barrier and
the max-over-ranks reduction).

Prints ONE JSON line (rank 0).  `roofline` uses the dominant kernel's average launch time
(HIP events on the library's stream, over the timed region) and the algorithmic bytes per
launch from a separate counting pass (DESIGN.md "Roofline accounting").  `cpu_baseline`
times the CPU oracle (oracle/librtx_oracle.so, the restatement pinned to the reference) on
a bounded crop of the same workload on this host's cores, and `rms_vs_cpu` compares the
GPU and CPU pixels of that crop at the same seed.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

WORKLOADS = {  # name -> (scene recipe, camera preset, width, spp, depth)
    "c2_final": ("final", "c2_final", 1200, 100, 50),
    "c3_bunny": ("bunny", "c3_bunny", 1000, 200, 20),
    "c1_three": ("three", "c1_three", 400, 4, 4),
    "c4_bunny4k": ("bunny", "c4_bunny4k", 3840, 1024, 50),
    "c5_mixed": ("mixed", "c5_mixed", 3840, 2048, 50),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
STRIPE_ROWS = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c2_final", choices=sorted(WORKLOADS))
    ap.add_argument("--spp", type=int, default=0, help="override samples per pixel (per GPU)")
    ap.add_argument("--mode", default="persistent", choices=["wavefront", "persistent"])
    ap.add_argument("--precision", default="fast", choices=["parity", "fast"])
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--schedule", default="auto", choices=["auto", "plain", "park"],
                    help="persistent fast schedule: auto = timed per scene by the library (default); "
                         "plain/park force one (identical results; used by scripts/profile.sh so the "
                         "trace holds no schedule-timing launches)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (=RCCL, one GPU per rank) or gloo (rehearsal)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # torch (plumbing: device buffers, barrier, max-over-ranks) must initialise its HIP
    # runtime before librtx.so is loaded into the process
    import torch

    dist = None
    torch.cuda.init()
    # one process per GPU; a gloo rehearsal may place several ranks on fewer devices
    dev_id = local % max(1, torch.cuda.device_count()) if world > 1 else 0
    torch.cuda.set_device(dev_id)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(args.dist_backend)

    import rtx

    scene_name, preset, width, spp, depth = WORKLOADS[args.workload]
    spp = args.spp or spp
    total_spp = spp * world  # weak scaling: N x samples over 1/N of the pixels
    host = rtx.HostScene.recipe(scene_name, 1234)
    dev = rtx.DeviceScene(host, device=dev_id)
    cam = rtx.camera(rtx.camera_config(preset, width=width))
    p = rtx.RenderParams()
    p.spp, p.max_depth, p.adaptive, p.seed = total_spp, depth, 0, args.seed
    p.mode, p.precision = rtx.MODES[args.mode], rtx.PRECISIONS[args.precision]
    if world > 1:
        p.stripe_rows, p.stripe_index, p.stripe_count = STRIPE_ROWS, rank, world
    sched_flags = {"auto": 0, "park": 2, "plain": 4}[args.schedule]  # RTX_FLAG_PARK / RTX_FLAG_NO_PARK
    p.flags = sched_flags
    npix = rtx.lib().rtx_render_pixel_count(cam, p)

    d_rgb = torch.empty((npix, 3), dtype=torch.float64, device=f"cuda:{dev_id}")
    d_spp = torch.empty((npix,), dtype=torch.int32, device=f"cuda:{dev_id}")

    def step():
        return dev.render_device(cam, p, d_rgb.data_ptr(), d_spp.data_ptr())

    if args.schedule == "auto" and args.mode == "persistent" and args.precision == "fast":
        # the library times its two persistent schedules on the first fast render of a scene
        # (a centre tile at this spp); trigger that here with a one-pixel render, so it never
        # lands in the timed region, whatever --warmup is
        q = rtx.RenderParams()
        q.spp, q.max_depth, q.adaptive, q.seed, q.mode, q.precision = p.spp, p.max_depth, 0, p.seed, p.mode, p.precision
        q.x0, q.y0, q.w, q.h = 0, 0, 1, 1
        dev.render_device(cam, q, d_rgb.data_ptr(), d_spp.data_ptr())

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    stats = [step() for _ in range(args.steps)]
    barrier()
    elapsed = time.perf_counter() - t0
    rays = sum(s["rays_total"] for s in stats)
    hot_ms = sum(s["hot_kernel_ms"] for s in stats)
    hot_launches = sum(s["hot_launches"] for s in stats)
    if dist is not None:
        red_dev = "cpu" if args.dist_backend == "gloo" else f"cuda:{dev_id}"
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.float64, device=red_dev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays_all = float(r.item())
    else:
        rays_all = float(rays)

    # counting pass (diagnostic kernel build) for algorithmic bytes per segment
    p.flags = 1 | sched_flags
    cst = step()
    p.flags = sched_flags
    segs = max(1, cst["rays_total"])
    nodes_per_seg = cst["node_visits"] / segs
    # SIMD efficiency of the traversal loops (fast BVH4 only): lane work / (64 x wave iterations)
    simd_nodes = cst["node_visits"] / (64.0 * cst["wave_node_iters"]) if cst["wave_node_iters"] else None
    simd_prims = cst["prim_tests"] / (64.0 * cst["wave_prim_iters"]) if cst["wave_prim_iters"] else None
    prims_per_seg = cst["prim_tests"] / segs
    # B_seg = 32*n_box + 48*n_tri + 16*n_sph + 32*n_rect + 96 (path state in + out).
    # One box = one 32-B node of the compact model; a visit of the 128-B F4Node tests four boxes,
    # of the 64-B BVH2 FNode two, of the reference-layout f64 node (parity) one.
    boxes_per_visit = 1 if args.precision == "parity" else cst["node_bytes"] // 32
    tris_per_seg = cst["tri_tests"] / segs
    sphs_per_seg = cst["sphere_tests"] / segs
    rects_per_seg = max(0.0, prims_per_seg - tris_per_seg - sphs_per_seg)
    bytes_per_seg = (32 * boxes_per_visit * nodes_per_seg + 48 * tris_per_seg + 16 * sphs_per_seg
                     + 32 * rects_per_seg + 96)
    segs_per_launch = rays / max(1, hot_launches)
    avg_launch_s = hot_ms / 1e3 / max(1, hot_launches)
    achieved_gbs = bytes_per_seg * segs_per_launch / avg_launch_s / 1e9
    traffic = valu = None
    tf = os.path.join(ROOT, "profiles", f"traffic_{args.workload}_{args.mode}_{args.precision}.json")
    if os.path.exists(tf):
        prof = json.load(open(tf))
        traffic = prof.get("hbm_bytes_per_launch")
        if prof.get("valu_busy") is not None:
            # The kernel's actual limiter is VALU issue (the scene is L2/MALL-resident): the
            # fraction of SIMD cycles that issue a VALU instruction, from the committed PMC
            # profile of this build (SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)).
            valu = {"busy_frac": prof["valu_busy"], "insts_per_launch": prof.get("valu_insts_per_launch"),
                    "source": prof.get("source"),
                    "note": "fraction of SIMD cycles issuing VALU (PMC, profiled run of this build)"}

    out = None
    if rank == 0:
        out = {
            "metric": "Mrays/s (primary+secondary) at fixed spp; RMS pixel error vs CPU ref",
            "value": rays_all / elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{args.workload}: {scene_name} scene {width}x{cam.image_height}, "
                                   f"{spp} spp/GPU-share, depth {depth}, fixed spp",
                       "scene_prims": int(host.desc().n_prims), "bvh_nodes": int(host.desc().n_nodes),
                       "mode": args.mode, "precision": args.precision, "spp_total": total_spp,
                       "pixels_per_rank": int(npix), "stripe_rows": STRIPE_ROWS if world > 1 else None,
                       "schedule": "park" if stats[-1].get("parked") else "plain",
                       "parallelism": f"tile-split x{world} (interleaved row stripes, no collectives)"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_persistent" if args.mode == "persistent" else "k_wf_bounce",
                         "avg_launch_ms": avg_launch_s * 1e3, "segments_per_launch": segs_per_launch,
                         "bytes_per_segment": bytes_per_seg, "nodes_per_segment": nodes_per_seg,
                         "prims_per_segment": prims_per_seg, "tris_per_segment": tris_per_seg,
                         "spheres_per_segment": sphs_per_seg, "boxes_per_visit": boxes_per_visit,
                         "simd_efficiency_nodes": simd_nodes, "simd_efficiency_prims": simd_prims,
                         "valu": valu,
                         "note": "algorithmic bytes per SURVEY 8(d); the scene is L2/MALL-resident, so "
                                 "HBM traffic (PMC) << algorithmic bytes and frac may exceed 1"},
            "rays_per_step": rays_all / args.steps,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"], out["rms_vs_cpu"] = cpu_baseline(rtx, dev, host, cam, preset, spp, depth, args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(rtx, dev, host, cam, preset, spp, depth, args):
    """Time the CPU oracle on a centred crop of the same workload; compare its pixels."""
    import tempfile

    import oracle_ctypes as orc

    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    W, H = cam.image_width, cam.image_height
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "scene.rtxs")
        host.write(path)
        s = orc.Scene(path)
        cfg = orc.camera_preset(preset)
        # probe on a small centre crop (twice: the first call also starts the thread pool),
        # then size the timed sample to ~10 s of wall time on `threads` cores, capped at the
        # whole frame: full-width bands of rows around the image centre
        probe = (0, H // 2 - 4, W, 8)
        for _ in range(2):
            t0 = time.perf_counter()
            s.render(cfg, W, spp, depth, args.seed, adaptive=0, rng="philox", mode="per_pixel", tile=probe,
                     threads=threads)
            per_row = (time.perf_counter() - t0) / 8
        ch = int(max(8, min(H, 10.0 / max(per_row, 1e-6))))
        cw = W
        tile = (0, max(0, H // 2 - ch // 2), cw, ch)
        t0 = time.perf_counter()
        ref, _, st = s.render(cfg, W, spp, depth, args.seed, adaptive=0, rng="philox", mode="per_pixel", tile=tile,
                              threads=threads)
        dt = time.perf_counter() - t0
    gpu, _, _ = dev.render(cam, spp, depth, seed=args.seed, adaptive=False, tile=tile, mode="wavefront",
                           precision="parity")
    rms = float(np.sqrt(np.mean((gpu - ref.reshape(-1, 3)) ** 2)))
    what = "the whole" if ch == H else f"centre band {cw}x{ch} of the same"
    base = {"value": st["rays"] / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{what} {W}x{H} frame, {spp} spp, depth {depth}, fixed spp, "
                      f"{st['rays']} segments in {dt:.1f}s (oracle/rtx_oracle.cc, OpenMP, philox)"}
    return base, rms


if __name__ == "__main__":
    main()
