#!/usr/bin/env python3
"""bench.py — Mrays/s of the MI355X path-tracing hot path (BASELINE.json metric).

A "step" is one complete frame: every sample of every pixel of the workload rendered through
the C ABI (rtx_render_multi: persistent kernel, accumulate, resolve, then the framebuffer
copied to the host), with the scene already resident in HBM.  The timed region therefore
runs from the first ray generation to the framebuffer on the host.

Workloads (BASELINE.json configs): the default is the north-star scene, the Stanford bunny:
  * 1 GPU:  C3, bunny 1000x562, 200 spp, depth 20, fixed spp
  * N GPUs: C4, bunny 3840x2160, 1024 spp, depth 50, the SAME frame split over the N ranks
    (strong scaling): the image's rows are interleaved 4-row stripes, stripe k -> rank k mod N
    (SURVEY §8e); every rank copies its stripes into one shared host framebuffer
    (/dev/shm); no collective touches the data path (a gloo process group carries only the
    timing barrier and the max-over-ranks reduction).
Other workloads: --workload c2_final | c5_mixed | c1_three | c4_bunny4k | c3_bunny.

Prints ONE JSON line (rank 0).  `roofline` prices the dominant kernel (k_persistent) against
its binding resource, VALU issue: useful lane-operations per second (VALU wave-instructions
x active lanes, per segment, from the committed rocprofv3 PMC profile of the same build and
workload) over the MI355X vector peak.  `cpu_baseline` times the reference itself
(oracle/_ref/ref_harness: its own sources, its OpenMP loops) on the same frame at reduced spp
on this host's available cores, with the CPU restatement (oracle/librtx_oracle.so, `port`)
timed beside it on a bounded band, and `rms_vs_cpu` compares that band with the GPU's render
of it by the same kernel build and schedule the timed frames used.
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
    "c1_three": ("three", "c1_three", 400, 4, 4),
    "c2_final": ("final", "c2_final", 1200, 100, 50),
    "c3_bunny": ("bunny", "c3_bunny", 1000, 200, 20),
    "c4_bunny4k": ("bunny", "c4_bunny4k", 3840, 1024, 50),
    "c5_mixed": ("mixed", "c5_mixed", 3840, 2048, 50),
}
# The VALU issue ceiling, MEASURED on gfx950 (scripts/microbench/valu_ceiling.hip, profiles/r05/
# valu_ceiling_*.jsonl): with two or more waves per SIMD, a wave64 VALU instruction holds the
# SIMD for one quad-cycle (4.1-4.3 cycles measured), except that two waves' all-VGPR
# v_fma/add/mul_f32, v_add_u32, v_and_b32 and v_mov_b32 issue as a PAIR in one quad-cycle (2.3
# cycles each: the guide's "2 cycles on SIMD-32", MI355X_MICROARCH.md:54); f64 add/mul/fma,
# v_max/cmp/cndmask/cvt/bfe/med3/add_co/mul_u32_u24/mul_lo, packed f32 and 32-bit ops with an
# SGPR operand never pair; transcendentals take 2 (f32) / 4 (f64) quad-cycles; one wave alone
# gets ~4.6-5 cycles per instruction.  A mixed stream pairs almost nothing (3 f32 : 1 f64 FMAs:
# 3.98 cycles per instruction).  PMC: SQ_ACTIVE_INST_VALU counts an instruction's quad-cycles,
# SQ_ACTIVE_INST_VALU2 the quad-cycles in which a pair issued, so the SIMD's VALU issue
# quad-cycles are their difference (checked against the measured cycles of every class within
# ~5 %: the microbenchmark's per-class counters, pmc_r7a_valu_ceiling.csv).
N_SIMD, CLOCK_HZ = 1024, 2.4e9
HBM_PEAK_GBS = 8000.0
L2_SHARED_GBS = 18800.0  # rows shared by every workgroup, served by the XCD's L2 (MI355X_MICROARCH.md)
STRIPE_ROWS = 4  # interleaved 4-row stripes: max/mean rank load 1.002 at N = 8 for C4 (8 rows: 1.011)
ADAPTIVE_MIN_SPP, ADAPTIVE_REL = 16, float(np.float32(0.05))  # wavefront.cc:42-43 (kRelThresh is a float)


def available_cpus():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


class SharedFrame:
    """The whole-frame host framebuffer: pinned memory (1 rank) or a /dev/shm file every rank
    maps (N ranks), registered as pinned when the runtime allows it."""

    def __init__(self, torch, npix, rank, world, dist, tag):
        self.torch, self.path, self.registered = torch, None, False
        nbytes = npix * 3 * 8
        if world == 1:
            self.t = torch.empty((npix, 3), dtype=torch.float64).pin_memory()
            self.arr = self.t.numpy()
            self.pinned = True
            return
        self.path = f"/dev/shm/rtx_bench_frame_{tag}"
        if rank == 0:
            with open(self.path, "wb") as f:
                f.truncate(nbytes)
        dist.barrier()
        self.arr = np.memmap(self.path, dtype=np.float64, mode="r+", shape=(npix, 3))
        self.pinned = False
        try:  # plumbing only: lets the library DMA straight into the shared frame
            rc = torch.cuda.cudart().cudaHostRegister(self.arr.ctypes.data, nbytes, 0)
            self.registered = self.pinned = int(getattr(rc, "value", rc)) == 0
        except Exception:  # noqa: BLE001  (pageable: the library stages through pinned memory)
            self.pinned = False

    def close(self, rank, dist):
        if self.registered:
            try:
                self.torch.cuda.cudart().cudaHostUnregister(self.arr.ctypes.data)
            except Exception:  # noqa: BLE001
                pass
        if self.path:
            del self.arr
            if dist is not None:
                dist.barrier()
            if rank == 0 and os.path.exists(self.path):
                os.unlink(self.path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed frames (0: ~4 s of frames, at least 3)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="auto", choices=["auto"] + sorted(WORKLOADS),
                    help="auto: c3_bunny on 1 GPU, c4_bunny4k split over N GPUs")
    ap.add_argument("--spp", type=int, default=0, help="override samples per pixel")
    ap.add_argument("--mode", default="persistent", choices=["wavefront", "persistent"])
    ap.add_argument("--precision", default="fast", choices=["parity", "fast"])
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--schedule", default="auto", choices=["auto", "plain", "park", "park_step"],
                    help="persistent fast schedule: auto = timed per scene by the library (default); "
                         "plain/park force one (identical results; used by scripts/profile.sh so the "
                         "trace holds no schedule-timing launches)")
    ap.add_argument("--generic", action="store_true", help="time the generic (unspecialised) kernel build")
    ap.add_argument("--adaptive", action="store_true",
                    help="the reference's default sampling (wavefront.cc:42-43, 62-69, 125-127): per-pixel "
                         "adaptive, at least 16 samples, relative error 0.05f, up to the workload's spp")
    ap.add_argument("--adapt-schedule", default="phases", choices=["phases"],
                    help="adaptive renders: one launch per phase (the library's schedule)")
    ap.add_argument("--adapt-tune", default="",
                    help="tuning of the adaptive phases (rtx.adapt_tune), e.g. phase_slots=4194304,phase_mstep=0.5 "
                         "(never changes results, only the work)")
    ap.add_argument("--min-spp", type=int, default=ADAPTIVE_MIN_SPP,
                    help="adaptive renders: samples of the first pass (the reference's 16; = spp runs the phase "
                         "kernel over exactly the fixed-spp frame's samples, an overhead experiment)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-adaptive-leg", action="store_true",
                    help="skip the adaptive-sampling frames timed beside a fixed-spp line")
    ap.add_argument("--no-generic-leg", action="store_true", help="skip the generic-build comparison frames")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--dist-backend", default="gloo",
                    help="process group of the N>1 timing barrier and max/sum reductions: gloo (default; no "
                         "collective touches the data path, so the host-side group the 1-GPU rehearsals run is "
                         "the one an 8-GPU run takes) or nccl (= RCCL)")
    args = ap.parse_args()
    if args.adaptive and args.mode != "persistent":
        # the metric counts the segments of the recorded samples, which the counting build
        # reports for the persistent kernel's adaptive schedules only (rtx_stats.rays_recorded)
        ap.error("--adaptive needs --mode persistent")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # torch (plumbing: pinned host memory, barrier, max-over-ranks) must initialise its HIP
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

    if args.adapt_tune:
        kv = dict(x.split("=") for x in args.adapt_tune.split(","))
        rtx.adapt_tune(**{k: (float(v) if k in ("phase_mstep", "margin1", "pool_w") else int(v)) for k, v in kv.items()})
    workload = args.workload if args.workload != "auto" else ("c3_bunny" if world == 1 else "c4_bunny4k")
    scene_name, preset, width, spp, depth = WORKLOADS[workload]
    spp = args.spp or spp
    host = rtx.HostScene.recipe(scene_name, 1234)
    dev = rtx.DeviceScene(host, device=dev_id)
    cam = rtx.camera(rtx.camera_config(preset, width=width))
    W, H = cam.image_width, cam.image_height
    sched_flags = (rtx.SCHEDULE_FLAGS[args.schedule] | (rtx.RTX_FLAG_GENERIC if args.generic else 0)
                   | rtx.ADAPT_SCHEDULE_FLAGS[args.adapt_schedule])

    def params(flags=sched_flags, generic=False, adaptive=None):
        p = rtx.RenderParams()
        p.spp, p.max_depth, p.seed = spp, depth, args.seed
        p.adaptive = int(args.adaptive if adaptive is None else adaptive)
        p.min_spp, p.rel_threshold = args.min_spp, ADAPTIVE_REL
        p.mode, p.precision = rtx.MODES[args.mode], rtx.PRECISIONS[args.precision]
        p.stripe_rows, p.stripe_index, p.stripe_count = STRIPE_ROWS, rank, world
        p.flags = flags | (rtx.RTX_FLAG_GENERIC if generic else 0)
        return p

    frame = SharedFrame(torch, W * H, rank, world, dist, os.environ.get("MASTER_PORT", "0"))
    if rank == 0:
        frame.arr[:] = np.nan  # every row must be written by some rank (checked after the run)
    scenes_arr = (rtx.C.c_void_p * 1)(dev.h.value)
    out_ptr = frame.arr.ctypes.data

    def step(p):
        st = rtx.Stats()
        rtx._check(rtx.lib().rtx_render_multi(scenes_arr, 1, rtx.C.byref(cam), rtx.C.byref(p), out_ptr, None,
                                              rtx.C.byref(st), None), "rtx_render_multi")
        return st.as_dict()

    if args.schedule == "auto" and args.mode == "persistent" and args.precision == "fast":
        # the library times its two persistent schedules on the first fast render of a scene
        # (a centre tile at this spp); trigger that here with a one-pixel render, so it never
        # lands in the timed region, whatever --warmup is
        q = rtx.RenderParams()
        q.spp, q.max_depth, q.adaptive, q.seed, q.mode, q.precision = spp, depth, 0, args.seed, 1, 1
        q.x0, q.y0, q.w, q.h = 0, 0, 1, 1
        tmp = torch.empty((1, 3), dtype=torch.float64, device=f"cuda:{dev_id}")
        dev.render_device(cam, q, tmp.data_ptr())

    p = params()
    t_warm = time.perf_counter()
    for _ in range(max(1, args.warmup)):
        step(p)
    per_frame = (time.perf_counter() - t_warm) / max(1, args.warmup)
    steps = args.steps or max(3, int(4.0 / max(per_frame, 1e-4)))
    if dist is not None:  # every rank times the same number of frames
        t = torch.tensor([steps], dtype=torch.int64, device="cpu" if args.dist_backend == "gloo" else f"cuda:{dev_id}")
        dist.broadcast(t, 0)
        steps = int(t.item())

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    stats = [step(p) for _ in range(steps)]
    barrier()
    elapsed = time.perf_counter() - t0
    rays = sum(s["rays_total"] for s in stats)
    hot_ms = sum(s["hot_kernel_ms"] for s in stats)
    hot_launches = sum(s["hot_launches"] for s in stats)
    build_bits, parked = stats[-1]["build"], stats[-1]["parked"]
    if dist is not None:
        red_dev = "cpu" if args.dist_backend == "gloo" else f"cuda:{dev_id}"
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.float64, device=red_dev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays_all = float(r.item())
        barrier()
    else:
        rays_all = float(rays)
    covered = bool(not np.isnan(frame.arr).any()) if rank == 0 else None

    # counting pass (diagnostic kernel build): segments, node visits and SIMD efficiency
    cst = step(params(rtx.RTX_FLAG_COUNT | sched_flags))
    segs = max(1, cst["rays_total"])
    # adaptive sampling traces some samples past a pixel's convergence and discards them: the
    # metric counts the segments of the recorded samples only (the counting pass renders the same
    # frame and counts them per slot; deterministic, so the timed frames recorded as many)
    recorded = cst["rays_recorded"] * steps
    if dist is not None:
        r = torch.tensor([float(recorded)], dtype=torch.float64, device=red_dev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        recorded = float(r.item())
    nodes_per_seg = cst["node_visits"] / segs
    simd_nodes = cst["node_visits"] / (64.0 * cst["wave_node_iters"]) if cst["wave_node_iters"] else None
    simd_prims = cst["prim_tests"] / (64.0 * cst["wave_prim_iters"]) if cst["wave_prim_iters"] else None
    prims_per_seg = cst["prim_tests"] / segs
    boxes_per_visit = 1 if args.precision == "parity" else cst["node_bytes"] // 32
    tris_per_seg, sphs_per_seg = cst["tri_tests"] / segs, cst["sphere_tests"] / segs
    rects_per_seg = max(0.0, prims_per_seg - tris_per_seg - sphs_per_seg)
    # SURVEY.md §8(d) byte model: B_seg = 32*n_box + 48*n_tri + 16*n_sph + 32*n_rect + 96.  The
    # scene is L2/MALL-resident, so these are bytes touched in cache, not HBM traffic.
    bytes_per_seg = (32 * boxes_per_visit * nodes_per_seg + 48 * tris_per_seg + 16 * sphs_per_seg
                     + 32 * rects_per_seg + 96)
    segs_per_launch = rays / max(1, hot_launches)
    avg_launch_s = hot_ms / 1e3 / max(1, hot_launches)

    roofline = valu_roofline(workload, args, segs_per_launch, avg_launch_s)
    roofline.update({
        "kernel": "k_persistent" if args.mode == "persistent" else "k_wf_extend",
        "avg_launch_ms": avg_launch_s * 1e3, "segments_per_launch": segs_per_launch,
        "bytes_touched": {"per_segment": bytes_per_seg, "GB_s": bytes_per_seg * segs_per_launch / avg_launch_s / 1e9,
                          "l2_frac": bytes_per_seg * segs_per_launch / avg_launch_s / 1e9 / L2_SHARED_GBS,
                          "note": "SURVEY 8(d) algorithmic bytes (nodes/primitives/path state) per segment; "
                                  "served from L2/MALL (the scene is cache-resident), not an HBM figure; l2_frac "
                                  "against the L2's shared-row rate, 16.8-18.8 TB/s chip-wide "
                                  "(MI355X_MICROARCH.md, indexed rows gathered from the XCD's L2; the top)"},
        "nodes_per_segment": nodes_per_seg, "prims_per_segment": prims_per_seg, "boxes_per_visit": boxes_per_visit,
        "simd_efficiency_nodes": simd_nodes, "simd_efficiency_prims": simd_prims,
        "wave_rounds_idle_frac": cst["wave_rounds_idle"] / cst["wave_rounds"] if cst["wave_rounds"] else None,
        "lane_occupancy": (cst["wave_lanes_live"] / (64.0 * (cst["wave_rounds"] - cst["wave_rounds_idle"]))
                           if cst["wave_rounds"] > cst["wave_rounds_idle"] else None),
    })

    generic_leg = None
    if world == 1 and not args.generic and not args.no_generic_leg and args.mode == "persistent":
        gp = params(generic=True)
        step(gp)
        g_steps = max(3, min(steps, int(1.5 / max(per_frame, 1e-4))))
        torch.cuda.synchronize()
        tg = time.perf_counter()
        gst = [step(gp) for _ in range(g_steps)]
        torch.cuda.synchronize()
        tg = time.perf_counter() - tg
        g_rays = cst["rays_recorded"] * g_steps if args.adaptive else sum(s["rays_total"] for s in gst)
        generic_leg = {"value": g_rays / tg / 1e6, "ms_per_step": tg * 1e3 / g_steps,
                       "steps": g_steps, "build": rtx.build_names(gst[-1]["build"]),
                       "note": "same frame with RTX_FLAG_GENERIC: no per-scene specialisation (same pixels)"}

    # the reference's default sampling (adaptive, WavefrontRenderer::Render) on the same frame,
    # timed beside the fixed-spp line so the driver's run measures it too
    adaptive_leg = None
    if world == 1 and not args.adaptive and not args.no_adaptive_leg and args.mode == "persistent":
        adaptive_leg = time_adaptive(torch, step, params, per_frame, rays_all / elapsed / 1e6)

    out = None
    if rank == 0:
        out = {
            "metric": "Mrays/s (primary+secondary) at fixed spp; RMS pixel error vs CPU ref",
            "sampling": sampling_text(args.adaptive),
            "value": (recorded if args.adaptive else rays_all) / elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{workload}: {scene_name} scene {W}x{H}, {spp} spp, depth {depth}, "
                                   + sampling_text(args.adaptive)
                                   + (f", one frame split over {world} GPUs" if world > 1 else ""),
                       "scene_prims": int(host.desc().n_prims), "bvh_nodes": int(host.desc().n_nodes),
                       "mode": args.mode, "precision": args.precision,
                       "schedule": ("park_step" if args.schedule == "park_step" else "park") if parked else "plain",
                       "kernel_build": rtx.build_names(build_bits),
                       "timed_region": "first ray generation -> framebuffer on the host (D2H inside each step)",
                       "framebuffer": "pinned host" if frame.pinned else "pageable host (pinned staging)",
                       "frame_rows_covered": covered,
                       "parallelism": f"tile-split x{world} (interleaved {STRIPE_ROWS}-row stripes, no collectives)"},
            "roofline": roofline,
            "rays_per_step": rays_all / steps,
        }
        if args.adaptive:
            out["value_note"] = ("adaptive: value counts the segments of the recorded samples "
                                 "(rays_recorded, counting pass); traced_value adds the samples traced past "
                                 "a pixel's convergence and discarded")
            out["traced_value"] = rays_all / elapsed / 1e6
            out["rays_recorded_per_step"] = recorded / steps
        if generic_leg:
            out["generic_build"] = generic_leg
        if adaptive_leg:
            out["adaptive"] = adaptive_leg
        if not args.no_cpu_baseline and world == 1:
            port, out["rms_vs_cpu"], out["rms_check"] = cpu_baseline(
                rtx, dev, host, cam, preset, scene_name, spp, depth, args, parked, build_bits)
            # the reference itself (its own sources, oracle/_ref/ref_harness) timed here, on the
            # same host cores: cpu_baseline; the port beside it (the RMS check's CPU side)
            ref = cpu_reference(host, preset, W, spp, depth, args)
            if ref is not None and "error" not in ref:
                ref["port"] = port
                ref["gpu_over_reference"] = out["value"] / ref["value"]
                ref["gpu_over_reference_spread"] = [out["value"] / ref["spread"][1], out["value"] / ref["spread"][0]]
                out["cpu_baseline"] = ref
            else:
                out["cpu_baseline"] = port
                if ref is not None:
                    out["cpu_reference_error"] = ref["error"]
            rc = out["rms_check"]
            if args.adaptive and rc["rows"] == [0, H]:  # the CPU rendered the whole frame
                rc["segments_gpu_recorded"] = int(cst["rays_recorded"])
                rc["recorded_segments_identical"] = int(cst["rays_recorded"]) == rc["segments_cpu"]
            if adaptive_leg:
                adaptive_leg.update(cpu_check_adaptive(rtx, dev, host, cam, preset, spp, depth, args,
                                                       adaptive_leg.pop("_recorded_whole")))
    frame.close(rank, dist)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def time_adaptive(torch, step, params, per_frame_fixed, fixed_value):
    """The same frame with the reference's default sampling (adaptive: at least 16 samples,
    relative error 0.05f, up to the workload's spp; wavefront.cc:42-43, 62-69, 125-127), ~2.5 s
    of frames.  value counts the segments of the samples the pixels record (the counting pass's
    rays_recorded: the same frame, deterministic); traced_value adds the samples traced past a
    pixel's convergence and discarded."""
    ap = params(adaptive=True)
    t = time.perf_counter()
    step(ap)  # first adaptive frame: workspace allocation
    step(ap)
    per = (time.perf_counter() - t) / 2
    n = max(3, min(200, int(2.5 / max(per, 1e-4))))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sts = [step(ap) for _ in range(n)]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    cst = step(params(ap.flags | 1, adaptive=True))  # RTX_FLAG_COUNT
    rec, traced = cst["rays_recorded"], sum(s["rays_total"] for s in sts) / n
    idle = cst["wave_rounds_idle"] / cst["wave_rounds"] if cst["wave_rounds"] else None
    hot_ms = sum(s["hot_kernel_ms"] for s in sts) / n
    return {"metric": "Mrays/s of the recorded samples' segments, adaptive sampling (the reference's default)",
            "value": rec * n / el / 1e6, "traced_value": traced * n / el / 1e6, "unit": "Mrays/s",
            "ms_per_step": el * 1e3 / n, "steps": n, "hot_kernel_ms_per_step": hot_ms,
            "hot_launches_per_step": sts[-1]["hot_launches"],
            "rays_recorded_per_step": rec, "rays_traced_per_step": traced,
            "recorded_fraction_of_traced": rec / max(1.0, traced), "vs_fixed_spp_value": rec * n / el / 1e6 / fixed_value,
            "schedule": "phases", "wave_rounds_idle_frac": idle,
            "sampling": sampling_text(True), "_recorded_whole": rec}


def cpu_check_adaptive(rtx, dev, host, cam, preset, spp, depth, args, recorded_whole):
    """The adaptive frame on the CPU oracle (whole frame when it takes under ~25 s on this host,
    else a centred band) against the GPU's render of the same pixels: sample counts, recorded
    segments (counting build) and RMS."""
    import tempfile

    import oracle_ctypes as orc

    threads = args.cpu_threads or available_cpus()
    W, H = cam.image_width, cam.image_height
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "scene.rtxs")
        host.write(path)
        s = orc.Scene(path)
        cfg = orc.camera_preset(preset)
        kw = dict(adaptive=1, rng="philox", mode="per_pixel", threads=threads)
        t0 = time.perf_counter()
        s.render(cfg, W, spp, depth, args.seed, tile=(0, H // 2 - 2, W, 4), **kw)
        per_row = (time.perf_counter() - t0) / 4
        ch = int(max(4, min(H, 25.0 / max(per_row, 1e-6))))
        tile = (0, max(0, H // 2 - ch // 2), W, ch)
        t0 = time.perf_counter()
        ref, ref_spp, st = s.render(cfg, W, spp, depth, args.seed, tile=tile, **kw)
        dt = time.perf_counter() - t0
    gpu, gpu_spp, gst = dev.render(cam, spp, depth, seed=args.seed, adaptive=True, tile=tile, mode="persistent",
                                   precision=args.precision, count=True, min_spp=ADAPTIVE_MIN_SPP,
                                   rel_threshold=ADAPTIVE_REL)
    whole = ch == H
    same_spp = bool(np.array_equal(gpu_spp, ref_spp.ravel()))
    return {"rms_vs_cpu": float(np.sqrt(np.mean((gpu - ref.reshape(-1, 3)) ** 2))),
            "rms_check": {"rows": [tile[1], tile[1] + tile[3]],
                          "sample_counts_identical": same_spp,
                          "pixels_sample_count_differs": int(np.sum(gpu_spp != ref_spp.ravel())),
                          **({} if same_spp or args.precision != "fast" else {"note": FAST_TIES_NOTE}),
                          "segments_cpu": int(st["rays"]), "segments_gpu_recorded": int(gst["rays_recorded"]),
                          "recorded_segments_identical": int(gst["rays_recorded"]) == int(st["rays"]),
                          "whole_frame_recorded_identical": (int(recorded_whole) == int(st["rays"])) if whole else None,
                          "mean_spp": float(np.mean(ref_spp)), "pixels_converged_early": float(np.mean(ref_spp < spp))},
            "cpu_baseline": {"value": st["rays"] / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
                             "sample": f"{'the whole' if whole else f'centre band {W}x{ch} of the same'} {W}x{H} frame, "
                                       f"adaptive, {st['rays']} segments in {dt:.1f}s (oracle/rtx_oracle.cc, philox)"}}


def sampling_text(adaptive):
    return (f"adaptive (min {ADAPTIVE_MIN_SPP} spp, rel. error 0.05f, max = spp)" if adaptive else "fixed spp")


def valu_roofline(workload, args, segs_per_launch, avg_launch_s):
    """VALU-issue roofline of the hot kernel from the committed PMC profile of this build and
    workload (profiles/valu_<workload>_*.json, scripts/profile.sh) and the launch time measured
    live (HIP events on the library's stream).

    achieved = useful lane-ops per second: SQ_INSTS_VALU x 64 x lane utilisation per segment
    (lane utilisation = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)) x segments per launch
    / launch time.  peak = the same instructions at the MEASURED best issue rate of their mix:
    every instruction that may pair (all but the f64, 64-bit integer, conversion and
    transcendental classes the PMC counts separately; an upper bound on what pairs, so the peak
    is optimistic and frac conservative) at half a quad-cycle, the f64 / int64 / cvt ones at one,
    transcendentals at 2 (f32) / 4 (f64), on 1024 SIMDs at 2.4 GHz.  frac = achieved / peak.
    valu_issue_frac = the measured share of SIMD cycles issuing VALU work, 4 x (SQ_ACTIVE_INST_VALU
    - SQ_ACTIVE_INST_VALU2) / SIMD cycles (idle lanes included)."""
    pf = os.path.join(ROOT, "profiles", f"valu_{workload}_{args.mode}_{args.precision}"
                      + ("_adaptive" if args.adaptive else "") + ".json")
    base = {"bound": "valu", "unit": "Tlane-op/s (VALU)"}
    if not os.path.exists(pf):
        return {**base, "achieved": None, "peak": None, "frac": None, "traffic": None, "note": f"no PMC profile {pf}"}
    prof = json.load(open(pf))
    ops_per_seg = prof["lane_ops_per_segment"]
    insts_per_seg = prof["valu_insts_per_segment"]
    achieved = ops_per_seg * segs_per_launch / avg_launch_s
    traffic = prof.get("hbm_bytes_per_segment")
    out = {**base, "achieved": achieved / 1e12, "peak": None, "frac": None,
           "traffic": traffic * segs_per_launch if traffic is not None else None,
           "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, scaled to this launch)",
           "hbm_GB_s": traffic * segs_per_launch / avg_launch_s / 1e9 if traffic is not None else None,
           "hbm_frac": (traffic * segs_per_launch / avg_launch_s / 1e9 / HBM_PEAK_GBS) if traffic is not None else None,
           "lane_utilisation": prof["lane_utilisation"], "lane_ops_per_segment": ops_per_seg,
           "valu_insts_per_segment": insts_per_seg, "source": prof["source"]}
    n = prof.get("valu_insts_per_launch")
    per = lambda k: prof.get(k + "_per_launch")  # noqa: E731
    need = ["sq_active_inst_valu2", "sq_insts_valu_int64", "sq_insts_valu_cvt", "sq_insts_valu_trans_f32"]
    if not n or any(per(k) is None for k in need):
        out["note"] = "profile predates the dual-issue counters (SQ_ACTIVE_INST_VALU2): re-profile for peak / frac"
        return out
    f64 = per("sq_insts_valu_add_f64") + per("sq_insts_valu_mul_f64") + per("sq_insts_valu_fma_f64")
    single = f64 + per("sq_insts_valu_int64") + per("sq_insts_valu_cvt")
    trans32, trans64 = per("sq_insts_valu_trans_f32"), per("sq_insts_valu_trans_f64")
    pairable = max(0.0, n - single - trans32 - trans64)
    qmin = 0.5 * pairable + single + 2.0 * trans32 + 4.0 * trans64  # quad-cycles per launch at the best rate
    peak = 64.0 * n / (4.0 * qmin / (N_SIMD * CLOCK_HZ))
    quads = prof["active_inst_valu_per_launch"] - per("sq_active_inst_valu2")
    segs_prof = prof["segments_per_launch"]
    issue = 4.0 * quads / segs_prof * segs_per_launch / avg_launch_s / (N_SIMD * CLOCK_HZ)
    # the class-priced peak: each class at its measured cost, the pairable share of the int32 / f32 /
    # unnamed classes from the kernel's ISA (scripts/isa_classes.py, its hot loops; unmeasured VOP2
    # ops counted as pairable), never below the instructions the PMC saw issue in pairs
    cls = class_priced(workload, args, prof, n, f64, trans32, trans64)
    out.update({"peak": peak / 1e12, "frac": achieved / peak, "valu_issue_frac": issue,
                "pairable_share_max": pairable / n, "paired_share": 2.0 * per("sq_active_inst_valu2") / n,
                "min_issue_ms": 4.0 * qmin / segs_prof * segs_per_launch / (N_SIMD * CLOCK_HZ) * 1e3,
                "note": "peak: the profile's instruction mix at the measured gfx950 issue costs (pairs of 32-bit "
                        "VOP2/VOP3 ops per quad-cycle, f64 / int64 / cvt one quad-cycle, transcendentals 2 / 4; "
                        "scripts/microbench/valu_ceiling.hip) on 1024 SIMDs x 2.4 GHz; valu_issue_frac: "
                        "4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SIMD cycles"})
    if cls is not None:
        qx = cls["qmin"]
        peak_x = 64.0 * n / (4.0 * qx / (N_SIMD * CLOCK_HZ))
        out.update({"peak_class_priced": peak_x / 1e12, "frac_class_priced": achieved / peak_x,
                    "min_issue_ms_class_priced": 4.0 * qx / segs_prof * segs_per_launch / (N_SIMD * CLOCK_HZ) * 1e3,
                    "pairable_share_class_priced": cls["pairable"] / n, "class_split": cls["source"],
                    "note_class_priced": "peak_class_priced prices every class at its measured gfx950 cost: only "
                                         "all-VGPR v_fma/add/mul_f32, v_add_u32, v_and_b32, v_mov_b32 pair (and, "
                                         "unmeasured, other all-VGPR VOP2 ops); cmp, cndmask, max, med3, bfe, "
                                         "lshl_add, add_co, lane moves, SGPR or literal operands, f64, int64, cvt "
                                         "one quad-cycle; the pairable share of each PMC class from the ISA of the "
                                         "kernel's loops, at least the PMC's paired instructions"})
    return out


def class_priced(workload, args, prof, n, f64, trans32, trans64):
    """Best issue time (quad-cycles per launch) of the profile's instruction mix with every class
    at its measured cost (profiles/r05/valu_ceiling_summary.json), the pairable share of the PMC's
    int32, f32 and unnamed classes taken from the kernel's ISA (profiles/r06/isa_classes_*.json,
    scripts/isa_classes.py) and floored at the instructions the PMC counted issuing as pairs."""
    f = os.path.join(ROOT, "profiles", "r06", f"isa_classes_{workload}" + ("_adaptive" if args.adaptive else "") + ".json")
    if not os.path.exists(f):
        return None
    isa = json.load(open(f))["loop"]
    per = lambda k: prof.get(k + "_per_launch") or 0.0  # noqa: E731
    dyn = {"f32": per("sq_insts_valu_add_f32") + per("sq_insts_valu_mul_f32") + per("sq_insts_valu_fma_f32"),
           "int32": per("sq_insts_valu_int32")}
    named = f64 + per("sq_insts_valu_int64") + per("sq_insts_valu_cvt") + trans32 + trans64 + dyn["f32"] + dyn["int32"]
    dyn["other"] = max(0.0, n - named)
    p_isa = sum(dyn[c] * isa.get(c, {}).get("pair_share_if_vop2_pairs", 0.0) for c in dyn)
    p = min(max(p_isa, 2.0 * per("sq_active_inst_valu2")), n - f64 - trans32 - trans64)
    return {"qmin": 0.5 * p + (n - p - trans32 - trans64) + 2.0 * trans32 + 4.0 * trans64, "pairable": p,
            "pairable_isa": p_isa, "source": os.path.relpath(f, ROOT)}


FAST_TIES_NOTE = ("fast precision: the f32-culled walk visits primitives in another order than the reference's, so "
                  "an exact t tie between two distinct primitives (the bunny's shared triangle edges) can resolve "
                  "to the other one; a pixel whose path meets one can take a different number of adaptive samples "
                  "(DESIGN.md §1, profiles/r05/diag_c4_adaptive_mismatch_r8m.txt); parity precision reproduces "
                  "the oracle's counts")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
ASSETS = os.path.join(ROOT, "3360-ray-tracer_amd", "assets")


def cpu_reference(host, preset, width, spp, depth, args):
    """The reference's own renderer timed on this host: oracle/_ref/ref_harness (the reference's
    CPURayIntegrator, BVH, materials and PixelState compiled from its sources by oracle/Makefile,
    driven by the Render() glue of wavefront.cc:40-242) with its OpenMP IntersectBatch
    (cpu_ray_integrator.h:24) and its parallel shading loop (wavefront.cc:105-217,
    REF_PAR_SHADE=1) on the threads the port gets, pinned one per core (OMP_PROC_BIND=close,
    OMP_PLACES=cores), at fixed spp on the whole frame.  A 1-spp probe sizes each timed render to
    about 4 s; three renders, the median reported with the spread.  None when the harness was
    not built (it needs /root/reference at build time; the built binary travels with the tree);
    an error dict when it fails (the bench line must survive a harness crash or time-out)."""
    import subprocess
    import tempfile

    if not os.path.exists(HARNESS):
        return None
    import oracle_ctypes as orc

    threads = args.cpu_threads or available_cpus()
    c = {"aspectRatio": 16 / 9.0, "vfov": 90.0, "defocusAngle": 0.0, "focusDist": 10.0}
    c.update(orc.camera_preset(preset))
    cam = [repr(float(c["aspectRatio"])), str(int(width)), repr(float(c["vfov"])),
           *[repr(float(x)) for x in c["lookfrom"]], *[repr(float(x)) for x in c["lookat"]],
           *[repr(float(x)) for x in c["vup"]], repr(float(c["defocusAngle"])), repr(float(c["focusDist"]))]
    env = dict(os.environ, REF_THREADS=str(threads), REF_PAR_SHADE="1", OMP_PROC_BIND="close", OMP_PLACES="cores")
    try:
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "scene.rtxs")
            host.write(path)

            def run(n, i):
                prefix = os.path.join(td, f"ref{n}_{i}")
                subprocess.run([HARNESS, "render", path, ASSETS, *cam, str(depth), str(n), "0", str(args.seed + i),
                                prefix], check=True, env=env, cwd=ASSETS, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL, timeout=300)
                return dict(line.split() for line in open(prefix + ".stats"))

            probe = run(1, 0)
            n = int(max(1, min(spp, 4.0 / max(float(probe["loop_seconds"]), 1e-3))))
            # (4K frames: the 1-spp probe alone is ~10-20 s; it is then one of the three)
            if n > 1:
                sts = [run(n, i) for i in range(3)]
            else:  # (a probe over ~8 s stands alone: the bench must finish in minutes)
                sts = [probe] + ([run(1, i) for i in (1, 2)] if float(probe["loop_seconds"]) < 8.0 else [])
    except (subprocess.CalledProcessError, subprocess.TimeoutExpired, OSError, ValueError, KeyError) as e:
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    rates = sorted(int(st["rays"]) / float(st["loop_seconds"]) / 1e6 for st in sts)
    rays, sec = sum(int(st["rays"]) for st in sts), sum(float(st["loop_seconds"]) for st in sts)
    mid = sts[len(sts) // 2]
    return {"value": rates[len(rates) // 2], "unit": "Mrays/s", "cores": threads, "nproc": os.cpu_count(), "kind": "reference",
            "runs": rates, "spread": [rates[0], rates[-1]],
            "sample": f"the whole {width}-wide frame at {n} spp (of {spp}), depth {depth}, fixed spp; {len(sts)} renders "
                      f"(seeds {args.seed}..), median reported; {rays} segments in {sec:.1f}s of the "
                      f"reference's pass loop (oracle/_ref/ref_harness: its own sources, OpenMP IntersectBatch + "
                      f"parallel shading loop on {threads} threads pinned one per core, std::mt19937 per thread)",
            "render_seconds_incl_p3": float(mid["render_seconds"]), "threads_reported": int(mid["threads"]),
            "pinning": "OMP_PROC_BIND=close OMP_PLACES=cores"}


def cpu_baseline(rtx, dev, host, cam, preset, scene_name, spp, depth, args, parked, build_bits):
    """Time the CPU oracle on a centred band of the same frame; compare its pixels with the
    GPU's render of the band by the timed kernel build and schedule."""
    import tempfile

    import oracle_ctypes as orc

    threads = args.cpu_threads or available_cpus()
    W, H = cam.image_width, cam.image_height
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "scene.rtxs")
        host.write(path)
        s = orc.Scene(path)
        cfg = orc.camera_preset(preset)
        # probe on a small centre band (twice: the first call also starts the thread pool),
        # then size the timed sample to ~15 s of wall time, capped at the whole frame
        probe = (0, H // 2 - 2, W, 4)
        ad = dict(adaptive=int(args.adaptive), rng="philox", mode="per_pixel", threads=threads)
        for _ in range(2):
            t0 = time.perf_counter()
            s.render(cfg, W, spp, depth, args.seed, tile=probe, **ad)
            per_row = (time.perf_counter() - t0) / 4
        ch = int(max(4, min(H, 15.0 / max(per_row, 1e-6))))
        tile = (0, max(0, H // 2 - ch // 2), W, ch)
        t0 = time.perf_counter()
        ref, ref_spp, st = s.render(cfg, W, spp, depth, args.seed, tile=tile, **ad)
        dt = time.perf_counter() - t0
    sched = ("park_step" if args.schedule == "park_step" else "park") if parked else "plain"
    gpu, gpu_spp, gst = dev.render(cam, spp, depth, seed=args.seed, adaptive=args.adaptive, tile=tile, mode=args.mode,
                                   precision=args.precision, schedule=sched if args.mode == "persistent" else None,
                                   generic=args.generic, min_spp=ADAPTIVE_MIN_SPP, rel_threshold=ADAPTIVE_REL)
    rms = float(np.sqrt(np.mean((gpu - ref.reshape(-1, 3)) ** 2)))
    what = "the whole" if ch == H else f"centre band {W}x{ch} of the same"
    base = {"value": st["rays"] / dt / 1e6, "unit": "Mrays/s", "cores": threads, "nproc": os.cpu_count(),
            "kind": "port",
            "sample": f"{what} {W}x{H} frame, {spp} spp, depth {depth}, fixed spp, "
                      f"{st['rays']} segments in {dt:.1f}s (oracle/rtx_oracle.cc, OpenMP on {threads} threads, philox)"
                      .replace("fixed spp", sampling_text(args.adaptive))}
    same_spp = bool(np.array_equal(gpu_spp, ref_spp.ravel()))
    check = {"mode": args.mode, "precision": args.precision, "schedule": sched,
             "kernel_build": rtx.build_names(gst["build"]), "same_build_as_timed": gst["build"] == build_bits,
             "rows": [tile[1], tile[1] + tile[3]],
             "sample_counts_identical": same_spp,
             "pixels_sample_count_differs": int(np.sum(gpu_spp != ref_spp.ravel())),
             **({} if same_spp or args.precision != "fast" else {"note": FAST_TIES_NOTE}),
             "segments_gpu": int(gst["rays_total"]), "segments_cpu": int(st["rays"])}
    if args.adaptive:
        check["pixels_converged_early"] = float(np.mean(ref_spp < spp))
        check["mean_spp"] = float(np.mean(ref_spp))
        # whole sample groups are traced; samples past a pixel's convergence are discarded
        check["recorded_fraction_of_traced_segments"] = st["rays"] / max(1, gst["rays_total"])
    return base, rms, check


if __name__ == "__main__":
    main()
