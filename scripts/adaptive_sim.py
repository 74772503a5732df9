#!/usr/bin/env python3
"""Adaptive phase schedule simulator (CPU only, no GPU): replays render_adaptive's policy
(csrc/rtx_capi.hip render_adaptive; k_adapt_record / adapt_next_batch / k_adapt_floor in
csrc/rtx_frame_kernels.h) over every sample of every pixel, rendered once at the full budget by
the CPU restatement (oracle/rtx_oracle.cc orc_render_samples, philox: the GPU's own samples).

The pixels' results do not depend on the policy (samples past a pixel's convergence are
discarded), only the work does: per phase, the slots, traced segments and pixels.  With a
cost model (segments / rate + a drain per launch + per-phase fixed costs) this ranks policy
variants before they are measured on the GPU.

  python3 scripts/adaptive_sim.py [--workload c3_bunny|c2_final] [--cache /tmp/adaptive_sim_c3.npz]
(profiles/r05/adaptive_sim_policies.txt: the policy grids this round's defaults came from)
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))

WORKLOADS = {"c3_bunny": ("bunny", "c3_bunny", 1000, 200, 20), "c2_final": ("final", "c2_final", 1200, 100, 50)}
MIN_SPP, REL = 16, 0.05


def samples(workload, cache, threads, seed=1234):
    if cache and os.path.exists(cache):
        z = np.load(cache)
        return z["L"], z["segs"]
    import oracle_ctypes as orc
    import rtx

    scene, preset, width, spp, depth = WORKLOADS[workload]
    path = f"/tmp/adaptive_sim_{scene}.rtxs"
    rtx.HostScene.recipe(scene, 1234).write(path)
    t = time.time()
    L, segs = orc.Scene(path).render_samples(orc.camera_preset(preset), width, spp, depth, seed, threads=threads)
    print(f"rendered {L.shape} in {time.time() - t:.1f}s", file=sys.stderr)
    L, segs = L.reshape(-1, spp, 3), segs.reshape(-1, spp)
    if cache:
        np.savez(cache, L=L, segs=segs)
    return L, segs


def prepare(L, segs):
    """Policy-independent per-pixel facts: the running statistics after n samples are the same
    whatever the batches (the record replays the same samples in order), so: the sample count at
    which IsConverged first holds (n >= MIN_SPP, exact form; budget + 1 when never), the
    prediction input need(n) = max_c var / (rel mu)^2 after n samples, and the segment prefix sums."""
    npix, spp = segs.shape
    cs = np.zeros((npix, spp + 1), np.int64)
    np.cumsum(segs, axis=1, dtype=np.int64, out=cs[:, 1:])
    need = np.zeros((npix, spp + 1), np.float32)
    nconv = np.full(npix, spp + 1, np.int64)
    mu = np.zeros((npix, 3))
    m2 = np.zeros((npix, 3))
    for j in range(spp):
        n = j + 1
        x = L[:, j]
        delta = x - mu
        mnew = mu + delta / n
        m2 += (x - mnew) * delta
        mu = mnew
        var = m2 / (n - 1) if n > 1 else np.zeros_like(m2)
        m = np.maximum(np.abs(mu), 1e-3)
        need[:, n] = np.max(var / (REL * REL * m * m), axis=1)
        if n >= MIN_SPP:
            ok = np.all(np.sqrt(var) / np.sqrt(float(n)) / m <= REL, axis=1)
            nconv = np.where((nconv > spp) & ok, n, nconv)
    return cs, need, nconv


def simulate(pre, budget, phase_slots=1 << 23, mstep=0.25, kmin_first=True, floor=True, min_batch=(4, 4),
             first=MIN_SPP, kcap=None, margins=None, floor_from=2, pool=0, width=None, pool_w=1.0,
             finish_slots=None, pool_r=1, capture=None):
    """Replays the phase policy; returns per-phase dicts (pixels, slots, traced and recorded
    segments) and the final sample counts."""
    cs, need_n, nconv = pre
    npix = cs.shape[0]
    kcap = kcap or budget
    n = np.zeros(npix, np.int64)
    k = np.full(npix, min(first, budget), np.int64)  # this phase's batch per pixel
    phases = []
    g = 1
    while True:
        act = np.nonzero(k > 0)[0]
        if act.size == 0:
            break
        kk, n0 = k[act], n[act]
        if capture is not None:  # the phase's pixels, first sample and batch (scripts: drain studies)
            capture.append((act.copy(), n0.copy(), kk.copy()))
        traced = int((cs[act, n0 + kk] - cs[act, n0]).sum())
        nc = nconv[act]
        nn = np.where(nc <= n0 + kk, nc, n0 + kk)
        cv = nc <= n0 + kk
        recorded = int((cs[act, nn] - cs[act, n0]).sum())
        n[act] = nn
        phases.append({"phase": g, "pixels": int(act.size), "slots": int(kk.sum()), "traced": traced,
                       "recorded": recorded})
        kmin = min(budget, -(-phase_slots // act.size)) if kmin_first else 0
        want_pix = act[~cv & (nn < budget)]
        k[:] = 0
        if want_pix.size == 0:
            break
        nw = n[want_pix]
        need = need_n[want_pix, nw].astype(np.float64)
        if pool:  # the prediction pooled over the pixel's 3x3 neighbourhood (each at its own n)
            cur = need_n[np.arange(npix), np.maximum(n, 1)].astype(np.float64).reshape(-1, width)
            cur[(n == 0).reshape(-1, width)] = np.nan
            R = pool_r
            pad = np.pad(cur, R, constant_values=np.nan)
            h, w_ = cur.shape
            stack = np.stack([pad[dy:dy + h, dx:dx + w_] for dy in range(2 * R + 1) for dx in range(2 * R + 1)])
            if pool == 2:
                pooled = np.nanmedian(stack, axis=0)
            else:
                wts = np.ones(stack.shape[0]); wts[stack.shape[0] // 2] = pool_w
                ok = ~np.isnan(stack)
                pooled = np.nansum(stack * wts[:, None, None], axis=0) / np.sum(ok * wts[:, None, None], axis=0)
            need = pooled.reshape(-1)[want_pix]
        left = budget - nw
        margin = (1.0 + mstep * (g - 1)) if margins is None else margins[min(g - 1, len(margins) - 1)]
        want = (need - nw) * margin
        kb = np.where(want < left, np.ceil(want), left).astype(np.int64)
        lo = np.minimum(np.maximum(min_batch[0] << min(g - 1, min_batch[1]), kmin), left)
        kb = np.maximum(kb, lo)
        kb = (kb + 3) & ~3
        kb = np.minimum(kb, np.minimum(left, kcap))
        if finish_slots is not None and int(np.minimum(left, kcap).sum() - kb.sum()) < finish_slots:
            kb = np.minimum(left, kcap)  # finishing every pixel now costs less than another phase
        elif floor and g + 1 >= floor_from and (floor != "if_small" or int(kb.sum()) < phase_slots):  # k_adapt_floor
            na = int((kb != 0).sum())
            km = -(-phase_slots // max(na, 1))
            kb = np.where(kb != 0, np.minimum((np.maximum(kb, np.minimum(km, left)) + 3) & ~3, np.minimum(left, kcap)), 0)
        k[want_pix] = kb
        g += 1
    return phases, n


def cost(phases, rate=8e9, drain=0.65e-3, per_phase=0.1e-3, first=2.2e-3):
    """Frame time model fitted to measured C3 frames (kernel traces under profiles/r05): phases
    after the first at a marginal segment rate plus a fixed launch cost (the launch's last paths
    walking alone: phase 4's 1.6 M segments take 0.81 ms), every phase with its record / expand /
    host round trip; the first phase (cheaper segments: sky pixels) as measured."""
    t = first + per_phase + sum(p["traced"] / rate + drain + per_phase for p in phases[1:])
    rec = sum(p["recorded"] for p in phases)
    return t, rec / t / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3_bunny")
    ap.add_argument("--cache", default="/tmp/adaptive_sim_c3.npz")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    args = ap.parse_args()
    L, segs = samples(args.workload, args.cache, args.threads)
    budget = WORKLOADS[args.workload][3]
    pre = prepare(L, segs)
    width = WORKLOADS[args.workload][2]
    variants = {  # margins: the batch margin after phase 1, 2, 3+ (the kernel: margin1, then 1 + 0.25 (g - 1))
        "round 4 (floor 2^23, own prediction)": dict(phase_slots=1 << 23, margins=[1.0, 1.25, 1.5]),
        "floor 2^20, own prediction": dict(phase_slots=1 << 20, margins=[1.0, 1.25, 1.5]),
        "default (floor 2^21, margin 0.8, pooled x8)": dict(phase_slots=1 << 21, margins=[0.8, 1.25, 1.5], pool=1,
                                                             pool_w=8.0, width=width),
        "default + finish below 2^22 slots": dict(phase_slots=1 << 21, margins=[0.8, 1.25, 1.5], pool=1, pool_w=8.0,
                                                   width=width, finish_slots=1 << 22),
    }
    for name, kw in variants.items():
        phases, n = simulate(pre, budget, **kw)
        t, v = cost(phases, drain=0.65e-3, rate=8e9)
        tr = sum(p["traced"] for p in phases)
        rc = sum(p["recorded"] for p in phases)
        desc = "; ".join(f"p{p['phase']} {p['pixels']} px {p['slots'] / 1e6:.2f}M slots {p['traced'] / 1e6:.1f}M tr "
                         f"{p['recorded'] / 1e6:.1f}M rec" for p in phases)
        print(f"{name:14s} model {t * 1e3:6.2f} ms {v:7.1f} rec Mrays/s | traced {tr / 1e6:.1f}M recorded {rc / 1e6:.1f}M "
              f"({rc / tr:.3f}) | {desc}")


if __name__ == "__main__":
    main()
