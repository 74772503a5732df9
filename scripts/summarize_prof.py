#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory into profiles/:

  <round>_<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  <round>_<tag>_pmc.json           per-kernel PMC counters (sum over the profiled launches)
  traffic_<workload>_<mode>_<precision>.json   HBM bytes per launch of the dominant kernel:
        FETCH_SIZE x 2 (gfx950 reports half of a wide coalesced read, MI355X_MICROARCH.md
        §HBM) + WRITE_SIZE, both in KiB units -> bytes, divided by the launch count.

usage: summarize_prof.py gpurun_out/prof_<tag> <round> <workload> <mode> <precision> [adaptive]

With `adaptive` (a bench --adaptive profile: phase launches of several instantiations), the
VALU and HBM figures are the sums over every non-counting k_persistent launch divided by the
segments of the profiled frames (warmup + steps frames of the PMC pass, identical frames), and
the files are named ..._adaptive.json.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d, rnd, workload, mode, prec = sys.argv[1:6]
    adaptive = len(sys.argv) > 6 and sys.argv[6] == "adaptive"
    tag = os.path.basename(d.rstrip("/")).replace("prof_", "")
    prof = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))[0]
    shutil.copyfile(stats, os.path.join(prof, f"kernel_stats_{tag}.csv"))
    bench = os.path.join(d, "bench_trace.json")
    if os.path.exists(bench):
        shutil.copyfile(bench, os.path.join(prof, f"bench_under_rocprof_{tag}.json"))
    counters = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            counters[k][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[(k, r["Counter_Name"])].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    out = {}
    for k, v in counters.items():
        n = max(len(launches[(k, c)]) for c in v)
        out[k] = {"launches": n, **v}
    json.dump(out, open(os.path.join(prof, f"pmc_{tag}.json"), "w"), indent=1, sort_keys=True)
    if adaptive:
        adaptive_profile(d, out, launches, rnd, tag, workload, mode, prec)
        return
    # non-counting instantiation of the hot kernel (k_persistent<STACK, FAST, COUNT, SCATTER, PARK>:
    # either schedule; the one with the most wave cycles is the frame kernel)
    hot = "k_persistent<32, true, false, false," if mode == "persistent" else "k_wf_extend<32, true, false>"
    if prec == "parity":
        hot = hot.replace("true, false", "false, false", 1)
    cands = [k for k, v in out.items() if hot in k and "FETCH_SIZE" in v and "WRITE_SIZE" in v]
    cands.sort(key=lambda k: -out[k].get("SQ_WAVE_CYCLES", out[k]["FETCH_SIZE"]))
    for k, v in [(k, out[k]) for k in cands[:1]]:
        if True:
            n_f = len(launches[(k, "FETCH_SIZE")])
            n_w = len(launches[(k, "WRITE_SIZE")])
            per = v["FETCH_SIZE"] * 2 * 1024 / n_f + v["WRITE_SIZE"] * 1024 / n_w
            valu = busy = None
            if "SQ_INSTS_VALU" in v:
                valu = v["SQ_INSTS_VALU"] / max(1, len(launches[(k, "SQ_INSTS_VALU")]))
            if "SQ_ACTIVE_INST_VALU" in v and "GRBM_GUI_ACTIVE" in v:
                # fraction of SIMD cycles issuing VALU: SQ_ACTIVE_INST_VALU counts quad-cycles per
                # wave (summed over waves; one wave issues VALU per SIMD per cycle), GRBM_GUI_ACTIVE
                # is summed over the 8 XCDs (MI355X_MICROARCH.md, cycle constants)
                act = v["SQ_ACTIVE_INST_VALU"] / max(1, len(launches[(k, "SQ_ACTIVE_INST_VALU")]))
                cyc = v["GRBM_GUI_ACTIVE"] / max(1, len(launches[(k, "GRBM_GUI_ACTIVE")])) / 8
                busy = 4 * act / (1024 * cyc)
            t = {"kernel": k, "hbm_bytes_per_launch": per, "valu_insts_per_launch": valu, "valu_busy": busy,
                 "fetch_kib_total": v["FETCH_SIZE"],
                 "write_kib_total": v["WRITE_SIZE"], "launches_fetch_pass": n_f, "launches_write_pass": n_w,
                 "source": f"profiles/{rnd}/pmc_{tag}.json", "correction": "FETCH_SIZE x2 (gfx950)"}
            json.dump(t, open(os.path.join(ROOT, "profiles", f"traffic_{workload}_{mode}_{prec}.json"), "w"),
                      indent=1)
            print(json.dumps(t))
            valu_profile(d, k, v, launches, per, rnd, tag, workload, mode, prec)


def per_launch(v, launches, k, c):
    return v[c] / max(1, len(launches[(k, c)]))


def valu_profile(d, k, v, launches, hbm_per_launch, rnd, tag, workload, mode, prec):
    """profiles/valu_<workload>_<mode>_<precision>.json: what bench.py's VALU roofline reads.
    Segments per launch come from the bench line of the PMC pass (the frames are identical)."""
    need = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU")
    if not all(c in v for c in need):
        return
    b = glob.glob(os.path.join(d, "bench_pmc_SQ_INSTS_VALU*.json"))
    segs = json.loads(open(b[0]).read().strip().splitlines()[-1])["roofline"]["segments_per_launch"]
    insts = per_launch(v, launches, k, "SQ_INSTS_VALU")
    active = per_launch(v, launches, k, "SQ_ACTIVE_INST_VALU")
    threads = per_launch(v, launches, k, "SQ_THREAD_CYCLES_VALU")
    # SQ_THREAD_CYCLES_VALU counts SQ_ACTIVE_INST_VALU's cycles x active lanes (same unit):
    # the ratio over 64 is the mean fraction of a wave's lanes that VALU instructions use
    util = threads / (64.0 * active)
    out = {"kernel": k, "segments_per_launch": segs, "valu_insts_per_launch": insts,
           "active_inst_valu_per_launch": active, "thread_cycles_valu_per_launch": threads,
           "lane_utilisation": util, "valu_insts_per_segment": insts / segs,
           "lane_ops_per_segment": insts * 64 * util / segs,
           "hbm_bytes_per_segment": hbm_per_launch / segs,
           "source": f"profiles/{rnd}/pmc_{tag}.json",
           "formula": "lane_ops_per_segment = SQ_INSTS_VALU x 64 x SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)"
                      " / segments; hbm = (FETCH_SIZE x 2 + WRITE_SIZE) x 1 KiB / segments"}
    for c in ("GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_ANY", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
              "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
              "SQ_ACTIVE_INST_VALU2", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
              "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
              "SQ_WAVES"):
        if c in v:
            out[c.lower() + "_per_launch"] = per_launch(v, launches, k, c)
    json.dump(out, open(os.path.join(ROOT, "profiles", f"valu_{workload}_{mode}_{prec}.json"), "w"), indent=1)
    print(json.dumps(out))


def adaptive_profile(d, out, launches, rnd, tag, workload, mode, prec):
    """Sums over the frame kernels (non-counting k_persistent launches, every phase) per segment;
    the counters also per launch (averaged over the phase launches of the profiled frames, every
    PMC pass running the same frames), so bench.py prices the adaptive mix as it does a fixed one."""
    ks = [k for k in out if k.startswith("void rtxd::k_persistent<") and ", true, false, false," in k]

    def total(c):
        return sum(out[k].get(c, 0.0) for k in ks)

    def frames_segments(pass_glob):
        b = glob.glob(os.path.join(d, pass_glob))
        j = json.loads(open(b[0]).read().strip().splitlines()[-1])
        return (j["warmup"] + j["steps"]) * j["rays_per_step"]

    segs_valu = frames_segments("bench_pmc_SQ_INSTS_VALU*.json")
    util = total("SQ_THREAD_CYCLES_VALU") / (64.0 * total("SQ_ACTIVE_INST_VALU"))
    insts = total("SQ_INSTS_VALU")
    hbm = None
    if all(glob.glob(os.path.join(d, f"bench_pmc_{c}*.json")) for c in ("FETCH_SIZE", "WRITE_SIZE")):
        hbm = (total("FETCH_SIZE") * 2 * 1024 / frames_segments("bench_pmc_FETCH_SIZE*.json")
               + total("WRITE_SIZE") * 1024 / frames_segments("bench_pmc_WRITE_SIZE*.json"))
    res = {"kernels": ks, "segments_profiled": segs_valu, "lane_utilisation": util,
           "valu_insts_per_segment": insts / segs_valu, "lane_ops_per_segment": insts * 64 * util / segs_valu,
           "hbm_bytes_per_segment": hbm, "source": f"profiles/{rnd}/pmc_{tag}.json",
           "formula": "sums over every phase launch of the frame kernels / segments of the profiled frames"}

    def nl(c):
        return max(1, sum(len(launches[(k, c)]) for k in ks))

    n_valu = nl("SQ_INSTS_VALU")
    res.update({"segments_per_launch": segs_valu / n_valu, "valu_insts_per_launch": insts / n_valu,
                "active_inst_valu_per_launch": total("SQ_ACTIVE_INST_VALU") / nl("SQ_ACTIVE_INST_VALU")})
    for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
              "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64", "SQ_ACTIVE_INST_VALU2", "SQ_INSTS_VALU_TRANS_F32",
              "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_FMA_F32"):
        if any(c in out[k] for k in ks):
            res[c.lower() + "_per_launch"] = total(c) / nl(c)
    json.dump(res, open(os.path.join(ROOT, "profiles", f"valu_{workload}_{mode}_{prec}_adaptive.json"), "w"),
              indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
