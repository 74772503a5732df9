#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory into profiles/:

  <round>_<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  <round>_<tag>_pmc.json           per-kernel PMC counters (sum over the profiled launches)
  traffic_<workload>_<mode>_<precision>.json   HBM bytes per launch of the dominant kernel:
        FETCH_SIZE x 2 (gfx950 reports half of a wide coalesced read, MI355X_MICROARCH.md
        §HBM) + WRITE_SIZE, both in KiB units -> bytes, divided by the launch count.

usage: summarize_prof.py gpurun_out/prof_<tag> <round> <workload> <mode> <precision>
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


if __name__ == "__main__":
    main()
