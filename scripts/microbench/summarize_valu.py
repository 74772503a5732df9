#!/usr/bin/env python3
"""Summarise a valu_ceiling run and its PMC pass into one JSON (profiles/r05/valu_ceiling_summary.json).

usage: summarize_valu.py <classes.jsonl (timed run)> <pmc.jsonl (the run under rocprofv3)> <counter_collection.csv> <out.json>

Per (class, waves per SIMD): the measured cycles per wave64 instruction (s_memtime stamps, the
timed run) and, from the PMC pass's median launch of that configuration, SQ_ACTIVE_INST_VALU /
SQ_INSTS_VALU, the paired share (SQ_ACTIVE_INST_VALU2 / SQ_ACTIVE_INST_VALU) and the cycles per
instruction the counter model gives: 4 x (ACTIVE - ACTIVE2) / INSTS.
"""
import collections
import csv
import json
import sys


def main():
    timed = [json.loads(x) for x in open(sys.argv[1])]
    pmc_cfg = [json.loads(x) for x in open(sys.argv[2])]
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(sys.argv[3])):
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(k for k in d if k > 60)  # (60 clock-warming launches first)
    counters = {}
    for i, c in enumerate(pmc_cfg):
        grp = ids[5 * i:5 * i + 5]
        v = d[grp[len(grp) // 2]]
        a, a2, n = v["SQ_ACTIVE_INST_VALU"], v["SQ_ACTIVE_INST_VALU2"], v["SQ_INSTS_VALU"]
        counters[(c["class"], c["waves_per_simd"])] = {
            "active_per_inst": a / n, "paired_share_of_active": a2 / a, "counter_cyc_per_inst": 4 * (a - a2) / n,
            "cyc_per_inst_under_pmc": c["cyc_per_inst"]}
    out = {"source": "scripts/microbench/valu_ceiling.hip (256 CUs x 1 workgroup of 256 x W threads, 8 independent "
                     "chains per wave, s_memtime / s_memrealtime stamps; medians over 5 launches)",
           "classes": []}
    for t in timed:
        e = {"class": t["class"], "waves_per_simd": t["waves_per_simd"], "cyc_per_inst": round(t["cyc_per_inst"], 3),
             "clock_ghz": round(t["clock_ghz"], 3)}
        e.update({k: round(v, 3) for k, v in counters.get((t["class"], t["waves_per_simd"]), {}).items()})
        out["classes"].append(e)
    json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
