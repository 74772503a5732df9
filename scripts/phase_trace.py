#!/usr/bin/env python3
"""One adaptive frame's kernel sequence from a rocprofv3 kernel trace (run_kernel_trace.csv):
durations and gaps of the phase launches, records, scans and slot-map expands.
  python3 scripts/phase_trace.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv [frame index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
fi = int(sys.argv[2]) if len(sys.argv) > 2 else -3
seq = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows), key=lambda x: x[1])
starts = [i for i, x in enumerate(seq) if x[0].startswith("rtxd::k_frame_init")]
i0, i1 = starts[fi], starts[fi + 1]
t0 = seq[i0][1]
tot = {}
for n, s, e in seq[i0:i1 + 1]:
    short = n.split("(")[0].replace("void ", "").replace("rtxd::", "")[:40]
    print(f"{short:42s} {(e - s) / 1e3:9.1f} us  start {(s - t0) / 1e3:9.1f}  end {(e - t0) / 1e3:9.1f}")
    tot[short.split("<")[0]] = tot.get(short.split("<")[0], 0) + (e - s) / 1e3
print("frame", (seq[i1][1] - t0) / 1e3, "us;", {k: round(v, 1) for k, v in tot.items()})
