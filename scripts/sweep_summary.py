#!/usr/bin/env python3
"""One line per bench JSON file: tag, value, traced_value, ms/step, idle wave-round fraction, lane
occupancy of tracing rounds (scripts/runs/r5*.sh sweeps).  usage: sweep_summary.py tag file.json"""
import json
import sys

tag, path = sys.argv[1], sys.argv[2]
d = json.loads(open(path).read().strip().splitlines()[-1])
r = d["roofline"]
print(tag, round(d["value"], 1), round(d.get("traced_value", 0.0), 1), round(d["ms_per_step"], 3),
      r.get("wave_rounds_idle_frac"), r.get("lane_occupancy"), flush=True)
