#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: calibrates the statistical parity leg (tests/test_statistical_parity.py).

For each case (C2 final / C3 bunny, fixed / adaptive; tests/stat_parity.py CASES) it renders the
test's fixed ensemble (K_ENSEMBLE restatement renders at ENSEMBLE_SEEDS) and NULL_RENDERS more
restatement renders at independent seeds, and compares each of the latter with the ensemble
exactly as the test compares the reference's render: the test's conditional null distribution.
Written to tests/golden/stat_null.json:
  * the ensemble's digest (the test refuses a calibration of another ensemble);
  * the chi2/dof null: mean, variance, empirical quantiles, and the central 1 - ALPHA interval of
    the scaled chi-square with that mean and variance (the test's bounds);
  * for the t-statistics, the null's exceedance rates at the two-sided 5 % and 1 % t_{K-1}
    levels (pooled tile values, image channels, mean spp), which check the t shape the bounds
    assume, and the number of null renders any check of the verdict rejects (expected 0).
  * the power check: each deliberate estimator change (oracle/rtx_oracle.cc g_perturb) against
    the ensemble, with the checks it fails.

usage: python oracle/gen_stat_null.py [threads]      (~5 min on 8 threads)
"""
import json
import os
import sys
import tempfile

import numpy as np
from scipy import stats as sps

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))

import stat_parity as sp  # noqa: E402

PERTURB = {1: "Lambertian BRDF x 0.98", 2: "sky x 1.02", 3: "dielectric refraction without the eta^2 factor"}


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    out = {"K": sp.K_ENSEMBLE, "ensemble_seeds": sp.ENSEMBLE_SEEDS, "null_renders": sp.NULL_RENDERS,
           "null_seeds": [sp.NULL_SEEDS[0], sp.NULL_SEEDS[-1], 7919], "alpha_per_check": sp.ALPHA,
           "width": sp.WIDTH, "spp": sp.SPP, "grid": sp.GRID, "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        for case in sorted(sp.CASES):
            path = sp.scene_file(sp.CASES[case][0], td)
            for adaptive in (False, True):
                key = sp.case_key(case, adaptive)
                ens = sp.ensemble(path, case, adaptive, threads)
                rs = [ens.compare(sp.restatement(path, case, adaptive, s, threads)) for s in sp.NULL_SEEDS]
                chi = np.array([r["chi2_dof"] for r in rs])
                fit = sp.chi2_fit(chi)
                K = ens.K
                q95, q99 = sps.t.ppf(0.975, K - 1), sps.t.ppf(0.995, K - 1)
                # pooled tile t-values are not stored per render: recompute them from the maxima's
                # definition would lose them, so take the image channels and spp here and the tile
                # pool from a dedicated pass over the first 50 null renders
                timg = np.array([r["t_image"] for r in rs]).ravel()
                tspp = np.array([r["t_spp"] for r in rs])
                pool = []
                for s in sp.NULL_SEEDS[:50]:
                    tiles, _, _ = sp.restatement(path, case, adaptive, s, threads)
                    t, live, _ = ens._t(tiles, ens.tiles)
                    pool.append(t[live])
                pool = np.concatenate(pool)
                false_alarms = [i for i, r in enumerate(rs) if sp.verdict(r, K, (fit["lo"], fit["hi"]), adaptive)]
                power = {}
                for mode, what in PERTURB.items():
                    r = ens.compare(sp.restatement(path, case, adaptive, 424242, threads, perturb=mode))
                    power[str(mode)] = {"change": what, "fails": sp.verdict(r, K, (fit["lo"], fit["hi"]), adaptive),
                                        "chi2_dof": r["chi2_dof"], "t_tile_max": r["t_tile_max"],
                                        "t_image": [float(x) for x in r["t_image"]]}
                out["cases"][key] = {
                    "ensemble_digest": ens.digest(),
                    "chi2_dof_null": {**fit, "min": float(chi.min()), "max": float(chi.max()),
                                      "q01": float(np.quantile(chi, 0.01)), "q50": float(np.quantile(chi, 0.5)),
                                      "q99": float(np.quantile(chi, 0.99))},
                    "t_exceed_5pct": {"tiles": float(np.mean(np.abs(pool) > q95)),
                                      "image": float(np.mean(np.abs(timg) > q95)),
                                      "spp": float(np.mean(np.abs(tspp) > q95)) if adaptive else None},
                    "t_exceed_1pct": {"tiles": float(np.mean(np.abs(pool) > q99)),
                                      "image": float(np.mean(np.abs(timg) > q99)),
                                      "spp": float(np.mean(np.abs(tspp) > q99)) if adaptive else None},
                    "t_tile_max_null_max": float(max(r["t_tile_max"] for r in rs)),
                    "t_image_null_max": float(np.abs(timg).max()),
                    "null_false_alarms": len(false_alarms),
                    "power": power,
                }
                c = out["cases"][key]
                print(key, "chi2 null mean %.3f sd %.3f bounds [%.3f, %.3f] range [%.3f, %.3f]" % (
                    fit["mean"], np.sqrt(fit["var"]), fit["lo"], fit["hi"], chi.min(), chi.max()),
                    "exceed5", c["t_exceed_5pct"], "false alarms", len(false_alarms),
                    "power", {m: bool(p["fails"]) for m, p in power.items()}, flush=True)
    dst = os.path.join(ROOT, "tests", "golden", "stat_null.json")
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main()
