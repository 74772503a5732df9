"""Statistics of the statistical parity leg (tests/test_statistical_parity.py), shared with the
script that calibrates them (oracle/gen_stat_null.py).  Test infrastructure only.

Two renders of one image by different Monte Carlo estimators agree when their difference is
within the Monte Carlo error.  That error is NOT taken from the per-pixel sample variances the
renderers keep (PixelState::m2 / n, pixel_state.h:41-49): under adaptive sampling a pixel stops
when its sample variance happens to be low (pixel_state.h:54-72, wavefront.cc:125-127), so
var / n is biased low, and the round-5 test's chi-square sat at ~1.3 under the null.  Instead
the error comes from an ENSEMBLE of K independent restatement renders (fixed seeds): for every
tile mean (8 x 8 tiles x 3 channels), image mean and mean sample count, y the reference's value,
x_1..x_K the ensemble's,

    t = (y - mean(x)) / (sd(x) * sqrt(1 + 1/K))

which, if y and the x_i come from the same estimator, is Student-t with K - 1 degrees of freedom
(tile means of ~350 pixels x 64 samples are normal to a good approximation), whatever the
sampling scheme does to the per-pixel variances.

Checks (each at a false-alarm level ALPHA, so a whole test run of 4 cases stays below 0.2 %):
  * image mean, per channel: |t| within the t_{K-1} quantile (Bonferroni over the 3 channels);
  * tiles: max |t| within the t_{K-1} quantile, Bonferroni over the ~190 tile values;
  * tiles: chi2/dof = mean t^2 within the central 1 - ALPHA of its null distribution, measured
    (oracle/gen_stat_null.py: NULL_RENDERS restatement renders at independent seeds against the
    SAME fixed ensemble, the test's exact conditional null) and fitted by a scaled chi-square of
    the same mean and variance (tile values are correlated across channels, so the analytic
    F(1, K-1) mean does not give the spread); quantiles committed in tests/golden/stat_null.json;
  * tiles whose ensemble has zero spread: y must equal the ensemble mean;
  * adaptive renders: mean samples per pixel, |t| within the t_{K-1} quantile.
"""
import hashlib

import numpy as np
from scipy import stats as sps

WIDTH, SPP, GRID = 200, 64, 8
K_ENSEMBLE = 32
ENSEMBLE_SEEDS = [1_000_003 * (i + 1) for i in range(K_ENSEMBLE)]
NULL_RENDERS = 200
NULL_SEEDS = [7_000_001 + 7919 * i for i in range(NULL_RENDERS)]
ALPHA = 1e-4
CASES = {  # name -> (scene recipe, camera preset, max depth)
    "c2_final": ("final", "c2_final", 50),
    "c3_bunny": ("bunny", "c3_bunny", 20),
}


def case_key(case, adaptive):
    return f"{case}_{'adaptive' if adaptive else 'fixed'}"


def summary(fb, spp, hw):
    """(tile means [GRID*GRID*3], image means [3], mean samples per pixel) of one render."""
    h, w = hw
    A = np.asarray(fb, dtype=np.float64).reshape(h, w, 3)
    tiles = []
    for ys in np.array_split(np.arange(h), GRID):
        for xs in np.array_split(np.arange(w), GRID):
            tiles.append(A[np.ix_(ys, xs)].reshape(-1, 3).mean(0))
    return np.concatenate(tiles), A.reshape(-1, 3).mean(0), float(np.mean(spp))


class Ensemble:
    def __init__(self, summaries):
        self.K = len(summaries)
        self.tiles = np.array([s[0] for s in summaries])
        self.img = np.array([s[1] for s in summaries])
        self.spp = np.array([s[2] for s in summaries])

    def digest(self):
        """Identifies the ensemble the committed null was measured against."""
        h = hashlib.sha256()
        for a in (self.tiles, self.img, self.spp):
            h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
        return h.hexdigest()[:16]

    def _t(self, y, x):
        m, s = x.mean(0), x.std(0, ddof=1)
        scale = s * np.sqrt(1.0 + 1.0 / self.K)
        live = scale > 0
        t = np.where(live, (y - m) / np.where(live, scale, 1.0), 0.0)
        zero_mismatch = int(np.sum(~live & (np.abs(y - m) > 1e-12)))
        return t, live, zero_mismatch

    def compare(self, s):
        tiles, img, spp = s
        tt, live, zm = self._t(tiles, self.tiles)
        ti, _, zmi = self._t(img, self.img)
        ts, _, _ = self._t(np.array([spp]), self.spp[:, None])
        t = tt[live]
        return {"t_image": ti, "tiles": int(live.sum()), "t_tile_max": float(np.abs(t).max()),
                "chi2_dof": float(np.mean(t ** 2)), "zero_var_mismatch": zm + zmi, "t_spp": float(ts[0]),
                "spp_mean": (spp, float(self.spp.mean()))}


def t_bound(K, n_family):
    """Two-sided t_{K-1} quantile of a family of n tests at family-wise level ALPHA."""
    return float(sps.t.ppf(1.0 - ALPHA / (2.0 * n_family), K - 1))


def chi2_fit(null_values):
    """Scaled chi-square a * chi2_nu / nu with the null's mean and variance; its central
    1 - ALPHA interval."""
    v = np.asarray(null_values, dtype=np.float64)
    m, var = float(v.mean()), float(v.var(ddof=1))
    nu = 2.0 * m * m / var
    lo = m * sps.chi2.ppf(ALPHA / 2.0, nu) / nu
    hi = m * sps.chi2.ppf(1.0 - ALPHA / 2.0, nu) / nu
    return {"mean": m, "var": var, "nu": nu, "lo": float(lo), "hi": float(hi)}


def scene_file(scene, directory):
    """The main.cc recipe's scene as a .rtxs file (the product's host scene writer)."""
    import os

    import rtx

    path = os.path.join(str(directory), f"{scene}.rtxs")
    if not os.path.exists(path):
        rtx.HostScene.recipe(scene, 1234).write(path)
    return path


def restatement(path, case, adaptive, seed, threads=8, perturb=0):
    """summary() of one restatement render (oracle/librtx_oracle.so, Philox stream)."""
    import oracle_ctypes as orc

    _, preset, depth = CASES[case]
    L = orc.lib()
    L.orc_set_perturb.argtypes = [orc.C.c_int]
    old = L.orc_set_perturb(int(perturb))
    try:
        fb, spp, _ = orc.Scene(path).render(orc.camera_preset(preset), WIDTH, SPP, depth, seed, adaptive=int(adaptive),
                                            rng="philox", mode="per_pixel", threads=threads)
    finally:
        L.orc_set_perturb(old)
    return summary(fb, spp, fb.shape[:2])


def ensemble(path, case, adaptive, threads=8):
    return Ensemble([restatement(path, case, adaptive, s, threads) for s in ENSEMBLE_SEEDS])


def verdict(r, K, chi2_bounds, adaptive):
    fails = []
    b_img = t_bound(K, 3)
    if not np.all(np.abs(r["t_image"]) <= b_img):
        fails.append(f"image mean t {np.round(r['t_image'], 2)} beyond {b_img:.2f}")
    b_tile = t_bound(K, r["tiles"])
    if r["t_tile_max"] > b_tile:
        fails.append(f"tile max |t| {r['t_tile_max']:.2f} > {b_tile:.2f}")
    lo, hi = chi2_bounds
    if not lo <= r["chi2_dof"] <= hi:
        fails.append(f"chi2/dof {r['chi2_dof']:.3f} outside [{lo:.3f}, {hi:.3f}]")
    if r["zero_var_mismatch"]:
        fails.append(f"{r['zero_var_mismatch']} zero-spread tiles differ")
    if adaptive:
        b_spp = t_bound(K, 1)
        if abs(r["t_spp"]) > b_spp:
            fails.append(f"mean spp t {r['t_spp']:.2f} beyond {b_spp:.2f} ({r['spp_mean']})")
    return fails
