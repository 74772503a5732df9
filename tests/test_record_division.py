"""k_adapt_record's division by the running sample count (rtx_frame_kernels.h div_by_count):
RecordSample's `delta / n` (pixel_state.h:30) formed from one reciprocal per sample and a
Markstein correction must equal the IEEE quotient bit for bit.  A small C program (gcc,
-ffp-contract=off, the C library's fma) checks random, integer-multiple and near-tie dividends
for every count up to 4096, and for sampled larger counts up to 2^31 (every power of two and its
neighbours, random counts between): the API accepts any spp budget, and the samples counter is
32-bit."""
import os
import subprocess

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static double div_by_count(double delta, double n, double y) {  /* as the kernel */
  double q = delta * y;
  q = fma(fma(-q, n, delta), y, q);
  if (!(fabs(delta) >= 0x1p-900 && fabs(delta) < INFINITY)) q = delta / n;
  return q;
}
static long bad = 0, tot = 0;
static void check_count(long n, int iters);
int main(void) {
  for (long n = 1; n <= 4096; n++) check_count(n, 1200);
  for (int k = 12; k <= 31; k++)  /* powers of two and their neighbours up to 2^31 */
    for (long d = -2; d <= 2; d++) {
      const long n = (1L << k) + d;
      if (n > 4096 && n <= (1L << 31)) check_count(n, 600);
    }
  for (int i = 0; i < 3000; i++) check_count(4097 + (long)(rnd() % ((1UL << 31) - 4096)), 200);
  printf("checked %ld mismatches %ld\n", tot, bad);
  return bad != 0;
}
static void check_count(long n, int iters) {
  {
    const double dn = (double)n, y = 1.0 / dn;
    for (int it = 0; it < iters; it++) {
      double a;
      switch (it % 5) {
        case 0: a = bits((rnd() & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 40 + rnd() % 60) << 52)); break;
        case 1: a = (double)(rnd() % 100000) * dn; break;
        case 2: { double b = bits((rnd() & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 30 + rnd() % 40) << 52));
                  a = nextafter(b * dn, (rnd() & 1) ? INFINITY : -INFINITY); break; }
        case 3: a = ((double)(rnd() % 2000001) - 1000000.0) / 1024.0; break;
        default: { const double sp[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 0x1p-1000, -0x1p-1074, 0x1p-900};
                   a = sp[rnd() % 8]; }
      }
      double q = div_by_count(a, dn, y), e = a / dn;
      tot++;
      if (!(isnan(q) && isnan(e)) && memcmp(&q, &e, 8) != 0) {
        if (bad < 5) printf("n=%ld a=%a got %a want %a\n", n, a, q, e);
        bad++;
      }
    }
  }
}
"""


def test_division_by_count_is_the_ieee_quotient(tmp_path):
    src, exe = tmp_path / "div.c", tmp_path / "div"
    src.write_text(SRC)
    try:
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"], check=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"gcc unavailable: {e}")
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout
