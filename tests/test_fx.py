"""Exact double sums (SK_FX, pinot_amd/csrc/pg_internal.h): the exponent-window split, the 128-bit adds and the final
rounding, checked against exact rational arithmetic (fractions.Fraction) on the host.

Every finite SUM / AVG input that is not provably an integer is m * 2^q (m < 2^53); the host bounds the table's nonzero
inputs by 2^klo <= |x| <= 2^khi, and the device adds x EXACTLY, as the integer x / 2^(u0 + 32 w), into the 128-bit
two's-complement window w that holds its exponent q (fx_split).  The final value is the windows' exact total rounded
once (fx_windows_to_double): the correctly rounded sum of the inputs for ANY range of magnitudes -- 1e30 next to 0.01,
Double.MAX_VALUE next to subnormals -- and the same bits in any order (the reference's double sum depends on its thread
scheduling).  The header's functions are __host__ __device__, so the same code compiled by g++ here is
what runs in the kernels and in the host finalisation."""
import math
import os
import struct
import subprocess
from fractions import Fraction

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = r"""
#include "pg_internal.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
// stdin: int32 klo, int32 khi, uint32 n, n doubles.  stdout: u0 nwin; per value "w lo hi"; the window sums in order
// and reversed (one "lo hi" line per window each); fx_final of the sum as its IEEE bits; then fx_final with special
// slots for +inf / -inf / NaN inputs
int main() {
  int32_t klo, khi; uint32_t n;
  if (fread(&klo, 4, 1, stdin) != 1 || fread(&khi, 4, 1, stdin) != 1 || fread(&n, 4, 1, stdin) != 1) return 1;
  std::vector<double> x(n);
  if (n && fread(x.data(), 8, n, stdin) != n) return 1;
  const int32_t u0 = pg::fx_u0(klo);
  const uint32_t nw = pg::fx_num_windows(klo, khi);
  printf("%d %u\n", u0, nw);
  std::vector<uint64_t> f(2 * nw, 0), r(2 * nw, 0);
  for (uint32_t i = 0; i < n; i++) {
    uint64_t lo, hi;
    const uint32_t w = pg::fx_split(x[i], u0, nw, lo, hi);
    printf("%u %llu %llu\n", w, (unsigned long long)lo, (unsigned long long)hi);
    pg::fx_add(f[2 * w], f[2 * w + 1], lo, hi);
  }
  for (uint32_t i = n; i-- > 0;) {
    uint64_t lo, hi;
    const uint32_t w = pg::fx_split(x[i], u0, nw, lo, hi);
    pg::fx_add(r[2 * w], r[2 * w + 1], lo, hi);
  }
  for (uint32_t w = 0; w < nw; w++) printf("%llu %llu\n", (unsigned long long)f[2 * w], (unsigned long long)f[2 * w + 1]);
  for (uint32_t w = 0; w < nw; w++) printf("%llu %llu\n", (unsigned long long)r[2 * w], (unsigned long long)r[2 * w + 1]);
  pg::AggSpec a{}; a.fx_shift = u0; a.fx_nwin = nw; a.sp_min = 0; a.sp_max = 0;
  const int64_t none_mn = pg::order_key(__builtin_inf()), none_mx = pg::order_key(-__builtin_inf());
  double d = pg::fx_final(a, f.data(), none_mn, none_mx);
  uint64_t b; __builtin_memcpy(&b, &d, 8);
  printf("%llu\n", (unsigned long long)b);
  const double cases[4] = {
    pg::fx_final(a, f.data(), pg::order_key(__builtin_inf()), pg::order_key(__builtin_inf())),    // +inf
    pg::fx_final(a, f.data(), pg::order_key(-__builtin_inf()), pg::order_key(-__builtin_inf())),  // -inf
    pg::fx_final(a, f.data(), pg::order_key(-__builtin_inf()), pg::order_key(__builtin_inf())),   // both
    pg::fx_final(a, f.data(), none_mn, pg::order_key(__builtin_nan("")))};                     // NaN
  for (double c : cases) printf("%.17g\n", c);
  return 0;
}
"""


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("fx")
    src = d / "fx.cpp"
    src.write_text(HARNESS)
    exe = d / "fx"
    subprocess.run(["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I" + os.path.join(ROOT, "pinot_amd", "csrc"), "-o", str(exe), str(src)], check=True)
    return str(exe)


def bounds(xs):
    """(klo, khi) as pinot_amd.plan.sum_bound forms them: 2^klo <= |x| <= 2^khi for the nonzero finite inputs."""
    a = np.abs(np.asarray(xs, dtype=np.float64))
    a = a[np.isfinite(a) & (a > 0)]
    khi = math.frexp(float(a.max()))[1]
    klo = math.frexp(float(a.min()))[1] - 1
    return klo, khi


def _run(exe, klo, khi, xs):
    data = struct.pack("<iiI", klo, khi, len(xs)) + np.asarray(xs, dtype=np.float64).tobytes()
    out = subprocess.run([exe], input=data, capture_output=True, check=True).stdout.decode().split("\n")
    u0, nw = (int(t) for t in out[0].split())
    vals = [tuple(int(t) for t in out[1 + i].split()) for i in range(len(xs))]
    o = 1 + len(xs)
    fwd = [tuple(int(t) for t in out[o + w].split()) for w in range(nw)]
    rev = [tuple(int(t) for t in out[o + nw + w].split()) for w in range(nw)]
    bits = int(out[o + 2 * nw])
    finals = [float(v) for v in out[o + 2 * nw + 1:o + 2 * nw + 5]]
    return u0, nw, vals, fwd, rev, struct.unpack("<d", struct.pack("<Q", bits))[0], finals


def _signed128(lo, hi):
    v = lo | (hi << 64)
    return v - (1 << 128) if v >> 127 else v


def _check(harness, xs, klo=None, khi=None):
    if klo is None:
        klo, khi = bounds(xs)
    u0, nw, vals, fwd, rev, got, finals = _run(harness, klo, khi, xs)
    assert 1 <= nw <= 64
    total = Fraction(0)
    for x, (w, lo, hi) in zip(xs, vals):
        unit = Fraction(2) ** (u0 + 32 * w)
        assert Fraction(float(x)) == _signed128(lo, hi) * unit, (x, w)   # every input converts EXACTLY
        if x != 0:
            m, e = math.frexp(abs(float(x)))
            q = max(e - 53, -1074)                                         # its last mantissa bit's exponent
            assert w == (q - u0) // 32, (x, w, q, u0)
            assert abs(_signed128(lo, hi)) < 2 ** 85
        total += Fraction(float(x))
    assert fwd == rev                                                      # the 128-bit adds commute: the same bits
    assert sum(_signed128(*p) * Fraction(2) ** (u0 + 32 * w) for w, p in enumerate(fwd)) == total
    assert got == float(total)                  # ONE round-to-nearest-even of the exact total (Fraction -> float)
    assert finals[0] == float("inf") and finals[1] == float("-inf")
    assert finals[2] != finals[2] and finals[3] != finals[3]   # +inf with -inf, and NaN: NaN
    return nw, got, total


@pytest.mark.parametrize("seed,scale", [(1, 1.0), (2, 1e12), (3, 1e-6), (4, 3.0e300), (5, 1.0)])
def test_fixed_point_sum_is_exact_and_order_free(harness, seed, scale):
    rng = np.random.default_rng(seed)
    xs = rng.normal(size=4000) * scale
    if seed == 5:  # values spanning many binades, with zeros and tiny values
        xs = np.concatenate([xs, rng.normal(size=500) * 2.0 ** -40, [0.0, -0.0, 2.0 ** -90, -(2.0 ** -90)]])
    _, got, exact = _check(harness, xs)
    # the reference's sequential double sum is within its own rounding error of the exact total (SURVEY: 1e-9)
    seq = 0.0
    for x in xs:
        seq += float(x)
    assert abs(Fraction(got) - exact) <= abs(Fraction(seq) - exact) + abs(exact) * Fraction(1, 2 ** 52)


def test_wide_range_inputs_keep_every_small_value(harness):
    """one 1e30 (or Double.MAX_VALUE) beside values in [0.01, 100) -- the old single-unit sum
    rounded the small ones to 0.  Each window is exact, so the small values' own sum survives, and a subset that never
    sees the large value sums exactly as the reference's double sum of it would (within its rounding error)."""
    rng = np.random.default_rng(11)
    small = rng.uniform(0.01, 100.0, 3000)
    for big in (1e30, np.finfo(np.float64).max, -1e30):
        xs = np.concatenate([small, [big]])
        nw, got, exact = _check(harness, xs)
        assert nw > 1
        # the windows of the small values alone (a group / filter that never sees `big`) under the SAME bounds
        klo, khi = bounds(xs)
        _, _, _, _, _, got_small, _ = _run(harness, klo, khi, small)
        seq = 0.0
        for x in small:
            seq += float(x)
        assert got_small == float(sum(Fraction(float(x)) for x in small))
        assert abs(got_small - seq) <= 1e-12 * abs(seq)
    # cancellation: 1e30 + small - 1e30 is exactly the small sum (a double sum loses it entirely)
    xs = np.concatenate([[1e30], small, [-1e30]])
    _, got, exact = _check(harness, xs)
    assert exact == sum(Fraction(float(x)) for x in small) and got == float(exact)


def test_products_and_subnormals(harness):
    """SUM(a*b) with both operands up to 1e9 and down to 1e-3: products in [1e-6, 1e18]; and subnormal inputs next to
    normal ones (the window of the smallest subnormal's exponent, 2^-1074)."""
    rng = np.random.default_rng(12)
    a = rng.uniform(1e-3, 1e9, 2000)
    b = rng.uniform(1e-3, 1e9, 2000)
    prods = a * b
    lo = math.frexp(1e-3 * 1e-3)[1] - 1
    hi = math.frexp(1e9)[1] * 2
    nw, _, _ = _check(harness, prods, lo, hi)
    assert nw >= 2
    sub = [5e-324, -5e-324 * 7, 2.0 ** -1060, 1.0, 3.5e-310, 1e300]
    nw, _, _ = _check(harness, sub)
    assert nw == 64 or nw >= 60


def test_integer_inputs_are_exact(harness):
    """Integers (PG_PLAN_F64_SUMS over integer columns): klo = 0, so every integer input converts exactly and the sum
    is the exact integer sum (rounded once only above 2^53)."""
    xs = [float(v) for v in np.random.default_rng(9).integers(-10 ** 12, 10 ** 12, 3000)]
    _, got, exact = _check(harness, xs, 0, math.frexp(max(abs(v) for v in xs))[1])
    assert exact == sum(int(v) for v in xs) and got == float(sum(int(v) for v in xs))


def test_plan_bounds_follow_the_expression():
    """pinot_amd.plan.sum_bound: the table-global (sum_exp, sum_exp_lo) sent with PG_SUM_BOUNDS -- a bound in
    [0.5, 1) is 0 and still explicit (sum_exp == 0 used to mean "let each GPU derive its own")."""
    from pinot_amd.plan import sum_bound

    class T:
        def __init__(self, hi, lo):
            self.hi, self.lo = hi, lo

        def abs_bound(self, c):
            return self.hi[c]

        def abs_low(self, c):
            return self.lo[c]

        def has_nonfinite(self, c):
            return False

    class E:
        def __init__(self, op, cols):
            self.op, self.cols = op, cols
    t = T({"a": 0.9, "b": 1e9, "c": 1e30}, {"a": 0.6, "b": 1e-3, "c": 0.01})
    assert sum_bound(t, E("COL", ["a"])) == (0, -1, False)
    khi, klo, _ = sum_bound(t, E("MUL", ["b", "b"]))
    assert 2.0 ** klo <= 1e-6 and 1e18 <= 2.0 ** khi
    khi, klo, _ = sum_bound(t, E("ADD", ["a", "c"]))
    assert 2.0 ** klo <= 0.01 * 2.0 ** -52 and 1e30 + 0.9 <= 2.0 ** khi
