"""Exact double sums (SK_FX, pinot_amd/csrc/pg_internal.h): the fixed-point conversion, the 128-bit add and the final
rounding, checked against exact rational arithmetic (fractions.Fraction) on the host.

The device accumulates every SUM / AVG input that is not provably an integer as round(x / 2^shift) in a 128-bit
two's-complement integer and converts the total once: the result is the exact sum of the rounded inputs, rounded to the
nearest double -- the same bits in any order (the reference's double sum depends on its thread scheduling; SURVEY
§8(e)).  The header's functions are __host__ __device__, so the same code compiled by g++ here is what runs in the
kernels and in the host finalisation."""
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
// stdin: int32 shift, uint32 n, n doubles.  stdout: per value "lo hi", then the sums in order and reversed ("lo hi"),
// then fx_to_double of the sum as its IEEE bits, then fx_final with special slots for +inf / -inf / NaN inputs
int main() {
  int32_t shift; uint32_t n;
  if (fread(&shift, 4, 1, stdin) != 1 || fread(&n, 4, 1, stdin) != 1) return 1;
  std::vector<double> x(n);
  if (n && fread(x.data(), 8, n, stdin) != n) return 1;
  uint64_t slo = 0, shi = 0, rlo = 0, rhi = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint64_t lo, hi;
    pg::fx_from_double(x[i], shift, lo, hi);
    printf("%llu %llu\n", (unsigned long long)lo, (unsigned long long)hi);
    pg::fx_add(slo, shi, lo, hi);
  }
  for (uint32_t i = n; i-- > 0;) { uint64_t lo, hi; pg::fx_from_double(x[i], shift, lo, hi); pg::fx_add(rlo, rhi, lo, hi); }
  printf("%llu %llu\n%llu %llu\n", (unsigned long long)slo, (unsigned long long)shi, (unsigned long long)rlo,
         (unsigned long long)rhi);
  double d = pg::fx_to_double(slo, shi, shift);
  uint64_t b; __builtin_memcpy(&b, &d, 8);
  printf("%llu\n", (unsigned long long)b);
  pg::AggSpec a{}; a.fx_shift = shift; a.sp_min = 0; a.sp_max = 0;
  const int64_t none_mn = pg::order_key(__builtin_inf()), none_mx = pg::order_key(-__builtin_inf());
  const double cases[5] = {
    pg::fx_final(a, slo, shi, none_mn, none_mx),                                             // no special input
    pg::fx_final(a, slo, shi, pg::order_key(__builtin_inf()), pg::order_key(__builtin_inf())), // +inf
    pg::fx_final(a, slo, shi, pg::order_key(-__builtin_inf()), pg::order_key(-__builtin_inf())), // -inf
    pg::fx_final(a, slo, shi, pg::order_key(-__builtin_inf()), pg::order_key(__builtin_inf())), // both
    pg::fx_final(a, slo, shi, none_mn, pg::order_key(__builtin_nan("")))};                  // NaN
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


def _run(exe, shift, xs):
    data = struct.pack("<iI", shift, len(xs)) + np.asarray(xs, dtype=np.float64).tobytes()
    out = subprocess.run([exe], input=data, capture_output=True, check=True).stdout.decode().split("\n")
    vals = [tuple(int(t) for t in out[i].split()) for i in range(len(xs))]
    fwd = tuple(int(t) for t in out[len(xs)].split())
    rev = tuple(int(t) for t in out[len(xs) + 1].split())
    bits = int(out[len(xs) + 2])
    finals = [float(v) for v in out[len(xs) + 3:len(xs) + 8]]
    return vals, fwd, rev, bits, finals


def _signed128(lo, hi):
    v = lo | (hi << 64)
    return v - (1 << 128) if v >> 127 else v


def _round_half_even(fr: Fraction) -> int:
    q, r = divmod(fr.numerator, fr.denominator)
    twice = 2 * r
    if twice > fr.denominator or (twice == fr.denominator and q & 1):
        q += 1
    return q


@pytest.mark.parametrize("seed,scale", [(1, 1.0), (2, 1e12), (3, 1e-6), (4, 3.0e300), (5, 1.0)])
def test_fixed_point_sum_is_exact_and_order_free(harness, seed, scale):
    rng = np.random.default_rng(seed)
    xs = rng.normal(size=4000) * scale
    if seed == 5:  # values spanning many binades of one bound, with exact ties at the unit
        xs = np.concatenate([xs, rng.normal(size=500) * 2.0 ** -40, [0.0, -0.0, 2.0 ** -90, -(2.0 ** -90)]])
    bound = float(np.abs(xs).max())
    e = int(np.frexp(bound)[1])                      # bound <= 2^e (pg_agg.sum_exp)
    shift = e + 40 - 126                             # fx_shift_for(e)
    vals, fwd, rev, bits, finals = _run(harness, shift, xs)
    unit = Fraction(2) ** shift
    units = []
    for x, (lo, hi) in zip(xs, vals):
        want = _round_half_even(Fraction(float(x)) / unit) if x >= 0 else -_round_half_even(-Fraction(float(x)) / unit)
        assert _signed128(lo, hi) == want, (x, lo, hi, want)
        units.append(want)
    assert fwd == rev                                # the 128-bit adds commute: any order, the same bits
    total = sum(units)
    assert _signed128(*fwd) == total
    got = struct.unpack("<d", struct.pack("<Q", bits))[0]
    assert got == float(total * unit)                # one round-to-nearest-even of the exact total
    assert finals[0] == got
    assert finals[1] == float("inf") and finals[2] == float("-inf")
    assert finals[3] != finals[3] and finals[4] != finals[4]   # +inf with -inf, and NaN: NaN
    # the reference's sequential double sum is within its own rounding error of the exact total (SURVEY: 1e-9)
    seq = 0.0
    for x in xs:
        seq += float(x)
    exact = sum(Fraction(float(x)) for x in xs)
    assert abs(Fraction(got) - exact) <= abs(Fraction(seq) - exact) + abs(exact) * Fraction(1, 2 ** 52)


def test_integer_inputs_are_exact(harness):
    """Integers (PG_PLAN_F64_SUMS over integer columns): the unit is a negative power of two, so every integer input
    converts exactly and the sum is the exact integer sum (rounded once only above 2^53)."""
    xs = [float(v) for v in np.random.default_rng(9).integers(-10 ** 12, 10 ** 12, 3000)]
    e = int(np.frexp(max(abs(v) for v in xs))[1])
    _, fwd, _, bits, _ = _run(harness, e + 40 - 126, xs)
    assert _signed128(*fwd) * Fraction(2) ** (e + 40 - 126) == sum(int(v) for v in xs)
    assert struct.unpack("<d", struct.pack("<Q", bits))[0] == float(sum(int(v) for v in xs))
