"""The device's polynomial transcendentals (rt_kernel.h sincos2pi, log_u01), host-only: the
coefficients are read from the kernel source and evaluated step by step in f64 with the same
fused operations (an fma is exact-product-plus-add, rounded once), then compared with the
exact values (mpmath, 200 bits). Both must stay within an ulp, like the libm results the oracle
uses (vec3.rs:244 / object.rs:127 phi = 2 pi r1; constant_medium.rs:75 log of a draw)."""
import math
import random
import re
from pathlib import Path

import mpmath as mp
import pytest

SRC = (Path(__file__).resolve().parent.parent / "surely-raytracing_amd" / "csrc" /
       "rt_kernel.h").read_text()
mp.mp.prec = 200


def _fn(name):
    i = SRC.index(f"void {name}(" if name == "sincos2pi" else f"double {name}(")
    return SRC[i:SRC.index("\n}\n", i)]


def _hexes(body, var):
    """The Horner coefficients of `var`, outermost first: the initial literal, then the fma_k
    constants in order."""
    first = re.search(rf"double {var} = (-?0x[0-9a-fp.+-]+);", body).group(1)
    rest = re.findall(rf"{var} = fma_k<__builtin_bit_cast\(uint64_t, \(?(?:double\)\()?"
                      rf"(-?0x[0-9a-fp.+-]+)\)?\)?>\({var}, \w+\);", body)
    return [float.fromhex(first)] + [float.fromhex(h) for h in rest]


def fma(a, b, c):
    return float(mp.mpf(a) * mp.mpf(b) + mp.mpf(c))


def ulps(v, exact):
    e = math.frexp(float(exact))[1]
    return float(abs(mp.mpf(v) - exact) / mp.mpf(2) ** (e - 53))


def test_sincos2pi_within_an_ulp():
    body = _fn("sincos2pi")
    S, C = _hexes(body, "s"), _hexes(body, "c")
    assert len(S) == 6 and len(C) == 6
    rng = random.Random(5)
    worst = 0.0
    for i in range(1500):
        u = rng.getrandbits(32) * 2.0 ** -32  # a draw: k * 2^-32
        t = 4.0 * u
        k = math.floor(t + 0.5)
        th = (t - k) * (0.5 * math.pi)
        x2 = th * th
        s = S[0]
        for c in S[1:]:
            s = fma(s, x2, c)
        s = fma(th * x2, s, th)
        c = C[0]
        for cc in C[1:]:
            c = fma(c, x2, cc)
        c = fma(fma(c, x2, -0.5), x2, 1.0)
        if th != 0.0:
            worst = max(worst, ulps(s, mp.sin(mp.mpf(th))))
        worst = max(worst, ulps(c, mp.cos(mp.mpf(th))))
    assert worst < 1.0, worst


def test_log_u01_within_an_ulp_and_log0():
    body = _fn("log_u01")
    R = _hexes(body, "r")
    assert len(R) == 7
    ln2_lo = float.fromhex(re.search(r"dk \* (0x[0-9a-fp.+-]+)\);  // ln2_lo", body).group(1))
    ln2_hi = float.fromhex(re.search(r"dk \* (0x[0-9a-fp.+-]+) - ", body).group(1))
    assert "x == 0.0 ? -kInf" in body  # log(0) = -inf: the reference's infinite free path

    def flog(x):
        m, e = math.frexp(x)
        if m < 0.7071067811865476:
            m, e = m * 2.0, e - 1
        f = m - 1.0
        hfsq = 0.5 * f * f
        s = float(mp.mpf(f) / mp.mpf(2.0 + f))  # div_nr: the IEEE quotient within an ulp
        z = s * s
        r = R[0]
        for c in R[1:]:
            r = fma(r, z, c)
        dk = float(e)
        t = fma(s, hfsq + r * z, dk * ln2_lo)
        return dk * ln2_hi - ((hfsq - t) - f)

    rng = random.Random(7)
    ks = [1, 2, 3, 2 ** 31, 2 ** 32 - 1, 0x5A827999] + [rng.getrandbits(32) for _ in range(1500)]
    worst = max(ulps(flog(k * 2.0 ** -32), mp.log(mp.mpf(k) * mp.mpf(2) ** -32))
                for k in ks if k)
    assert worst < 1.0, worst


@pytest.mark.parametrize("name", ["sincos2pi", "log_u01"])
def test_polynomials_use_sgpr_constant_fmas(name):
    """The Horner steps go through fma_k (v_fma_f64 with the constant in an SGPR pair), not a
    plain fma the compiler would turn into v_fmac_f64 plus two constant moves per step."""
    body = _fn(name)
    assert body.count("fma_k<") >= 5
