"""Fit the fp32 polynomial kernels used by rt_fmath (device) and the oracle (host).

The path tracer needs sin/cos/log/acos/atan2 (vec3.rs:240-250, object.rs:114-132,
constant_medium.rs:75, texture.rs:127-130). Hardware/libm transcendentals differ between the
CPU and gfx950, so both sides evaluate the SAME polynomials with the same fma/mul/add order.
This script produces the coefficients (weighted least squares on Chebyshev nodes, then rounded
to float) and reports the fp32-evaluated max error. Run: python fit_fmath.py
"""
import numpy as np


def f32(x):
    return np.float32(x)


def fit_odd(fn, lo, hi, nterms, rel=True):
    # fn(x) ~= x * P(x^2), P of nterms coefficients
    k = np.arange(4000)
    x = 0.5 * (lo + hi) + 0.5 * (hi - lo) * np.cos(np.pi * (k + 0.5) / 4000)
    x = x[x != 0]
    y = fn(x)
    A = np.stack([x ** (2 * i + 1) for i in range(nterms)], 1)
    w = 1 / np.abs(y) if rel else np.ones_like(y)
    c, *_ = np.linalg.lstsq(A * w[:, None], y * w, rcond=None)
    return [float(np.float32(v)) for v in c]


def fit_even(fn, lo, hi, nterms):
    k = np.arange(4000)
    x = 0.5 * (lo + hi) + 0.5 * (hi - lo) * np.cos(np.pi * (k + 0.5) / 4000)
    y = fn(x)
    A = np.stack([x ** (2 * i) for i in range(nterms)], 1)
    w = 1 / np.abs(y)
    c, *_ = np.linalg.lstsq(A * w[:, None], y * w, rcond=None)
    return [float(np.float32(v)) for v in c]


def horner_odd(c, x):
    x = f32(x)
    x2 = f32(x * x)
    p = f32(c[-1])
    for ci in reversed(c[:-1]):
        p = f32(np.fma(p, x2, f32(ci))) if hasattr(np, "fma") else f32(p * x2 + f32(ci))
    return f32(p * x)


def horner_even(c, x):
    x = f32(x)
    x2 = f32(x * x)
    p = f32(c[-1])
    for ci in reversed(c[:-1]):
        p = f32(p * x2 + f32(ci))
    return p


def report(name, c):
    print(f"// {name}")
    for v in c:
        print(f"  {np.float32(v).item().hex()}f, /* {v:.9g} */")


if __name__ == "__main__":
    q = np.pi / 2
    # sin/cos of a quarter-turn fraction r in [-1/2, 1/2]: theta = r*pi/2
    s = fit_odd(lambda r: np.sin(q * r), -0.5, 0.5, 5)
    c = fit_even(lambda r: np.cos(q * r), -0.5, 0.5, 6)
    report("SINQ (x r, r^3, ...)", s)
    report("COSQ (1, r^2, ...)", c)
    # sin/cos of theta in [-pi/4, pi/4]
    s2 = fit_odd(np.sin, -np.pi / 4, np.pi / 4, 5)
    c2 = fit_even(np.cos, -np.pi / 4, np.pi / 4, 6)
    report("SIN (x, x^3, ...)", s2)
    report("COS (1, x^2, ...)", c2)
    # atan on [-(2-sqrt3), 2-sqrt3]
    t = 2 - np.sqrt(3)
    a = fit_odd(np.arctan, -t, t, 6)
    report("ATAN", a)
    # asin on [-1/2, 1/2]
    b = fit_odd(np.arcsin, -0.5, 0.5, 7)
    report("ASIN", b)
    # error report in float64 evaluation of float coefficients
    for name, cc, fn, lo, hi, odd in [
        ("sinq", s, lambda r: np.sin(q * r), -0.5, 0.5, True),
        ("cosq", c, lambda r: np.cos(q * r), -0.5, 0.5, False),
        ("sin", s2, np.sin, -np.pi / 4, np.pi / 4, True),
        ("cos", c2, np.cos, -np.pi / 4, np.pi / 4, False),
        ("atan", a, np.arctan, -t, t, True),
        ("asin", b, np.arcsin, -0.5, 0.5, True),
    ]:
        x = np.linspace(lo, hi, 100001)
        x = x[x != 0]
        p = np.zeros_like(x)
        for i, ci in enumerate(cc):
            p += ci * x ** (2 * i + (1 if odd else 0))
        err = np.max(np.abs(p - fn(x)) / np.abs(fn(x)))
        print(f"// {name}: max rel err (f64 eval of f32 coeffs) = {err:.3g}")
