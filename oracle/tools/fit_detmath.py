"""Fit the polynomial cores of the deterministic f32 elementary functions.

Test/oracle tooling only.  The fitted coefficients are pasted (as float32 hex-exact
decimal literals) into BOTH oracle/detmath_ref.h and the product's csrc/detmath.h;
the two headers are separate restatements that must evaluate identically.

Method: Lawson-weighted least squares on Chebyshev nodes (converges to minimax of the
relative error), float64, then rounded to float32.
"""
import numpy as np


def lawson(f_target, basis, x, iters=60, rel=True):
    A = np.stack([b(x) for b in basis], axis=1)
    y = f_target(x)
    scale = np.abs(y) if rel else np.ones_like(y)
    scale[scale == 0] = 1.0
    w = np.ones_like(x) / len(x)
    for _ in range(iters):
        sw = np.sqrt(w) / scale
        c, *_ = np.linalg.lstsq(A * sw[:, None], y * sw, rcond=None)
        err = np.abs(A @ c - y) / scale
        w = w * err
        w /= w.sum()
    return c, np.max(np.abs(A @ c - y) / scale)


def cheb(a, b, n=4000):
    k = np.arange(n)
    return 0.5 * (a + b) + 0.5 * (b - a) * np.cos((2 * k + 1) * np.pi / (2 * n))


def show(name, c):
    c32 = c.astype(np.float32)
    print(name, ", ".join(repr(float(v)) + "f" for v in c32))


if __name__ == "__main__":
    # exp: e^r = 1 + r + r^2*(c2 + c3 r + ... + c6 r^4), r in [-ln2/2, ln2/2]
    r = cheb(-0.3466, 0.3466)
    basis = [lambda x, k=k: x ** (k + 2) for k in range(5)]
    c, e = lawson(lambda x: np.expm1(x) - x, basis, r)
    show("exp c2..c6", c); print("  max rel err (of e^r - 1 - r)", e)
    # sin: sin r = r + r^3*(s0 + s1 z + s2 z^2 + s3 z^3), z=r^2, |r|<=pi/4
    z = cheb(1e-12, (np.pi / 4) ** 2)
    from math import factorial
    sin_core = lambda zz: sum((-1) ** k * zz ** (k - 1) / factorial(2 * k + 1) for k in range(1, 14))
    c, e = lawson(sin_core,
                  [lambda zz, k=k: zz ** k for k in range(4)], z)
    show("sin s0..s3", c); print("  max rel err", e)
    # cos: cos r = 1 - z/2 + z^2*(k0 + k1 z + k2 z^2 + k3 z^3)
    from math import factorial
    cos_core = lambda zz: sum((-1) ** k * zz ** (k - 2) / factorial(2 * k) for k in range(2, 14))
    c, e = lawson(cos_core,
                  [lambda zz, k=k: zz ** k for k in range(4)], z)
    show("cos k0..k3", c); print("  max rel err", e)
    # asin: asin x = x + x*z*P(z), z = x^2 in [0, 0.25]
    z = cheb(1e-12, 0.25)
    from math import comb
    asin_core = lambda zz: sum(comb(2 * k, k) / (4 ** k * (2 * k + 1)) * zz ** (k - 1) for k in range(1, 40))
    c, e = lawson(asin_core,
                  [lambda zz, k=k: zz ** k for k in range(6)], z)
    show("asin p0..p5", c); print("  max rel err", e)
    # atan: atan t = t + t*z*A(z), z = t^2 in [0, 1]
    z = cheb(1e-12, 1.0)
    for deg in (8, 9, 10, 11):
        def atan_core(zz):
            ser = sum((-1) ** k * zz ** (k - 1) / (2 * k + 1) for k in range(1, 40))
            dirr = (np.arctan(np.sqrt(zz)) - np.sqrt(zz)) / (np.sqrt(zz) * zz)
            return np.where(zz < 0.25, ser, dirr)
        c, e = lawson(atan_core,
                      [lambda zz, k=k: zz ** k for k in range(deg)], z)
        print("atan deg", deg, "err", e)
    show("atan a0..", c)
