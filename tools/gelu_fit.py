"""Fit and check of the GEMM epilogues' GELU (csrc/common.hpp gelu_erf): GELU(x) = relu(x) - |x| 2^q(a),
a = min(|x|, 6), q a degree-6 polynomial fitted to log2 Phi(-a) (Phi the normal cdf) by iteratively
re-weighted least squares towards the minimax of the GELU error a Phi(-a) |q - log2 Phi(-a)|.
Prints the f32 coefficients and the error of the f32 evaluation (Horner with fused multiply-adds)
against the f64 erf GELU, next to the Abramowitz-Stegun 7.1.26 form it replaced.
    python tools/gelu_fit.py"""
import numpy as np
from scipy.special import erf, erfc

A, D = 6.0, 6


def fit(d=D, amax=A):
    a = np.linspace(0, amax, 20001)
    f = np.log2(0.5 * erfc(a / np.sqrt(2)))
    w = a * 0.5 * erfc(a / np.sqrt(2)) + 1e-9
    V = np.vander(a, d + 1, increasing=True)
    ww = w.copy()
    for _ in range(60):
        c, *_ = np.linalg.lstsq(V * ww[:, None], f * ww, rcond=None)
        err = (V @ c - f) * w
        ww = np.maximum(ww * (np.abs(err) / np.abs(err).max()) ** 0.3 + 1e-12, w * 1e-3)
    return [np.float32(v) for v in c]


def gelu_poly(x, c):
    a = np.minimum(np.abs(x), np.float32(A))
    q = np.full_like(a, c[-1])
    for k in range(len(c) - 2, -1, -1):  # fma: exact product + sum, one rounding
        q = (q.astype(np.float64) * a + np.float64(c[k])).astype(np.float32)
    e = np.exp2(q.astype(np.float64)).astype(np.float32)
    return (-np.abs(x).astype(np.float64) * e + np.maximum(x, 0)).astype(np.float32)


def gelu_as(x):
    z = np.abs(x) * np.float32(0.70710678)
    t = (1 / (np.float32(0.3275911) * z + 1)).astype(np.float32)
    p = np.float32(1.061405429) * t - np.float32(1.453152027)
    for k in (1.421413741, -0.284496736, 0.254829592):
        p = p * t + np.float32(k)
    e = 1 - p * t * np.exp(-z * z).astype(np.float32)
    return (0.5 * x * (1 + np.copysign(e, x))).astype(np.float32)


def main():
    c = fit()
    x = np.concatenate([np.linspace(-16, 16, 1600001, dtype=np.float32),
                        (np.random.default_rng(1).standard_normal(1000000) * 3).astype(np.float32)])
    r = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    print("coefficients (a^0 .. a^6):", ", ".join(f"{v:.9e}" for v in c))
    for name, g in (("exp2-poly", gelu_poly(x, c)), ("A&S 7.1.26", gelu_as(x))):
        err = np.abs(g - r)
        print(f"{name:10s}: max |err| {err.max():.3e} (x = {x[err.argmax()]:.4f}), |x| < 3: {err[np.abs(x) < 3].max():.3e}")


if __name__ == "__main__":
    main()
