"""Coefficients of the compositors' reproducible exp (lsr_common.h expf_repro, oracle orc_exp):
e^r ~ 1 + r (1 + r (c2 + r (c3 + r (c4 + r c5)))) on [-ln2/2, ln2/2], minimax in relative error
(LP on a dense grid, scipy), rounded to float32; then the float32 pipeline
  y = fma(x, log2 e, 1.5 2^23); k = y - 1.5 2^23; r = fma(k, -ln2_f, x); p = Horner; p * 2^k
is measured in ulp against float64 exp over x in [-87, 0] (fma emulated in float64: the product
of two floats is exact there).  Usage: python tools/exp_minimax.py"""
import numpy as np
from scipy.optimize import linprog

h = np.log(2.0) / 2
r = np.linspace(-h, h, 4001)
deg = 5
free = list(range(2, deg + 1))
# variables: c2..c5, t ; minimise t s.t. |(1 + r + sum c_k r^k) / e^r - 1| <= t
A, b = [], []
for ri in r:
    e = np.exp(ri)
    row = [ri ** k / e for k in free]
    base = (1 + ri) / e - 1
    A.append(row + [-1.0]); b.append(-base)
    A.append([-v for v in row] + [-1.0]); b.append(base)
res = linprog(np.r_[np.zeros(len(free)), 1.0], A_ub=np.array(A), b_ub=np.array(b),
              bounds=[(None, None)] * len(free) + [(0, None)], method="highs")
c = np.float32(res.x[:-1])
print("model max rel err", res.x[-1])
print("coefficients c2..c5 (float32):", [repr(float(v)) for v in c])

f32 = np.float32
LOG2E, MAGIC, LN2 = f32(1.44269504088896341), f32(12582912.0), f32(np.log(2.0))


def fma(a, b, cc):
    return f32(np.float64(a) * np.float64(b) + np.float64(cc))


def expf(x):
    x = np.maximum(f32(x), f32(-87.0))
    y = fma(x, LOG2E, MAGIC)
    k = f32(y - MAGIC)
    rr = fma(k, -LN2, x)
    p = f32(c[-1])
    for ck in c[-2::-1]:
        p = fma(p, rr, ck)
    p = fma(p, rr, f32(1.0))
    p = fma(p, rr, f32(1.0))
    sc = (y.view(np.uint32) << np.uint32(23)) + np.uint32(0x3F800000)
    return f32(p * sc.view(np.float32))


xs = np.concatenate([-np.random.default_rng(0).uniform(0, 87, 2_000_000), -np.linspace(0, 6, 200_001)]).astype(f32)
got = expf(xs).astype(np.float64)
ref = np.exp(xs.astype(np.float64))
ulp = np.spacing(ref.astype(f32)).astype(np.float64)
err = np.abs(got - ref) / ulp
print("max ulp over [-87, 0]:", err.max(), " over [-6, 0]:", err[xs > -6].max())


def expf_cw2(x):   # the same with the two-constant Cody-Waite reduction (the kernels' current one)
    x = np.maximum(f32(x), f32(-87.0))
    y = fma(x, LOG2E, MAGIC)
    k = f32(y - MAGIC)
    rr = fma(k, f32(-0.693145751953125), x)
    rr = fma(k, f32(-1.428606765330187045e-06), rr)
    p = f32(c[-1])
    for ck in c[-2::-1]:
        p = fma(p, rr, ck)
    p = fma(p, rr, f32(1.0))
    p = fma(p, rr, f32(1.0))
    sc = (y.view(np.uint32) << np.uint32(23)) + np.uint32(0x3F800000)
    return f32(p * sc.view(np.float32))


err2 = np.abs(expf_cw2(xs).astype(np.float64) - ref) / ulp
print("two-constant reduction: max ulp over [-87, 0]:", err2.max(), " over [-6, 0]:", err2[xs > -6].max())
