"""TEST INFRASTRUCTURE ONLY: generates tests/golden/*.json known-answer vectors.

The reference has no tests or fixtures and cannot be compiled here (Ceres
absent, §8c), so parity is pinned by vectors computed independently of both the C
oracle and the HIP kernels: the SnavelyReprojectionError functor
(src/snavely_reprojection_error.hh:39-118) and Ceres' AngleAxisRotatePoint branch
semantics (rotation.h) are written symbolically in sympy, differentiated
symbolically (what forward-mode autodiff computes), and evaluated at 40 significant
digits with mpmath, then rounded to double.

Usage: python oracle/gen_golden.py   (deterministic; rewrites tests/golden/)
"""
import json
import os
import random

import mpmath as mp
import sympy as sp

mp.mp.dps = 40
EPS = 2.220446049250313e-16  # DBL_EPSILON: Ceres' branch threshold on theta^2
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")

X = sp.symbols("X0:3")
W0 = sp.symbols("w0_0:3")
T0 = sp.symbols("t0_0:3")
W1 = sp.symbols("w1_0:3")
T1 = sp.symbols("t1_0:3")
PARAMS = list(X) + list(W0) + list(T0) + list(W1) + list(T1)


def cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def rotate(w, p, big):
    if big:  # Rodrigues, theta^2 > DBL_EPSILON
        th = sp.sqrt(w[0] ** 2 + w[1] ** 2 + w[2] ** 2)
        k = [wi / th for wi in w]
        kx = cross(k, p)
        kp = k[0] * p[0] + k[1] * p[1] + k[2] * p[2]
        return [p[i] * sp.cos(th) + kx[i] * sp.sin(th) + k[i] * kp * (1 - sp.cos(th)) for i in range(3)]
    wx = cross(w, p)  # first-order branch: R = I + [w]x
    return [p[i] + wx[i] for i in range(3)]


def residual_expr(nf, nk, compose, big0, big1, K, obs):
    cx, cy, f0, f1, k0, k1 = K
    if compose:
        P2 = rotate(W1, list(X), big1)
        P2 = [P2[i] + T1[i] for i in range(3)]
        P = rotate(W0, P2, big0)
    else:
        P = rotate(W0, list(X), big0)
    P = [P[i] + T0[i] for i in range(3)]
    xp, yp = P[0] / P[2], P[1] / P[2]
    fx = f0
    fy = f1 if nf == 2 else f0
    r2 = xp * xp + yp * yp
    d = 1
    if nk == 2:
        d = 1 + r2 * (k0 + k1 * r2)
    if nk == 1:
        d = 1 + r2 * k0
    return [fx * d * xp + cx - obs[0], fy * d * yp + cy - obs[1]]


def rand_rot(rng, regime):
    if regime == "big":
        th = rng.uniform(0.05, 2.5)
    elif regime == "near":  # theta^2 just above DBL_EPSILON: Rodrigues branch
        th = (EPS * rng.uniform(1.05, 4.0)) ** 0.5
    elif regime == "small":  # theta^2 <= DBL_EPSILON: first-order branch
        th = (EPS * rng.uniform(0.0, 0.9)) ** 0.5
    else:  # zero rotation
        return [0.0, 0.0, 0.0]
    v = [rng.gauss(0, 1) for _ in range(3)]
    n = sum(x * x for x in v) ** 0.5
    w = [th * x / n for x in v]
    return w


def is_big(w):
    th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2]  # evaluated in double, as Ceres does
    return th2 > EPS


def functor_cases():
    rng = random.Random(20261015)
    cases = []
    cache = {}
    regimes = ["big", "near", "small", "zero"]
    for compose in (False, True):
        for nf in (1, 2):
            for nk in (0, 1, 2):
                for reg in regimes:
                    for rep in range(8 if reg in ("big",) else 5):
                        # camera pose with the point ~1 unit in front
                        w0 = rand_rot(rng, reg)
                        w1 = rand_rot(rng, "big" if rep % 2 == 0 else reg) if compose else [0.0] * 3
                        t0 = [rng.uniform(-0.2, 0.2), rng.uniform(-0.2, 0.2), rng.uniform(0.8, 1.5)]
                        t1 = [rng.uniform(-0.1, 0.1) for _ in range(3)] if compose else [0.0] * 3
                        Xv = [rng.uniform(-0.3, 0.3) for _ in range(3)]
                        if compose and not is_big(w0) and rep % 2 == 1:
                            pass
                        cx = float(int(rng.uniform(400, 1300)))
                        cy = float(int(rng.uniform(400, 1300)))
                        f0 = rng.uniform(500, 5000)
                        f1 = rng.uniform(500, 5000)
                        k0 = rng.uniform(-0.1, 0.1)
                        k1 = rng.uniform(-0.01, 0.01)
                        K = [cx, cy, f0, f1, k0, k1]
                        obs = [rng.uniform(0, 2000), rng.uniform(0, 2000)]
                        big0, big1 = is_big(w0), is_big(w1)
                        key = (nf, nk, compose, big0, big1)
                        Ks = sp.symbols("cx cy f0 f1 k0 k1")
                        Os = sp.symbols("ox oy")
                        if key not in cache:
                            res = residual_expr(nf, nk, compose, big0, big1, Ks, Os)
                            jac = [[sp.diff(ri, v) for v in PARAMS] for ri in res]
                            args = PARAMS + list(Ks) + list(Os)
                            cache[key] = (sp.lambdify(args, res, "mpmath"),
                                          sp.lambdify(args, jac, "mpmath"))
                        fres, fjac = cache[key]
                        vals = [mp.mpf(v) for v in (Xv + w0 + t0 + w1 + t1 + K + obs)]
                        r = [float(v) for v in fres(*vals)]
                        J = [[float(v) for v in row] for row in fjac(*vals)]
                        if not compose:
                            J = [row[:9] + [0.0] * 6 for row in J]
                        cases.append(dict(nf=nf, nk=nk, compose=compose, regime=reg,
                                          X=Xv, ext0=w0 + t0, ext1=(w1 + t1) if compose else None,
                                          intr=K, obs=obs, residual=r, jacobian=J))
    return cases


def rotation_cases():
    rng = random.Random(7)
    out = []
    for i in range(64):
        reg = ["big", "big", "near", "small"][i % 4]
        w = rand_rot(rng, reg)
        if i % 16 == 5:
            w = [0.0, 0.0, 0.0]
        th = mp.sqrt(sum(mp.mpf(x) ** 2 for x in w))
        # exact rotation matrix (column-major like Ceres) and quaternion (w,x,y,z)
        if th > 0:
            k = [mp.mpf(x) / th for x in w]
        else:
            k = [mp.mpf(0)] * 3
        c, s = mp.cos(th), mp.sin(th)
        R = [[c + k[0] ** 2 * (1 - c), k[0] * k[1] * (1 - c) - k[2] * s, k[1] * s + k[0] * k[2] * (1 - c)],
             [k[2] * s + k[0] * k[1] * (1 - c), c + k[1] ** 2 * (1 - c), -k[0] * s + k[1] * k[2] * (1 - c)],
             [-k[1] * s + k[0] * k[2] * (1 - c), k[0] * s + k[1] * k[2] * (1 - c), c + k[2] ** 2 * (1 - c)]]
        R_cm = [float(R[r][cc]) for cc in range(3) for r in range(3)]
        q = [mp.cos(th / 2)] + [kk * mp.sin(th / 2) for kk in k]
        # AngleAxisRotatePoint on a random point, exact for the branch Ceres takes
        p = [rng.uniform(-1, 1) for _ in range(3)]
        if is_big(w):
            Rp = [sum(R[r][cc] * p[cc] for cc in range(3)) for r in range(3)]
        else:
            wx = cross([mp.mpf(x) for x in w], [mp.mpf(x) for x in p])
            Rp = [mp.mpf(p[i]) + wx[i] for i in range(3)]
        out.append(dict(aa=w, R_colmajor=R_cm, quat=[float(x) for x in q], point=p,
                        rotated=[float(x) for x in Rp]))
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    fc = functor_cases()
    with open(os.path.join(OUT, "functor_cases.json"), "w") as f:
        json.dump(dict(source="oracle/gen_golden.py (sympy symbolic derivative, mpmath 40 digits)",
                       reference="src/snavely_reprojection_error.hh:39-118; Ceres rotation.h branch",
                       columns="X(3) | w0(3) t0(3) | w1(3) t1(3)", cases=fc), f, indent=0)
    rc = rotation_cases()
    with open(os.path.join(OUT, "rotation_cases.json"), "w") as f:
        json.dump(dict(source="oracle/gen_golden.py (mpmath 40 digits)",
                       reference="ceres rotation.h: AngleAxisRotatePoint, QuaternionToAngleAxis, "
                                 "RotationMatrixToAngleAxis (DeepArcManager.cc:141-147)",
                       cases=rc), f, indent=0)
    print(f"wrote {len(fc)} functor cases, {len(rc)} rotation cases to {OUT}")


if __name__ == "__main__":
    main()
