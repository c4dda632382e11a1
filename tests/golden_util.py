"""Helpers to turn tests/golden/ fixtures into dab problems."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def functor_cases():
    with open(os.path.join(GOLDEN, "functor_cases.json")) as f:
        return json.load(f)["cases"]


def rotation_cases():
    with open(os.path.join(GOLDEN, "rotation_cases.json")) as f:
        return json.load(f)["cases"]


def cases_problem(pkg, cases):
    """All functor cases as one problem: one point/extrinsic pair/intrinsic per case."""
    n = len(cases)
    obs = np.array([c["obs"] for c in cases], float)
    pts = np.array([c["X"] for c in cases], float)
    ext, e0, e1 = [], [], []
    for c in cases:
        e0.append(len(ext))
        ext.append(c["ext0"])
        if c["compose"]:
            e1.append(len(ext))
            ext.append(c["ext1"])
        else:
            e1.append(-1)
    intr = np.array([c["intr"] for c in cases], float)
    return pkg.Problem(obs, np.arange(n), e0, e1, np.arange(n), pts, np.array(ext, float), intr,
                       [c["nf"] for c in cases], [c["nk"] for c in cases])


def golden_arrays(cases):
    r = np.array([c["residual"] for c in cases], float)
    J = np.array([c["jacobian"] for c in cases], float)
    return r, J


# Tolerances (stated, fp64). Residuals: relative to max(1, |r|). Jacobians: relative to the
# largest entry of the case's Jacobian. Near Ceres' small-angle branch (theta^2 just above
# DBL_EPSILON) forward-mode autodiff through w = aa/theta loses ~8 digits (measured 9e-10);
# the closed-form HIP Jacobian does not, so it is held to the tight bound everywhere.
TOL_RES = 1e-12
TOL_JAC = 1e-11
TOL_JAC_AUTODIFF_NEAR = 1e-7
