"""Generate the tiny .deeparc round-trip fixtures (TEST INFRASTRUCTURE).

The reference's data files are stripped, so the fixtures are synthetic:
  * tests/golden/tiny_rig.deeparc: a shared-extrinsic rig, 3 arcs x 4 rings;
  * tests/golden/tiny_bal.deeparc: 5 independent cameras.
They exercise every input form the reader accepts: rotations as angle-axis (3),
quaternion (4) and column-major matrix (9); |f| = 1 and 2; |k| = 0, 1 and 2;
fractional principal points (truncated, Q1) and fractional colours (truncated, Q2).
Next to each one the script writes what the reference produces from it, computed with
the oracle restatement (oracle/deeparc_ref.py):
  <name>.expected.deeparc  the output of DeepArcManager::write after read;
  <name>.expected.ply      the output of writePly;
  <name>.expected.json     camera centres, the hemisphere fit and block/point counts.

    python oracle/gen_deeparc_fixtures.py
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def aa_to_quat(w):
    th = math.sqrt(sum(v * v for v in w))
    if th == 0.0:
        return [1.0, 0.0, 0.0, 0.0]
    s = math.sin(th / 2) / th
    return [math.cos(th / 2), w[0] * s, w[1] * s, w[2] * s]


def problem_to_deeparc(prob, shared, n_arc, n_ring, rot_forms, rng, pp_frac=0.5):
    """The .deeparc text of a synthetic Problem (rig: the reference's arc/ring layout)."""
    import oracle

    lines = ["%.6f" % 0.01]
    ne = prob.ext.shape[0]
    ni = prob.intr.shape[0]
    n_cams = n_arc if shared else ne
    lines.append("%d %d %d %d %d" % (prob.num_obs, ni, n_cams, n_ring if shared else 0, prob.points.shape[0]))
    for o in range(prob.num_obs):
        e0, e1, k = int(prob.obs_ext0[o]), int(prob.obs_ext1[o]), int(prob.obs_intr[o])
        if shared:
            a = k
            ring_ext = e1 if e1 >= 0 else (e0 if e0 >= n_arc else -1)
            r = ring_ext - n_arc + 1 if ring_ext >= 0 else 0
        else:
            a, r = k, e0
        lines.append("%d %d %d %.17g %.17g" % (a, r, int(prob.obs_point[o]), prob.obs_xy[o, 0], prob.obs_xy[o, 1]))
    for i in range(ni):
        K = prob.intr[i]
        nf, nk = int(prob.intr_nf[i]), int(prob.intr_nk[i])
        f = [K[2], K[3]][:nf]
        kk = [K[4], K[5]][:nk]
        cx, cy = K[0] + pp_frac, K[1] + pp_frac  # truncated back to K[0], K[1] by the reader
        lines.append("%.17g %.17g %d %s %d %s" % (cx, cy, nf, " ".join("%.17g" % v for v in f), nk,
                                                 " ".join("%.17g" % v for v in kk)))
    for e in range(ne):
        w, t = list(prob.ext[e, :3]), list(prob.ext[e, 3:])
        form = rot_forms[e % len(rot_forms)]
        if form == 4:
            rot = aa_to_quat(w)
        elif form == 9:
            rot = list(oracle.aa_to_rotmat(np.array(w)))
        else:
            rot = w
        lines.append("%.17g %.17g %.17g %d %s" % (t[0], t[1], t[2], len(rot), " ".join("%.17g" % v for v in rot)))
    for p in range(prob.points.shape[0]):
        col = rng.uniform(0, 255.99, 3)
        lines.append("%.17g %.17g %.17g %.3f %.3f %.3f" % (tuple(prob.points[p]) + tuple(col)))
    return "\n".join(lines) + "\n"


def make(pkg, kind, rng):
    if kind == "rig":
        prob = pkg.synth(kind=1, num_arcs=3, num_rings=4, num_points=30, obs_per_point=4, seed=71)
        # |k| and |f| variety on the three arc intrinsics
        prob.intr_nf[:] = [2, 1, 2]
        prob.intr_nk[:] = [0, 1, 2]
        prob.intr[1, 4] = 0.01
        prob.intr[2, 4:6] = [-0.02, 0.003]
        return prob, problem_to_deeparc(prob, True, 3, 4, [3, 4, 9], rng)
    prob = pkg.synth(kind=0, num_cameras=5, num_points=30, obs_per_point=3, seed=72)
    prob.intr_nf[:] = [1, 2, 1, 2, 1]
    prob.intr_nk[:] = [2, 1, 0, 2, 1]
    prob.intr[:, 3] = prob.intr[:, 2] * 1.001  # a distinct f1 where |f| = 2
    return prob, problem_to_deeparc(prob, False, 5, 0, [9, 3, 4], rng)


def expected(path):
    import deeparc_ref as ref

    s = ref.read_deeparc(path)
    centers = ref.camera_centers(s)
    c, R = ref.hemisphere_fit(centers)
    return s, dict(camera_centers=centers, hemisphere_center=c, hemisphere_radius=R,
                   n_blocks=len(s["blocks"]), n_points=len(s["points"]))


def main():
    import _pkgload

    pkg = _pkgload.load()
    rng = np.random.default_rng(7)
    out_dir = os.path.join(ROOT, "tests", "golden")
    import deeparc_ref as ref

    for kind in ("rig", "bal"):
        _, text = make(pkg, kind, rng)
        path = os.path.join(out_dir, "tiny_%s.deeparc" % kind)
        open(path, "w").write(text)
        s, meta = expected(path)
        open(path.replace(".deeparc", ".expected.deeparc"), "w").write(ref.write_deeparc(s))
        open(path.replace(".deeparc", ".expected.ply"), "w").write(ref.write_ply(s))
        json.dump(meta, open(path.replace(".deeparc", ".expected.json"), "w"), indent=1)
        print("wrote", path)


if __name__ == "__main__":
    main()
