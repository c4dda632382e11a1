"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's host-side semantics.

It is the checker for the host adapter (deeparc-sfm_amd/host, libdeeparc_host.so), and
never the product. It restates:
  * .deeparc reader      DeepArcManager.cc:26-196. Quirks: Q1 principal point truncated
                         to int; Q2 colour truncated to int; rotations given as 3 / 4 / 9
                         numbers go through Ceres' conversions (oracle C library).
  * .deeparc writer      DeepArcManager.cc:426-499 (std::fixed, 6 decimals, points
                         re-indexed, angle-axis out; quirk Q7).
  * PLY writer           DeepArcManager.cc:263-328 (default ostream format = "%g").
  * camera centres       DeepArcManager.cc:242-261, 501-518 (empty when not shared, Q6).
  * filterPoint3d        DeepArcManager.cc:332-424. Quirk Q4: observations with
                         mse < bound are the ones dropped; hemisphere cut |X-c|^2 > R/2.
  * hemisphere fit       sfm.cc:83-101 + hemisphere_radius.hh: r_i = |c - p_i|^2 - R,
                         Ceres TR-LM semantics restated on a dense
                         4x4 system.
  * solve() marshalling  sfm.cc:31-63 + ParameterBlock.hh:68-94, to a dab_problem.
Parity against the reference itself is unpinned: it cannot be built here.
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle  # noqa: E402  (C oracle: rotation conversions, residuals)


def _c_trunc(v):
    """C++ double -> int conversion (toward zero)."""
    return int(math.trunc(v))


def read_deeparc(path):
    toks = open(path).read().split()
    pos = 0

    def nxt(kind):
        nonlocal pos
        t = toks[pos]
        pos += 1
        return int(t) if kind is int else float(t)

    s = {}
    s["version"] = nxt(float)
    nb, ni, na, nr, npnt = (nxt(int) for _ in range(5))
    s["shared"] = nr != 0
    s["arc"], s["ring"] = na, nr
    ne = na + nr - 1 if nr != 0 else na
    s["blocks"] = [[nxt(int), nxt(int), nxt(int), nxt(float), nxt(float)] for _ in range(nb)]
    intr = []
    for _ in range(ni):
        cx, cy = nxt(float), nxt(float)
        nf = nxt(int)
        f = [nxt(float) for _ in range(nf)]
        nk = nxt(int)
        k = [nxt(float) for _ in range(nk)]
        intr.append(dict(center=[float(_c_trunc(cx)), float(_c_trunc(cy))], f=f, k=k))
    s["intr"] = intr
    ext = []
    for _ in range(ne):
        t = [nxt(float), nxt(float), nxt(float)]
        n = nxt(int)
        rot = [nxt(float) for _ in range(n)]
        if n == 9:
            aa = list(oracle.rotmat_to_aa(np.array(rot)))
        elif n == 4:
            aa = list(oracle.quat_to_aa(np.array(rot)))
        else:
            aa = rot
        ext.append(dict(t=t, w=[float(a) for a in aa]))
    s["ext"] = ext
    s["points"] = []
    for _ in range(npnt):
        x, y, z, r, g, b = (nxt(float) for _ in range(6))
        s["points"].append(dict(X=[x, y, z], rgb=[_c_trunc(r), _c_trunc(g), _c_trunc(b)]))
    # block -> point object identity: blocks hold the index into the *current* list
    for b in s["blocks"]:
        b.append(b[2])  # [pos_arc, pos_ring, pid_from_file, x, y, point_index]
    # extrinsic ids as the writer will print them (buildHemisphere relabels ring ids)
    if s["shared"]:
        for a in range(na):
            ext[a]["id"] = a
            for r in range(nr):
                ext[ring_index(r, na)]["id"] = r
    else:
        for i, e in enumerate(ext):
            e["id"] = i
        cams = {}
        for b in s["blocks"]:
            cams.setdefault(b[1], b[0])
        s["cameras"] = sorted(cams.items())  # (extrinsic id, intrinsic id)
    return s


def ring_index(r, arc):
    return 0 if r == 0 else r + arc - 1


def block_extrinsics(s, b):
    """(first, second-or-None) extrinsic indices of a block (ParameterBlock::get())."""
    a, r = b[0], b[1]
    if not s["shared"]:
        return r, None
    if r == 0:
        return a, None
    if a == 0:
        return ring_index(r, s["arc"]), None
    return a, ring_index(r, s["arc"])


def _f6(v):
    return "%.6f" % v


def write_deeparc(s):
    out = ["0.010000\n", "%d %d " % (len(s["blocks"]), len(s["intr"]))]
    out.append("%d %d " % (s["arc"], s["ring"]) if s["shared"] else "%d 0 " % len(s["cameras"]))
    out.append("%d\n" % len(s["points"]))
    for b in s["blocks"]:
        e0, e1 = block_extrinsics(s, b)
        cam = s["ext"][ring_index(b[1], s["arc"])]["id"] if s["shared"] else s["ext"][b[1]]["id"]
        out.append("%d %d %d %s %s\n" % (b[0], cam, b[5], _f6(b[3]), _f6(b[4])))
    for k in s["intr"]:
        line = "%s %s %d" % (_f6(k["center"][0]), _f6(k["center"][1]), len(k["f"]))
        line += "".join(" " + _f6(v) for v in k["f"])
        line += " %d" % len(k["k"]) + "".join(" " + _f6(v) for v in k["k"])
        out.append(line + "\n")
    for e in s["ext"]:
        out.append("%s %s %s 3 %s %s %s\n" % tuple(_f6(v) for v in e["t"] + e["w"]))
    for p in s["points"]:
        out.append("%s %s %s %d %d %d\n" % (tuple(_f6(v) for v in p["X"]) + tuple(p["rgb"])))
    return "".join(out)


def _rotmat(w):
    return np.array(oracle.aa_to_rotmat(np.array(w, float))).reshape(3, 3, order="F")


def _cam_pos(e):
    R = _rotmat(e["w"])
    t = np.array(e["t"])
    return list(-(R.T @ t))


def _cam_pos2(arc, ring):
    R1, R2 = _rotmat(ring["w"]), _rotmat(arc["w"])
    t1, t2 = np.array(ring["t"]), np.array(arc["t"])
    return list(-(R1.T @ t1) - R1.T @ (R2.T @ t2))


def camera_centers(s):
    if not s["shared"]:
        return []
    out = []
    for a in range(s["arc"]):
        for r in range(s["ring"]):
            if r == 0:
                out.append(_cam_pos(s["ext"][a]))
            elif a == 0:
                out.append(_cam_pos(s["ext"][ring_index(r, s["arc"])]))
            else:
                out.append(_cam_pos2(s["ext"][a], s["ext"][ring_index(r, s["arc"])]))
    return out


def write_ply(s):
    ncam = s["arc"] * s["ring"] if s["shared"] else len(s["cameras"])
    out = ["ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
           "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\n"
           "end_header\n" % (len(s["points"]) + ncam)]
    if s["shared"]:
        for a in range(s["arc"]):
            for r in range(s["ring"]):
                if r == 0:
                    c, col = _cam_pos(s["ext"][a]), "0 255 0\n"
                elif a == 0:
                    c, col = _cam_pos(s["ext"][ring_index(r, s["arc"])]), "0 255 0\n"
                else:
                    c, col = _cam_pos2(s["ext"][a], s["ext"][ring_index(r, s["arc"])]), "255 0 255\n"
                out.append("".join("%g " % v for v in c) + col)
    else:
        for eid, _ in s["cameras"]:
            out.append("".join("%g " % v for v in _cam_pos(s["ext"][eid])) + "0 255 0\n")
    for p in s["points"]:
        out.append("".join("%g " % v for v in p["X"]) + "%d %d %d\n" % tuple(p["rgb"]))
    return "".join(out)


def to_problem(pkg, s, freeze_camera=False):
    """The dab_problem of solve() (sfm.cc:31-63): observation o = block o."""
    nb = len(s["blocks"])
    xy = np.array([[b[3], b[4]] for b in s["blocks"]], float).reshape(-1, 2)
    opt = np.array([b[5] for b in s["blocks"]], np.int32)
    e0 = np.zeros(nb, np.int32)
    e1 = np.full(nb, -1, np.int32)
    gauge = np.zeros(len(s["ext"]), np.uint8)
    for o, b in enumerate(s["blocks"]):
        a, c = block_extrinsics(s, b)
        e0[o] = a
        e1[o] = -1 if c is None else c
        if b[0] == 0 and b[1] == 0:
            gauge[a] = 1
    oin = np.array([b[0] for b in s["blocks"]], np.int32)
    pts = np.array([p["X"] for p in s["points"]], float).reshape(-1, 3)
    ext = np.array([e["w"] + e["t"] for e in s["ext"]], float).reshape(-1, 6)
    intr = np.array([[k["center"][0], k["center"][1], k["f"][0], k["f"][1] if len(k["f"]) == 2 else 0.0,
                      k["k"][0] if len(k["k"]) >= 1 else 0.0, k["k"][1] if len(k["k"]) >= 2 else 0.0]
                     for k in s["intr"]], float).reshape(-1, 6)
    nf = np.array([len(k["f"]) for k in s["intr"]], np.int32)
    nk = np.array([len(k["k"]) for k in s["intr"]], np.int32)
    return pkg.Problem(xy, opt, e0, e1, oin, pts, ext, intr, nf, nk, gauge, freeze_camera)


def filter_point3d(pkg, s, error_boundary, center, radius):
    """DeepArcManager.cc:332-424 on the scene dict (in place). Returns the kept block mask."""
    prob = to_problem(pkg, s)
    r, _ = oracle.eval_residuals(pkg, prob) if prob.num_obs else (np.zeros((0, 2)), 0.0)
    keep = [not ((rr[0] * rr[0] + rr[1] * rr[1]) / 2.0 < error_boundary) for rr in r]
    used = [False] * len(s["points"])
    for b, k in zip(s["blocks"], keep):
        if k:
            used[b[5]] = True
    alive = []
    for i, p in enumerate(s["points"]):
        d2 = 0.0
        for k in range(3):
            d = p["X"][k] - center[k]
            d2 += d * d
        alive.append(used[i] and not (d2 > radius / 2))
    keep = [k and alive[b[5]] for b, k in zip(s["blocks"], keep)]
    new_index, pts = {}, []
    for i, p in enumerate(s["points"]):
        if alive[i]:
            new_index[i] = len(pts)
            pts.append(p)
    blocks = []
    for b, k in zip(s["blocks"], keep):
        if k:
            blocks.append(b[:5] + [new_index[b[5]]])
    s["blocks"], s["points"] = blocks, pts
    return keep


def tiny_lm(fun, x, max_iteration=1000):
    """Ceres TR-LM on a small dense problem; fun(x) -> (r, J)."""
    ftol, gtol, ptol, min_rel = 1e-6, 1e-10, 1e-8, 1e-3
    x = np.array(x, float)
    r, J = fun(x)
    cost = 0.5 * float(r @ r)
    s = 1.0 / (1.0 + np.sqrt((J * J).sum(axis=0)))
    def gmax_of(x, J, r):
        g = J.T @ r
        return max((abs(a - (a + (-b))) for a, b in zip(x, g)), default=0.0)
    gmax = gmax_of(x, J, r)
    x_norm = float(np.sqrt(x @ x))
    radius, dec, best, xbest, ok_step, invalid, it = 1e4, 2.0, cost, x.copy(), True, 0, 0
    while True:
        if ok_step and cost < best:
            best, xbest = cost, x.copy()
        if it >= max_iteration or (ok_step and gmax <= gtol) or radius <= 1e-32:
            break
        it += 1
        Js = J * s
        A = Js.T @ Js
        d = np.clip(np.diag(A), 1e-6, 1e32)
        A = A + np.diag(np.sqrt(d / radius) ** 2)
        try:
            L = np.linalg.cholesky(A)
            y = np.linalg.solve(L.T, np.linalg.solve(L, Js.T @ r))
            good = True
        except np.linalg.LinAlgError:
            good = False
        if good:
            delta = -y * s
            m = J @ delta
            model = float(-(m * (r + m / 2.0)).sum())
        if not good or not np.isfinite(model) or not model > 0.0:
            invalid += 1
            if invalid >= 5:
                break
            radius /= dec
            dec *= 2.0
            ok_step = False
            continue
        invalid = 0
        xc = x + delta
        rc, Jc = fun(xc)
        ccost = 0.5 * float(rc @ rc)
        if not np.isfinite(ccost):
            ccost = sys.float_info.max
        if float(np.sqrt(((x - xc) ** 2).sum())) <= ptol * (x_norm + ptol):
            break
        if abs(cost - ccost) <= ftol * cost:
            break
        rho = (cost - ccost) / model
        if rho > min_rel:
            x, r, J, cost = xc, rc, Jc, ccost
            x_norm = float(np.sqrt(x @ x))
            gmax = gmax_of(x, J, r)
            radius = min(1e16, radius / max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3))
            dec, ok_step = 2.0, True
        else:
            radius /= dec
            dec *= 2.0
            ok_step = False
    return xbest


def hemisphere_fit(centers, center=(0.0, 0.0, 0.0), radius=1.0, max_iteration=1000):
    if len(centers) == 0:
        return list(center), radius
    P = np.array(centers, float)

    def fun(x):
        d = x[:3] - P
        r = np.array([((dd[0] * dd[0]) + dd[1] * dd[1]) + dd[2] * dd[2] for dd in d]) - x[3]
        J = np.concatenate([2.0 * d, -np.ones((len(P), 1))], axis=1)
        return r, J

    x = tiny_lm(fun, [center[0], center[1], center[2], radius], max_iteration)
    return list(x[:3]), float(x[3])


def solve_scene(pkg, s, max_iteration=1000, max_second=3600, freeze_camera=False, num_threads=8):
    """solve() (sfm.cc:31-75) on the scene with the C oracle's LM; parameters in place."""
    prob = to_problem(pkg, s, freeze_camera)
    opts = pkg.options(max_num_iterations=max_iteration, max_solver_time_in_seconds=max_second,
                       num_threads=num_threads)
    summ = oracle.solve(pkg, prob, opts)
    for i, p in enumerate(s["points"]):
        p["X"] = [float(v) for v in prob.points[i]]
    for i, e in enumerate(s["ext"]):
        e["w"] = [float(v) for v in prob.ext[i, :3]]
        e["t"] = [float(v) for v in prob.ext[i, 3:]]
    return summ


def run_pipeline(pkg, path, max_iteration=100, error_boundary=5.0, num_threads=8):
    """sfm.cc main() (lines 79-129) without the PLY snapshots; returns (scene, report)."""
    s = read_deeparc(path)
    c, R = hemisphere_fit(camera_centers(s))
    summ = solve_scene(pkg, s, max_iteration, freeze_camera=True, num_threads=num_threads)
    solves, its = 1, summ["num_iterations"]
    filter_point3d(pkg, s, error_boundary, c, R)
    old, cur, step = 1, 10000000, 0
    while cur != old:
        step += 1
        old = cur
        summ = solve_scene(pkg, s, max_iteration, num_threads=num_threads)
        solves, its = solves + 1, its + summ["num_iterations"]
        filter_point3d(pkg, s, error_boundary, c, R)
        cur = len(s["points"])
    return s, dict(hemisphere_center=c, hemisphere_radius=R, rounds=step, blocks=len(s["blocks"]),
                   points=len(s["points"]), solves=solves, lm_iterations=its, final_cost=summ["final_cost"])
