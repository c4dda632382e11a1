"""N > 1 path on the CPU: world_size-2 gloo processes.

The library shards by point (Problem.shard / point_owner) and relies on two facts:
every per-point quantity (V, g_p, the Schur factor, the back-substitution) is local to
the owning rank, and every camera-side quantity (cost, g_c, the U / cross blocks, the
Schur rhs and the PCG operator's Y part) is a plain sum of per-shard contributions that
one all-reduce combines. Each rank evaluates its shard with the CPU oracle; the
all-reduced camera terms and the gathered point terms must equal the single-process
evaluation of the global problem. The gauge (ext_const) is decided on the global
problem before sharding, as sfm.cc:50-53 does per block.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _terms(prob, r, J):
    """cost, g over (points | ext) and the dense camera Gram block from J [N][2][15]."""
    npt, ne = prob.points.shape[0], prob.ext.shape[0]
    gp = np.zeros((npt, 3))
    ge = np.zeros((ne, 6))
    U = np.zeros((6 * ne, 6 * ne))
    np.add.at(gp, prob.obs_point, np.einsum("nrk,nr->nk", J[:, :, 0:3], r))
    np.add.at(ge, prob.obs_ext0, np.einsum("nrk,nr->nk", J[:, :, 3:9], r))
    comp = prob.obs_ext1 >= 0
    np.add.at(ge, prob.obs_ext1[comp], np.einsum("nrk,nr->nk", J[comp][:, :, 9:15], r[comp]))
    cols = [(prob.obs_ext0, J[:, :, 3:9], np.ones(len(r), bool)),
            (prob.obs_ext1, J[:, :, 9:15], comp)]
    for ea, Ja, ma in cols:
        for eb, Jb, mb in cols:
            m = ma & mb
            for o in np.nonzero(m)[0]:
                a, b = ea[o], eb[o]
                U[6 * a:6 * a + 6, 6 * b:6 * b + 6] += Ja[o].T @ Jb[o]
    return 0.5 * float((r * r).sum()), gp, ge, U


def _worker(rank, world, port, out_q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import _pkgload
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = _pkgload.load()
        prob = pkg.synth(kind=1, num_arcs=3, num_rings=5, num_points=300, obs_per_point=5, seed=51)
        owner = prob.point_owner(world)
        sh = prob.shard(rank, world)
        r, J = oracle.eval_jacobians(pkg, sh, 1)
        cost, gp, ge, U = _terms(sh, r, J)
        # camera side: one all-reduce (sum); point side: owner-local, gathered by sum
        cam = torch.from_numpy(np.concatenate([[cost], ge.ravel(), U.ravel()]))
        dist.all_reduce(cam)
        mine = owner == rank
        gp_local = np.where(mine[:, None], gp, 0.0)
        pts = torch.from_numpy(gp_local.copy())
        dist.all_reduce(pts)
        # every shard's observations belong to points it owns, and the shards cover all
        nobs = torch.tensor([sh.num_obs], dtype=torch.int64)
        dist.all_reduce(nobs)
        touched = np.zeros(prob.points.shape[0], bool)
        touched[sh.obs_point] = True
        ok_local = bool(np.all(owner[sh.obs_point] == rank)) and not np.any(touched & ~mine)
        flag = torch.tensor([0 if ok_local else 1])
        dist.all_reduce(flag)
        if rank == 0:
            rf, Jf = oracle.eval_jacobians(pkg, prob, 1)
            cf, gpf, gef, Uf = _terms(prob, rf, Jf)
            c = cam.numpy()
            ne = prob.ext.shape[0]
            out_q.put(dict(
                cost=(c[0], cf), ge=float(np.abs(c[1:1 + 6 * ne] - gef.ravel()).max()),
                ge_scale=float(np.abs(gef).max()),
                U=float(np.abs(c[1 + 6 * ne:] - Uf.ravel()).max()), U_scale=float(np.abs(Uf).max()),
                gp=float(np.abs(pts.numpy() - gpf).max()), gp_scale=float(np.abs(gpf).max()),
                nobs=(int(nobs.item()), prob.num_obs), partition_ok=int(flag.item()) == 0,
                balance=[int((owner[prob.obs_point] == k).sum()) for k in range(world)]))
    finally:
        dist.destroy_process_group()


def test_point_sharded_terms_sum_to_global():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(k, world, port, q)) for k in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res["partition_ok"]
    assert res["nobs"][0] == res["nobs"][1]
    b = res["balance"]
    assert abs(b[0] - b[1]) <= 0.05 * sum(b)
    assert res["cost"][0] == pytest.approx(res["cost"][1], rel=1e-13)
    assert res["ge"] <= 1e-12 * res["ge_scale"]
    assert res["U"] <= 1e-12 * res["U_scale"]
    assert res["gp"] <= 1e-14 * res["gp_scale"]


def test_point_owner_contiguous_and_balanced(pkg):
    prob = pkg.synth(kind=0, num_cameras=20, num_points=1000, obs_per_point=6, seed=52)
    for world in (1, 2, 3, 8):
        own = prob.point_owner(world)
        assert own.min() == 0 and own.max() == world - 1
        assert np.all(np.diff(own) >= 0)  # contiguous point ranges
        cnt = np.bincount(own[prob.obs_point], minlength=world)
        assert cnt.sum() == prob.num_obs
        assert cnt.max() - cnt.min() <= 2 * 6
        shards = [prob.shard(k, world) for k in range(world)]
        assert sum(s.num_obs for s in shards) == prob.num_obs
