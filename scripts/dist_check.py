"""Multi-rank check of the RCCL path on whatever GPUs the box has.

Launch: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
        --master-port P scripts/dist_check.py [--device D]
Every rank solves its point shard of one global problem through dab_create_dist; rank 0
also solves the global problem on one handle and compares the LM trajectories (explicit
Schur and PCG). With --device D every rank uses device D (ranks sharing one GPU; RCCL
refuses that, so pair it with --host-collective, which stages the library's collectives
through gloo and exercises every other part of the sharded path).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=-1)
    ap.add_argument("--host-collective", action="store_true",
                    help="stage the library's all-reduces through gloo (ranks sharing a GPU)")
    ap.add_argument("--config", default="", help="a named configuration (core.CONFIGS) instead of "
                    "the small BAL and rig problems, e.g. c3_1kcam: BASELINE config 4's partition")
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--expect-p2p", action="store_true",
                    help="fail unless the one-shot peer-to-peer all-reduce carried the sums")
    ap.add_argument("--live-together", action="store_true",
                    help="keep the three sharded handles of a problem alive at once (bench.py holds two: "
                    "each takes its own slot of the peer-to-peer arena)")
    ap.add_argument("--expect-no-p2p", action="store_true",
                    help="fail if the peer-to-peer path is in use (its set-up self-test must have "
                    "failed over to the other collectives)")
    ap.add_argument("--solvers", default="explicit,pcg,auto",
                    help="comma list of the linear solvers to check (explicit, pcg, auto)")
    ap.add_argument("--tol", type=float, default=1e-8,
                    help="largest relative per-iteration cost difference against the single handle")
    ap.add_argument("--expect-cg-equal", action="store_true",
                    help="fail unless every iteration's CG count equals the single handle's")
    ap.add_argument("--expect-auto", default="",
                    help="fail unless AUTO ran this solver on the ranks (explicit | pcg)")
    ap.add_argument("--timeout-rank", type=int, default=-1,
                    help="this rank's evaluation pass runs a frame wait that never completes "
                    "(DAB_EVAL_SIDE=7): every rank's dab_solve must fail with the timeout, none may hang")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = a.device if a.device >= 0 else int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    import _pkgload

    pkg = _pkgload.load()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        buf[:] = torch.tensor(list(pkg.Solver.unique_id()), dtype=torch.uint8)
    dist.broadcast(buf, 0)
    uid = bytes(buf.tolist())
    def gloo_allreduce(arr, op):
        t = torch.from_numpy(arr)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)

    if a.timeout_rank >= 0:
        # one rank's pass times out inside the launch; its error word travels with the cost's
        # all-reduce, so every rank must fail the same call (DAB_E_DEVICE), none may hang
        if rank == a.timeout_rank:
            os.environ["DAB_EVAL_SIDE"] = "7"  # read when the handle is created
        glob = pkg.synth(**pkg.CONFIGS[a.config]) if a.config else \
            pkg.synth(kind=0, num_cameras=40, num_points=4000, obs_per_point=6, seed=61)
        s = pkg.Solver(dev, rank, world, uid, host_allreduce=gloo_allreduce if a.host_collective else None)
        msg = ""
        try:
            s.set_problem(glob.copy().shard(rank, world))
            sched = s.eval_fused()
            s.solve(pkg.options(max_num_iterations=3))
        except RuntimeError as e:
            msg = str(e)
        finally:
            s.close()
        failed = torch.tensor([1 if "timed out" in msg else 0], dtype=torch.int32)
        dist.all_reduce(failed)
        if rank == 0:
            ok = int(failed.item()) == world and sched == 2
            sys.stdout.write(f"DIST_CHECK {'OK' if ok else 'FAIL'} timeout: {int(failed.item())}/{world} ranks "
                             f"failed closed, eval schedule {sched}, rank 0: {msg!r}\n")
            sys.stdout.flush()
        dist.destroy_process_group()
        return

    names = {"explicit": pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, "pcg": pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG,
             "auto": pkg.DAB_LINEAR_SOLVER_AUTO}
    solvers = [names[x] for x in a.solvers.split(",")]
    out = {}
    for kind in ((a.config,) if a.config else ("bal", "rig")):
        if kind == "bal":
            glob = pkg.synth(kind=0, num_cameras=40, num_points=4000, obs_per_point=6, seed=61)
        elif kind == "rig":
            glob = pkg.synth(kind=1, num_arcs=5, num_rings=12, num_points=3000, obs_per_point=7, seed=62)
        else:
            glob = pkg.synth(**pkg.CONFIGS[kind])
        owner = glob.point_owner(world)
        live = []
        if a.live_together:  # every handle of this problem created (and its arena slot taken) up front
            for _ in range(3):
                h = pkg.Solver(dev, rank, world, uid, host_allreduce=gloo_allreduce if a.host_collective else None)
                live.append(h)
        for li, lst in enumerate(solvers):
            opts = pkg.options(max_num_iterations=a.iters, linear_solver_type=lst)
            ref = None
            if rank == 0:
                g1 = glob.copy()
                s1 = pkg.Solver(dev)
                s1.set_problem(g1)
                ropts = opts
                if lst == pkg.DAB_LINEAR_SOLVER_AUTO:
                    # what AUTO must pick on several ranks: the exact step for small camera
                    # systems (the rig), PCG for large ones (BAL / config 4)
                    want = (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR if glob.ext.shape[0] <= 160
                            else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
                    ropts = pkg.options(max_num_iterations=a.iters, linear_solver_type=want)
                ref = (s1.solve(ropts), g1.points.copy(), g1.ext.copy())
                s1.close()
            dist.barrier()
            mine = glob.copy().shard(rank, world)
            s = live[li] if live else pkg.Solver(dev, rank, world, uid,
                                                 host_allreduce=gloo_allreduce if a.host_collective else None)
            s.set_problem(mine)
            sched = s.eval_fused()
            p2p = s.comm_p2p()
            summ = s.solve(opts)
            if not live:
                s.close()
            pts = torch.from_numpy(np.where((owner == rank)[:, None], mine.points, 0.0))
            dist.all_reduce(pts)
            ext = torch.from_numpy(mine.ext.copy())
            dist.all_reduce(ext, op=dist.ReduceOp.MAX)
            ext_min = torch.from_numpy(mine.ext.copy())
            dist.all_reduce(ext_min, op=dist.ReduceOp.MIN)
            if rank == 0:
                rs, rp, re = ref
                ca = [it["cost"] for it in summ["iterations"]]
                cb = [it["cost"] for it in rs["iterations"]]
                n = min(len(ca), len(cb))
                out[f"{kind}_{lst}"] = dict(
                    iters=(summ["num_iterations"], rs["num_iterations"]),
                    term=(summ["termination"], rs["termination"]),
                    max_rel_cost=float(max(abs(x - y) / abs(y) for x, y in zip(ca[:n], cb[:n]))),
                    cg_equal=[it["linear_solver_iterations"] for it in summ["iterations"]]
                    == [it["linear_solver_iterations"] for it in rs["iterations"]],
                    final=(summ["final_cost"], rs["final_cost"]),
                    dpts=float(np.abs(pts.numpy() - rp).max()),
                    dext=float(np.abs(ext.numpy() - re).max()),
                    ext_ranks_equal=bool(torch.equal(ext, ext_min)),
                    eval_schedule=sched, p2p=p2p,
                    solver_used=(summ["linear_solver_type_used"], rs["linear_solver_type_used"]))
        for h in live:
            h.close()
    if rank == 0:
        print(json.dumps(out, indent=1))
        auto_want = names.get(a.expect_auto, None)
        bad = [k for k, v in out.items()
               if v["iters"][0] != v["iters"][1] or v["max_rel_cost"] > a.tol or v["dpts"] > 1e-6
               or (a.expect_cg_equal and not v["cg_equal"])
               or (auto_want is not None and k.endswith(f"_{pkg.DAB_LINEAR_SOLVER_AUTO}")
                   and v["solver_used"][0] != auto_want)
               or v["dext"] > 1e-6 or not v["ext_ranks_equal"]
               or (not k.startswith("rig") and v["eval_schedule"] != 2)  # BAL shards: the split fused pass
               or (a.expect_p2p and v["p2p"] != 1)
               or (a.expect_no_p2p and v["p2p"] != 0)
               or v["solver_used"][0] != v["solver_used"][1]]
        sys.stdout.write("DIST_CHECK " + ("FAIL " + ",".join(bad) if bad else "OK") + "\n")  # one write
        sys.stdout.flush()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
