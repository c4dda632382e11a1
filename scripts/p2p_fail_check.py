"""Failure path of the one-shot peer-to-peer all-reduce (dab_p2p.hip): two ranks on one
device (host-staged handles with DAB_P2P=1, the one-GPU rehearsal), a small BAL problem
solved with PCG, so every collective of the LM loop is a peer-to-peer call. Rank 1 skips
one call (DAB_P2P_SKIP_CALL, a test knob read when its handle is created): rank 0's call
times out (DAB_P2P_TIMEOUT_MS), poisons its output instead of summing, and every later call
of either rank fails at once, so BOTH ranks must return DAB_E_COMM from dab_solve with the
caller's points / extrinsics bitwise unchanged (no write-back of a corrupted solve).

Launch: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
        --master-port P scripts/p2p_fail_check.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["DAB_P2P"] = "1"
    os.environ["DAB_P2P_TIMEOUT_MS"] = "3000"
    if rank == 1:
        os.environ["DAB_P2P_SKIP_CALL"] = "20"
    import numpy as np
    import torch
    import torch.distributed as dist

    import _pkgload

    pkg = _pkgload.load()
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def gloo_allreduce(arr, op):
        t = torch.from_numpy(arr)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)

    glob = pkg.synth(kind=0, num_cameras=40, num_points=4000, obs_per_point=6, seed=61)
    mine = glob.copy().shard(rank, world)
    s = pkg.Solver(0, rank, world, b"\0" * 128, host_allreduce=gloo_allreduce)
    s.set_problem(mine)
    assert s.comm_p2p() == 1, "the peer-to-peer all-reduce is not active"
    p0, e0 = mine.points.copy(), mine.ext.copy()
    t = time.perf_counter()
    err = ""
    try:
        s.solve(pkg.options(max_num_iterations=30, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG,
                            function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0))
    except RuntimeError as ex:
        err = str(ex)
    dt = time.perf_counter() - t
    s.close()
    ok = ("libdab error -5" in err and np.array_equal(mine.points, p0) and np.array_equal(mine.ext, e0))
    res = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(res, op=dist.ReduceOp.MIN)
    print(f"rank {rank}: {dt:.1f} s, error {err!r}, arrays unchanged "
          f"{np.array_equal(mine.points, p0) and np.array_equal(mine.ext, e0)}", flush=True)
    dist.barrier()  # every rank's line is out before the verdict (torchrun merges the streams)
    if rank == 0:
        # one write: separate print arguments could interleave with the other rank's line
        sys.stdout.write("P2P_FAIL_CHECK " + ("OK" if int(res.item()) == 1 else "FAIL") + "\n")
        sys.stdout.flush()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
