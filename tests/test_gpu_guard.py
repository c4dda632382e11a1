"""The device memory-safety net, failing closed (DAB_DEV_GUARD, csrc/dab_devmem.h).

Every device buffer of a handle (problem buffers, set-up scratch, the buffers kept across
set-ups, the Cholesky's scratch, entry-point temporaries) comes from one allocator, which
under DAB_DEV_GUARD=1 puts a zero canary after every block and re-reads them all after each
dab_set_problem / dab_solve / dab_filter / dab_dense_spd_solve: an overwritten canary makes
the call return DAB_E_DEVICE with the block named in dab_last_error. The canaries are a
process-wide mode, so each case runs in a fresh child process:
  * every solver path once under the guard, each call asserting rc 0: the rig's matrix-free
    PCG in fp64 and mixed precision, the rig's exact step (block tiles + dense Cholesky), a
    BAL exact step whose dense Cholesky is large enough for the captured-graph schedule
    (19 blocks) and a BAL PCG, filterPoint3d on the device, the dense SPD solve;
  * the net's self-test (DAB_DEV_GUARD=2 dirties one canary after set-up): the set-up must
    fail with DAB_E_DEVICE naming the overrun block, not return normally."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {root!r})
import _pkgload
pkg = _pkgload.load()
E, P = pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG
def run(prob, lst, f32=0, iters=3):
    s = pkg.Solver(0)
    s.set_problem(prob)
    out = s.solve(pkg.options(max_num_iterations=iters, linear_solver_type=lst, pcg_fp32=f32))
    assert out["num_iterations"] >= 1, out
    return s
rig = pkg.synth(kind=1, num_arcs=6, num_rings=12, num_points=4000, obs_per_point=6, seed=11)
for lst, f32 in ((P, 0), (P, 1), (E, 0)):
    run(rig.copy(), lst, f32).close()
bal = pkg.synth(kind=0, num_cameras=200, num_points=6000, obs_per_point=8, seed=12)
s = run(bal.copy(), E)
ok, pk = s.filter(5.0, [0.0, 0.0, 0.0], 1e6)
assert ok.shape[0] == bal.num_obs
rng = np.random.default_rng(0)
M = rng.standard_normal((300, 300)); A = M @ M.T + 300 * np.eye(300); b = rng.standard_normal(300)
x, ms, good = s.dense_spd_solve(A, b)
assert good and np.linalg.norm(A @ x - b) <= 1e-9 * np.linalg.norm(b)
s.close()
run(bal.copy(), P).close()
print("GUARD OK")
"""

SELFTEST = r"""
import sys
sys.path.insert(0, {root!r})
import _pkgload
pkg = _pkgload.load()
s = pkg.Solver(0)
try:
    s.set_problem(pkg.synth(kind=0, num_cameras=20, num_points=500, obs_per_point=5, seed=5))
except RuntimeError as e:
    print("FAILED CLOSED:", e)
    sys.exit(0)
print("NOT CAUGHT")
sys.exit(3)
"""


def _child(code, mode, timeout=240):
    env = dict(os.environ, DAB_DEV_GUARD=str(mode))
    return subprocess.run([sys.executable, "-c", code.format(root=ROOT)], env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_guarded_solver_paths_rc0(gpu):
    r = _child(CHILD, 1)
    assert r.returncode == 0 and "GUARD OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "dab guard" not in r.stderr, r.stderr[-4000:]


def test_guard_fails_closed_on_overrun(gpu):
    r = _child(SELFTEST, 2)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "FAILED CLOSED" in r.stdout and "overrun" in r.stdout and "problem buffers" in r.stdout, r.stdout


def test_eval_pass_wait_timeout_fails_closed(pkg, gpu, monkeypatch):
    """k_eval_bal's in-launch waits (the camera frames' flag, the point waves' barrier) are
    bounded: a wait that runs out sets the pass's error word and the call fails with
    DAB_E_DEVICE instead of hanging or returning numbers built on missing data.
    DAB_EVAL_SIDE=7 makes the camera waves wait for a frame flag value that never comes."""
    monkeypatch.setenv("DAB_EVAL_SIDE", "7")
    prob = pkg.synth(kind=0, num_cameras=30, num_points=2000, obs_per_point=5, seed=91)
    s = pkg.Solver(0)
    try:
        s.set_problem(prob.copy())
        assert s.eval_fused() == 1
        with pytest.raises(RuntimeError, match="timed out"):
            s.solve(pkg.options(max_num_iterations=2))
        # the failure was reported by that call: the next call starts clean and fails on its
        # own pass again (not on a stale word)
        with pytest.raises(RuntimeError, match="timed out"):
            s.solve(pkg.options(max_num_iterations=2))
    finally:
        s.close()
    # the same handle without the test side solves normally after a re-create
    monkeypatch.delenv("DAB_EVAL_SIDE")
    s = pkg.Solver(0)
    try:
        s.set_problem(prob.copy())
        assert s.solve(pkg.options(max_num_iterations=2))["num_iterations"] >= 1
    finally:
        s.close()


@pytest.mark.parametrize("bad_rank", [0, 1])
def test_eval_pass_wait_timeout_fails_every_rank(gpu, bad_rank):
    """The same bounded wait running out on ONE rank of a sharded solve (the split schedule's
    camera-side launch): its error bits ride in the fixed-point cost words, which every rank
    all-reduces before it reads the pass, so every rank's dab_solve fails with the timeout
    at the same call — no rank goes on into the next collective and hangs."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "dist_check.py"), "--device", "0", "--host-collective",
           "--timeout-rank", str(bad_rank)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "DIST_CHECK OK" in p.stdout, p.stdout[-3000:]


@pytest.mark.parametrize("side", ["1", "2", "3", "4", "5", "6"])
def test_release_library_refuses_eval_ablations(pkg, gpu, monkeypatch, side):
    """DAB_EVAL_SIDE's timing ablations (half a pass, no tables, no frames: wrong sums by
    design) exist only in -DDAB_ABLATIONS builds. With the variable set, the release library
    must either return exactly the unset run's results or fail (it fails: DAB_E_INVALID);
    it may never return rc 0 with wrong numbers."""
    prob = pkg.synth(kind=0, num_cameras=30, num_points=2000, obs_per_point=5, seed=91)
    opts = pkg.options(max_num_iterations=3)
    s = pkg.Solver(0)
    try:
        s.set_problem(prob.copy())
        ref = s.solve(opts)
    finally:
        s.close()
    monkeypatch.setenv("DAB_EVAL_SIDE", side)
    s = pkg.Solver(0)
    try:
        s.set_problem(prob.copy())
        try:
            got = s.solve(opts)
        except RuntimeError as e:
            assert "timing ablation" in str(e), e
        else:
            assert [it["cost"] for it in got["iterations"]] == [it["cost"] for it in ref["iterations"]]
    finally:
        s.close()
