"""Sharded multi-rank path on the GPU: two ranks on one device, the library's collectives
staged through gloo (dab_create_dist_host; RCCL refuses two ranks per GPU). Each rank
solves its point shard; the LM trajectories (explicit Schur and PCG, BAL and rig) must
match the single-handle solve of the global problem (costs 1e-8 relative, parameters 1e-6)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_match_single_handle(gpu):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "dist_check.py"), "--device", "0", "--host-collective"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "DIST_CHECK OK" in p.stdout, p.stdout[-3000:]


def test_two_ranks_p2p_allreduce_match_single_handle(gpu):
    """The one-shot peer-to-peer all-reduce (dab_p2p.hip: IPC-mapped peer regions, flags,
    fixed rank-order sums) on the one-GPU rehearsal: two processes on one device map each
    other's regions (DAB_P2P=1 enables it on host-staged handles), so every camera-sized sum
    of the sharded solve (camera blocks on the communication stream beside the point side,
    PCG products, Schur-Jacobi blocks, fixed-point cost words) goes through the kernel,
    the rest through gloo. Same trajectories as the single handle."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DAB_P2P="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "dist_check.py"), "--device", "0", "--host-collective", "--expect-p2p"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "DIST_CHECK OK" in p.stdout, p.stdout[-3000:]


@pytest.mark.parametrize("live", [False, True])
def test_four_ranks_p2p_six_groups(gpu, live):
    """Four processes, six handles each (BAL and rig x three solver types), every one with
    its own peer-to-peer group: in sequence, or three alive at once per problem (bench.py
    holds two at once on several ranks). Groups take slots of a per-process arena exported
    once: re-exporting a fresh region per group let importers resolve the new handle to the
    peer's freed one (the self-test failed from the third group on and the freed memory was
    written). Every group must verify and match the single handle."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DAB_P2P="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "dist_check.py"), "--device", "0", "--host-collective", "--expect-p2p",
           "--iters", "6"] + (["--live-together"] if live else [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "DIST_CHECK OK" in p.stdout, p.stdout[-3000:]
    assert "not verified" not in p.stderr, p.stderr[-3000:]


def test_rccl_one_rank_per_gpu(gpu):
    """The product multi-GPU path: one process per GPU, dab_create_dist (RCCL over xGMI),
    every collective on RCCL. Runs whenever the box shows two or more devices (the driver's
    8-GPU node); a one-GPU box skips it (RCCL refuses two ranks per device)."""
    import torch
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip(f"{n} device(s) visible: the RCCL path needs two")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "scripts", "dist_check.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "DIST_CHECK OK" in p.stdout, p.stdout[-3000:]


def test_p2p_missed_call_fails_closed(gpu):
    """A peer that misses one peer-to-peer all-reduce (DAB_P2P_SKIP_CALL on rank 1) must not
    leave the other rank summing stale slots: the waiting call times out (3 s here), writes
    poison instead of a sum, every later call fails at once, and BOTH ranks' dab_solve
    return DAB_E_COMM with the caller's parameter arrays untouched (scripts/p2p_fail_check.py)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "p2p_fail_check.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "P2P_FAIL_CHECK OK" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]


def test_p2p_selftest_failure_falls_back(gpu):
    """The peer-to-peer path is trusted only after a verified exchange at set-up (two exact
    integer sums per context). A rank that contributes a wrong word (DAB_P2P_SELFTEST_SKEW)
    makes every rank's check fail; all ranks then agree to keep the other collectives
    (here the host-staged ones), report p2p = 0, and the sharded trajectories still match
    the single handle."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DAB_P2P="1", DAB_P2P_SELFTEST_SKEW="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "dist_check.py"), "--device", "0", "--host-collective", "--expect-no-p2p",
           "--config", "c2_100cam", "--iters", "4"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "DIST_CHECK OK" in p.stdout, p.stdout[-3000:]
