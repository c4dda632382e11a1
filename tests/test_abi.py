"""C ABI: libdab.so loads, exports every symbol include/dab.h declares, and its host-only
utilities (options defaults, synthetic problems) behave. No compute calls need a GPU here."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "dab.h")).read()
    decl = r"^(?:int|void|const char\*)\s+(dab_[a-z_0-9]+)\s*\("
    return sorted(set(re.findall(decl, src, flags=re.M)))


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.load_library()
    declared = header_symbols()
    assert len(declared) >= 18
    out = subprocess.check_output(["nm", "-D", "--defined-only", pkg.LIB_PATH], text=True)
    exported = set(re.findall(r" T (dab_\w+)", out))
    for name in declared:
        assert name in exported, name
        assert hasattr(lib, name)
    assert set(declared) == set(pkg.SIGNATURES), "ctypes table out of sync with include/dab.h"


def test_options_defaults_match_ceres(pkg):
    o = pkg.options()
    assert o.linear_solver_type == pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR  # DENSE_SCHUR, sfm.cc:67
    assert (o.function_tolerance, o.gradient_tolerance, o.parameter_tolerance) == (1e-6, 1e-10, 1e-8)
    assert o.initial_trust_region_radius == 1e4 and o.max_trust_region_radius == 1e16
    assert (o.min_lm_diagonal, o.max_lm_diagonal) == (1e-6, 1e32)
    assert o.min_relative_decrease == 1e-3 and o.max_num_consecutive_invalid_steps == 5
    assert o.jacobi_scaling == 1 and o.num_threads == 16  # sfm.cc:9,70


def test_synth_deterministic_and_shaped(pkg):
    a = pkg.synth(kind=0, num_cameras=30, num_points=200, obs_per_point=5, seed=9)
    b = pkg.synth(kind=0, num_cameras=30, num_points=200, obs_per_point=5, seed=9)
    for k in ("obs_xy", "obs_point", "obs_ext0", "obs_ext1", "points", "ext", "intr"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))
    assert a.num_obs == 1000 and a.ext.shape == (30, 6) and a.intr.shape == (30, 6)
    assert (a.obs_ext1 == -1).all() and a.ext_const[0] == 1 and a.ext_const[1:].sum() == 0
    # every point observed by distinct cameras
    for p in range(200):
        cams = a.obs_ext0[a.obs_point == p]
        assert len(cams) == 5 and len(set(cams.tolist())) == 5
    # intrinsics: integer principal point (Intrinsic.hh:24-27), |f|=1, |k|=2
    assert (a.intr[:, :2] == np.floor(a.intr[:, :2])).all()
    assert (a.intr_nf == 1).all() and (a.intr_nk == 2).all()


def test_synth_rig_mapping(pkg):
    A, R = 4, 6
    p = pkg.synth(kind=1, num_arcs=A, num_rings=R, num_points=300, obs_per_point=6, seed=4)
    assert p.ext.shape == (A + R - 1, 6) and p.intr.shape == (A, 6)
    # ParameterBlock::get(): ring 0 -> arc only; arc 0 -> ring only; else arc∘ring
    single = p.obs_ext1 < 0
    assert ((p.obs_ext0[~single] < A) & (p.obs_ext1[~single] >= A)).all()
    assert (p.obs_intr == np.where(single & (p.obs_ext0 >= A), 0, p.obs_intr)).all()
    np.testing.assert_array_equal(p.ext[0], np.zeros(6))  # arc[0] = identity (world frame)
    assert (p.intr_nf == 2).all() and (p.intr_nk == 0).all()


def test_synth_rejects_bad_config(pkg):
    lib = pkg.load_library()
    cfg = pkg.synth_config(kind=0, num_cameras=3, num_points=10, obs_per_point=5)
    n = C.c_int32()
    rc = lib.dab_synth_sizes(C.byref(cfg), C.byref(n), None, None, None)
    assert rc == -1 and "bad config" in pkg.last_error()


def test_no_device_fails_loudly(pkg):
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="device"):
        pkg.Solver(0)
