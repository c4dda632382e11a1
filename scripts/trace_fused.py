"""Per-wave timeline of k_eval_bal from the timing build (scripts/trace_build.sh:
s_memrealtime stamps, 100 MHz, at kernel entry / after staging / after the entry loop /
at exit, per work-group and wave). Prints, relative to the earliest entry stamp, the
distribution of each phase boundary over camera and point waves.

usage: python scripts/trace_fused.py CONFIG [side]   (DAB_EVAL_SIDE: 0 both, 1 point side, 2 camera side, ...)
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
abi = sys.modules["deeparc_sfm_amd._abi"]
lib = abi.load_library(os.environ.get("DAB_TRACE_LIB", os.path.join(ROOT, "scripts", "trace", "libdab.so")))
abi._LIB = lib
cfg = sys.argv[1]
side = int(sys.argv[2]) if len(sys.argv) > 2 else 0
os.environ["DAB_EVAL_SIDE"] = str(side)  # k_eval_bal's timing ablation (1 point side, 2 camera side)
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
s.set_problem(prob)
s.bench_eval_pass(True, 20)
s.sync()
s.bench_kernel_ms()
s.bench_eval_pass(True, 50)
s.sync()
jk, _ = s.bench_kernel_ms()
print(f"{cfg} abl={side} lib={os.path.basename(os.path.dirname(lib._name))}: kernel {jk * 1e3:.1f} us (50-pass average)")
buf = np.zeros(256 * 16 * 8, dtype=np.uint64)
runs = []
for rep in range(5):
    lib.dab_trace_clear()
    s.bench_eval_pass(True, 1)
    s.sync()
    lib.dab_trace_fetch(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)))
    runs.append(buf.reshape(256, 16, 8).astype(np.int64).copy())
s.close()
for r, t in enumerate(runs):
    have = t[:, :, 0] > 0
    t0 = t[:, :, 0][have].min()
    rel = np.where(t > 0, (t - t0) * 0.01, np.nan)  # us
    print(f"{cfg} side={side} run {r}: work-groups with stamps {int(have.any(axis=1).sum())}")
    for name, ws in (("point", slice(0, 8)), ("camera", slice(8, 16))):
        x = rel[:, ws, :]
        if np.isnan(x[:, :, 0]).all():
            continue
        q = lambda a: " ".join(f"{v:6.2f}" for v in np.nanpercentile(a, [0, 10, 50, 90, 100]))
        print(f"  {name:6s} entry   {q(x[:, :, 0])}")
        print(f"  {name:6s} staged  {q(x[:, :, 1])}")
        print(f"  {name:6s} loopend {q(x[:, :, 2])}")
        print(f"  {name:6s} exit    {q(x[:, :, 3])}")
        print(f"  {name:6s} loop    {q(x[:, :, 2] - x[:, :, 1])}   (per wave, percentiles 0/10/50/90/100)")
if os.environ.get("DAB_TRACE_PER_WAVE"):
    t = runs[-1]
    have = t[:, :, 0] > 0
    t0 = t[:, :, 0][have].min()
    rel = np.where(t > 0, (t - t0) * 0.01, np.nan)
    print("per logical wave: median staged / loop end / exit (us)")
    for w in range(16):
        print(f"  wave {w:2d}: " + " ".join(f"{np.nanmedian(rel[:, w, k]):6.2f}" for k in (1, 2, 3)))
if os.environ.get("DAB_TRACE_PER_WG"):
    # the tail: which work-groups end last, and does their lateness come from a late start
    # (dispatch) or from a slow run? Per work-group: first entry, last exit, by XCD (b % 8)
    t = runs[-1]
    have = t[:, :, 0] > 0
    t0 = t[:, :, 0][have].min()
    rel = np.where(t > 0, (t - t0) * 0.01, np.nan)
    ent = np.nanmin(rel[:, :, 0], axis=1)
    ext_ = np.nanmax(rel[:, :, 3], axis=1)
    dur = ext_ - ent
    print("per work-group: entry / exit / duration percentiles 0/10/50/90/100 (us)")
    for name, a in (("entry", ent), ("exit", ext_), ("duration", dur)):
        print(f"  {name:8s} " + " ".join(f"{v:6.2f}" for v in np.nanpercentile(a, [0, 10, 50, 90, 100])))
    print(f"  corr(entry, exit) {np.corrcoef(ent[have.any(axis=1)], ext_[have.any(axis=1)])[0, 1]:.2f}")
    for x in range(8):
        sel = np.arange(256) % 8 == x
        print(f"  XCD {x}: entry median {np.nanmedian(ent[sel]):5.2f}  exit median {np.nanmedian(ext_[sel]):5.2f}  "
              f"max {np.nanmax(ext_[sel]):5.2f}")
    last = np.argsort(-np.nan_to_num(ext_, nan=-1))[:12]
    print("  last 12 work-groups (block: entry exit):", " ".join(f"{b}:{ent[b]:.1f}/{ext_[b]:.1f}" for b in last))
    # prologue hops (stamps 4-6 of the camera waves: chunk bounds, first indices, first
    # points, each once every load in flight has returned; stamp 5 of the point waves:
    # their tables built, before the barrier)
    print("prologue (median over waves, us): entry / first barrier:",
          " ".join(f"{np.nanmedian(rel[:, :, k]):6.2f}" for k in (0, 7)),
          "| camera bounds / indices / points / frame:",
          " ".join(f"{np.nanmedian(rel[:, 8:, k]):6.2f}" for k in (4, 5, 6, 1)),
          "| point tables built / barrier passed:", " ".join(f"{np.nanmedian(rel[:, :8, k]):6.2f}" for k in (5, 1)))
if os.environ.get("DAB_TRACE_PER_WAVE") and hasattr(lib, "dab_trace_hwid"):
    hw = np.zeros(256 * 16, dtype=np.uint32)
    lib.dab_trace_hwid(hw.ctypes.data_as(C.POINTER(C.c_uint)))
    hw = hw.reshape(256, 16)
    simd = (hw >> 4) & 3
    print("SIMD of each logical wave relative to wave 0's, (s_w - s_0) mod 4 (most common over the "
          "work-groups; share):")
    for w in range(16):
        vals, cnt = np.unique((simd[:, w] - simd[:, 0]) % 4, return_counts=True)
        print(f"  wave {w:2d}: {vals[cnt.argmax()]} ({cnt.max() / cnt.sum():.2f})")
