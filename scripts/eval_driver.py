"""Runs PASSES evaluation passes of CONFIG (knobs from the environment), for profilers.

usage: python scripts/eval_driver.py CONFIG PASSES
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
prob = pkg.synth(**pkg.CONFIGS[sys.argv[1]])
s = pkg.Solver(0)
s.set_problem(prob)
s.bench_eval_pass(True, int(sys.argv[2]))
s.sync()
print("passes done, fused schedule", s.eval_fused())
s.close()
