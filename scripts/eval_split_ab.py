"""The evaluation pass at C3 on the split schedule (DAB_EVAL_SPLIT=1 set by the caller):
64 passes through dab_bench_eval_pass, for a kernel trace; DAB_LIB selects another build of
libdab (an A/B of two libraries under the same command)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
if os.environ.get("DAB_LIB"):
    abi = sys.modules[pkg.__name__ + "._abi"]
    abi._LIB = abi.load_library(os.path.join(ROOT, os.environ["DAB_LIB"]))
prob = pkg.synth(**pkg.CONFIGS["c3_1kcam"])
s = pkg.Solver(0)
s.set_problem(prob)
print("eval schedule", s.eval_fused())
s.bench_eval_pass(True, 8)
s.sync()
s.bench_eval_pass(True, 64)
s.sync()
print("kernel ms", s.bench_kernel_ms())
s.close()
