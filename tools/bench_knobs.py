"""Run bench.py in this process after setting library A/B knobs, so two settings can be compared on one box.
Usage: python tools/bench_knobs.py dq_store=<0|1|2> c_store=<0|1> -- [bench.py args]"""
import ctypes as ct
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
from python_src_quants.cextension import lib  # noqa: E402

knobs = {"dq_store": lib.cdequantize_set_store_policy, "c_store": lib.chgemm_set_c_store}
argv = sys.argv[1:]
rest = argv[argv.index("--") + 1:] if "--" in argv else []
for a in (argv[:argv.index("--")] if "--" in argv else argv):
    k, v = a.split("=")
    knobs[k](ct.c_int(int(v)))
sys.argv = [os.path.join(ROOT, "bench.py")] + rest
runpy.run_path(sys.argv[0], run_name="__main__")
