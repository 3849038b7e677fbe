"""A/B lab: run bench.py against an experimental build of the library (LAB_LIB=path), e.g.
    LAB_LIB=exp/lib_x.so python scripts/ab_lib.py --steps 20 --warmup 5 --no-cpu"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orleans_amd import _lib as L  # noqa: E402

if os.environ.get("LAB_LIB"):
    L.LIB_PATH = os.path.abspath(os.environ["LAB_LIB"])
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(L.__file__), "..", "bench.py"), run_name="__main__")
