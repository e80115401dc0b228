"""Run bench.py against another build of the library (A/B on one box):
    python tools/bench_with_lib.py tools/bin/libX.so --kind ct12 --steps 10 ..."""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from codec_tcc_amd import _lib  # noqa: E402

_lib.load(os.path.abspath(sys.argv[1]))
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
