"""tools/tune.py against another build of the library (A/B of code changes on one box):
    python tools/tune_with_lib.py tools/bin/libX.so --batch 256 --size 512 --rounds 3"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from codec_tcc_amd import _lib  # noqa: E402

_lib.load(os.path.abspath(sys.argv[1]))
sys.argv = [os.path.join(REPO, "tools", "tune.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
