"""Run a script against another build of libfdx.so (A/B studies; tools only):
    python tools/with_lib.py tools/ab/libfdx_X.so bench.py --steps 5 ...
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)
from fdx import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
_probe = __import__("ctypes").CDLL(_lib.LIB_PATH)
for _name in [k for k in _lib.SIGNATURES if not hasattr(_probe, k)]:  # an older build: symbols it lacks
    del _lib.SIGNATURES[_name]
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
