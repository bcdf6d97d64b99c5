"""Run pytest against another build of libfdx.so (A/B studies; tools only):
    python tools/pytest_with_lib.py tools/ab/libfdx_X.so tests/test_gpu_parity.py -m gpu -x -q
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)
from fdx import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:]))
