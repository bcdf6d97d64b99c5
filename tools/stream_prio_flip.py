"""Run bench.py with run_fused's stream priorities overridden (A/B; tools only):
    python tools/stream_prio_flip.py CRIT SIDE bench.py --steps 10 ...
CRIT = the customer half / assembly / forest stream, SIDE = the terminal half (lower = higher).
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)
from fdx.pipeline import FraudPipeline  # noqa: E402

FraudPipeline.crit_priority = int(sys.argv[1])
FraudPipeline.side_priority = int(sys.argv[2])
sys.argv = sys.argv[3:]
runpy.run_path(sys.argv[0], run_name="__main__")
