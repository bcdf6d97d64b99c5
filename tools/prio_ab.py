"""Run a script with torch's current stream replaced by a stream of the given priority
(stream-priority A/B for the pipeline's caller stream; tools only):
    python tools/prio_ab.py -1 bench.py --steps 10 ...
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

prio = int(sys.argv[1])
sys.argv = sys.argv[2:]
with torch.cuda.stream(torch.cuda.Stream(priority=prio)):
    runpy.run_path(sys.argv[0], run_name="__main__")
