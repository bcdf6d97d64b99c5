"""Time fdx_forest_prepare alone (configs[2] rows: the bench model's check rows resampled to
--rows, float64 [n, 15] resident) -- prepare-kernel A/B studies (tools only):
    python tools/with_lib.py tools/ab/libfdx_X.so tools/prepare_ab.py --rows 100000000
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
from fdx import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
arr = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
       for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
dev = torch.device("cuda:0")
f = ops.Forest(arr, 15, z["mean"], z["scale"])
g = torch.Generator(device=dev)
g.manual_seed(20240601)
idx = torch.randint(0, len(z["check_X"]), (args.rows,), device=dev, generator=g)
X = torch.from_numpy(z["check_X"]).to(dev)[idx]
ws = ops.workspace(f.workspace_size(args.rows), dev)
for _ in range(2):
    ops.forest_prepare(f, X, ws)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(args.reps):
    ops.forest_prepare(f, X, ws)
ev[1].record()
torch.cuda.synchronize()
ms = ev[0].elapsed_time(ev[1]) / args.reps
out = torch.empty(args.rows, dtype=torch.float64, device=dev)
ops.forest_traverse(f, args.rows, ws, out)
exp = torch.from_numpy(z["check_proba"]).to(dev)[idx]
print(json.dumps({"rows": args.rows, "prepare_ms": round(ms, 3), "bit_exact": bool(torch.equal(out, exp)),
                  "gb_s": round(args.rows * 152 / ms / 1e6, 1)}))
