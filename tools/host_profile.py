"""Host-side time of FraudPipeline.run_fused by fdx.ops function (perf_counter around every
call, the pipeline's own Python in between), for config 2 -- where the step's host thread
spends its time while it enqueues (tools only).
usage: python tools/host_profile.py [--steps 5]
"""
import argparse
import collections
import functools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch

    import bench
    from fdx import ops, synth
    from fdx.pipeline import FraudPipeline

    acc = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for name in dir(ops):
        f = getattr(ops, name)
        if callable(f) and not name.startswith("_") and getattr(f, "__module__", "") == "fdx.ops":
            def wrap(fn, nm):
                @functools.wraps(fn)
                def w(*a, **k):
                    t = time.perf_counter()
                    try:
                        return fn(*a, **k)
                    finally:
                        acc[nm] += time.perf_counter() - t
                        cnt[nm] += 1
                return w
            setattr(ops, name, wrap(f, name))
    dev = torch.device("cuda", 0)
    g = synth.generate_device(50_000, 100_000, 183, seed=1234, device=dev)
    arrays, mean, scale, _, _ = bench.load_model(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    forest = ops.Forest(arrays, 15, mean, scale)
    pipe = FraudPipeline(forest=forest)
    n = g["ts"].numel()
    proba = torch.empty(n, dtype=torch.float64, device=dev)
    cols = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"])
    for _ in range(2):
        pipe.run_fused(*cols, 50_000, 100_000, proba)
    torch.cuda.synchronize()
    acc.clear()
    cnt.clear()
    tot = 0.0
    for _ in range(args.steps):
        t = time.perf_counter()
        pipe.run_fused(*cols, 50_000, 100_000, proba)
        tot += time.perf_counter() - t
        torch.cuda.synchronize()
    print(f"run_fused host time per step: {tot / args.steps * 1e3:.3f} ms")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:34s} {v / args.steps * 1e3:8.3f} ms/step  ({cnt[k] // args.steps} calls)")


if __name__ == "__main__":
    main()
