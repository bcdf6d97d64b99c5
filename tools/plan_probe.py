"""Time the one-launch customer layout plan alone (fdx_customer_layout_plan_async on the
config-2 segment offsets: 50k customers, lengths from the GPU generator), 50 launches after a
warm-up, HIP events on one stream; prints one JSON line.  (Round 3 attributed its time with
study builds stopping after each phase -- profiles/r03ao_plan_phases.txt; that switch is gone.)
    python tools/plan_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))


def main():
    import torch

    from fdx import ops, synth

    dev = torch.device("cuda", 0)
    g = synth.generate_device(50_000, 100_000, 183, seed=1234, customer_offset=0, device=dev)
    _, seg, _, _ = ops.rekey_payload(g["customer"], 50_000)
    st = torch.cuda.current_stream()
    for _ in range(5):
        ops.customer_layout_plan_async(seg, 3, st).result()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pend = []
    a.record()
    for _ in range(50):
        pend.append(ops.customer_layout_plan_async(seg, 3, st))
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"plan_us": round(a.elapsed_time(b) / 50 * 1e3, 1), "n_seg": seg.numel() - 1}))


if __name__ == "__main__":
    main()
