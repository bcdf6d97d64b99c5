"""§8(f) row 3: the GPU generator (csrc/fdx_synth.hip via fdx.synth.generate_device).

Config 1 (5k customers / 10k terminals / 183 days): its statistics against the reference
generator's own output (tests/golden/config1_stats.json, same tolerances as the numpy
generator, tests/synth_stats.py); structure: global time order, ids in range, every terminal
strictly within radius r of its customer (data_generator.ipynb:420-437), amounts in cents,
fraud = scenario > 0, scenario 1 <=> amount > 220 where no later scenario overrode it;
determinism (same seed, same table); and a config-4 rank shard's size and time."""
import time

import numpy as np
import pytest
import torch

import synth_stats
from fdx import synth

pytestmark = pytest.mark.gpu


def _host(d):
    return {k: v.cpu().numpy() for k, v in d.items()}


def test_gpu_generator_matches_reference_statistics_config1(dev):
    for seed in (0, 1):
        d = _host(synth.generate_device(5000, 10000, 183, seed=seed, device=dev, with_scenario=True))
        secs = (d["ts"] - synth.START_NS) // synth.NS
        synth_stats.assert_close(synth_stats.stats(d["day"], secs, d["customer"], d["terminal"], d["amount"],
                                                   d["fraud"], d["scenario"]))


def test_gpu_generator_structure_and_determinism(dev):
    d1 = synth.generate_device(2000, 4000, 60, r=5.0, seed=11, customer_offset=7000, device=dev, with_scenario=True)
    d2 = synth.generate_device(2000, 4000, 60, r=5.0, seed=11, customer_offset=7000, device=dev, with_scenario=True)
    for k in d1:
        assert torch.equal(d1[k], d2[k]), k
    h = _host(d1)
    n = len(h["ts"])
    assert n > 100_000
    assert (np.diff(h["ts"]) >= 0).all()
    secs = (h["ts"] - synth.START_NS) // synth.NS
    np.testing.assert_array_equal(secs // 86400, h["day"])
    assert ((secs % 86400) > 0).all()
    assert h["customer"].min() >= 7000 and h["customer"].max() < 9000
    assert h["terminal"].min() >= 0 and h["terminal"].max() < 4000
    # same profiles and terminal map as the host generator with this seed (customers 7000..8999
    # of a population of 9,000)
    _, cx, cy, mean_amount, _, tx, ty = synth._profiles(9000, 4000, 5.0, 11, 10_000)
    c = h["customer"]
    dist = np.sqrt((tx[h["terminal"]] - cx[c]) ** 2 + (ty[h["terminal"]] - cy[c]) ** 2)
    assert (dist < 5.0).all()
    cents = h["amount"] * 100
    assert np.allclose(cents, np.rint(cents), atol=1e-6)
    assert (h["amount"] >= 0).all()
    np.testing.assert_array_equal(h["fraud"], (h["scenario"] > 0).astype(np.uint8))
    s1 = h["scenario"] == 1
    assert (h["amount"][s1] > 220).all()
    assert not ((h["amount"] > 220) & (h["scenario"] == 0)).any()


def test_gpu_generator_config4_rank_shard(dev):
    """One rank of BASELINE config 4 (1M customers / 2M terminals / 365 days over 8 GPUs):
    125k customers x 365 days ~ 87.5M transactions in HBM, generated in seconds."""
    t0 = time.perf_counter()
    d = synth.generate_device(125_000, 2_000_000, 365, seed=5, customer_offset=125_000 * 3, device=dev)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = d["ts"].numel()
    assert 85e6 < n < 90e6, n
    assert bool((d["ts"][1:] >= d["ts"][:-1]).all())
    assert int(d["customer"].min()) >= 375_000 and int(d["customer"].max()) < 500_000
    print(f"config-4 shard: {n} tx generated in {dt:.2f} s")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gpu_generator_customer_ranges_union_is_world1(dev, world):
    """the bench's ranks generate contiguous customer ranges of one
    population (every draw keyed by the global customer id, the profiles and compromised
    customers drawn for the population).  Each range's output must be the world-1 generation
    filtered to its customers, row for row, every column -- so the multi-GPU union is the same
    data at every N."""
    C, T, D = 24_000, 30_000, 90
    whole = _host(synth.generate_device(C, T, D, seed=1234, device=dev, with_scenario=True))
    n_seen = 0
    for r in range(world):
        lo, hi = r * C // world, (r + 1) * C // world
        part = _host(synth.generate_device(hi - lo, T, D, seed=1234, customer_offset=lo, n_customers_total=C,
                                           device=dev, with_scenario=True))
        m = (whole["customer"] >= lo) & (whole["customer"] < hi)
        assert m.sum() == len(part["ts"]) > 0
        for k in whole:
            np.testing.assert_array_equal(part[k], whole[k][m], err_msg=f"rank {r} of {world}: {k}")
        n_seen += len(part["ts"])
    assert n_seen == len(whole["ts"])
    assert (whole["scenario"] == 3).sum() > 0  # the scenario-3 draws are covered
