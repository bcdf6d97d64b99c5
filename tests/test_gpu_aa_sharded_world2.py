"""The multi-GPU orchestration at world 2, executed: two ranks on the one GPU of the box, gloo
process group, every kernel the HIP one (the reference's only parallelism is
Spark local[*], Makefile:26-34).

ShardedPipeline.run -- the side-stream overlap, the split-size host sync, the owner-side records
over the received rows, the reply assembly into the scoring rows, rows_out -- and
ShardedStreamScorer.score's per-batch exchange run unchanged; only the two collectives
(fdx.distributed.all_to_all_split_pairs and alltoallv) are swapped for host-staged forms that
copy the device buffers through host memory and run the same gloo all-to-all / batched
point-to-point there (RCCL needs one GPU per rank).  Each rank's probabilities and featurized
table must equal the single-GPU fused path on the union of the shards, row for row, bit for bit.

The ranks are spawned before this process touches the GPU (the file sorts first among the GPU
tests), and the single-GPU reference runs inside rank 0 after the sharded work.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C, N_TERMS, DAYS, BATCH = 1200, 2500, 60, 8192


def _data():
    sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
    from fdx import synth

    shards = [synth.generate(C, N_TERMS, DAYS, r=15, seed=77 + r, customer_offset=C * r) for r in range(2)]
    whole = {k: np.concatenate([s[k] for s in shards]) for k in ("ts", "customer", "terminal", "amount", "fraud")}
    o = np.argsort(whole["ts"], kind="stable")
    return {k: v[o] for k, v in whole.items()}


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    for p in (ROOT, os.path.join(ROOT, "real-time_fraud_detection_system_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    from fdx import distributed as D
    from fdx import ops
    from fdx.pipeline import FraudPipeline
    from fdx.streaming import ShardedStreamScorer, StreamScorer
    from table_check import table_as_X

    dist.init_process_group("gloo", rank=rank, world_size=world)
    staged_v = D.alltoallv

    def pairs_host(out, inp, group=None):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), group=group)
        out.copy_(h)
        return out

    def alltoallv_host(out, inp, out_splits, in_splits, group=None):
        h = torch.empty(out.shape, dtype=out.dtype)
        staged_v(h, inp.cpu(), out_splits, in_splits, group)
        out.copy_(h)
        return out

    D.all_to_all_split_pairs, D.alltoallv = pairs_host, alltoallv_host
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    d = _data()
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    res = {}

    # batch: this rank's customers' rows (time order), ShardedPipeline.run with the table
    m = (d["customer"] >= C * rank) & (d["customer"] < C * (rank + 1))
    args = [T(d[k][m], dt) for k, dt in (("ts", torch.int64), ("customer", torch.int32), ("terminal", torch.int32),
                                           ("amount", torch.float64), ("fraud", torch.uint8))]
    n = int(m.sum())
    sp = D.ShardedPipeline(FraudPipeline(forest=forest), world, rank, N_TERMS, customer_base=C * rank,
                           n_customers_local=C)
    for rep in range(2):  # twice: the second step reuses the streams and the slot hint
        proba = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
        rows = ops.FeatureTable(n * 11 // 10 + 4096, dev)
        stats = {}
        sp.run(*args, proba, ops.workspace(forest.workspace_size(n * 11 // 10 + 4096), dev), rows_out=rows,
               stats=stats)
        torch.cuda.synchronize()
    res["proba"] = proba.cpu().numpy()
    res["X"] = table_as_X(rows, sp.pipe.last_slots, d["amount"][m])
    res["send_rows"] = np.array(stats["send_rows"])

    # streaming: common time cuts, each rank scores its customers' rows of every micro-batch
    cuts = np.r_[np.arange(0, len(d["ts"]), BATCH), len(d["ts"])]
    ss = ShardedStreamScorer(forest, world, rank, C, C * rank, N_TERMS, terminal_ring=1024, max_batch=BATCH,
                             max_recv=BATCH * world)
    sp_out = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        mb = m[a:b]
        cols = [T(d[k][a:b][mb], dt) for k, dt in (("ts", torch.int64), ("customer", torch.int32),
                                                    ("amount", torch.float64), ("terminal", torch.int32),
                                                    ("fraud", torch.uint8))]
        sp_out.append(ss.score(*cols).cpu().numpy().copy())
    ss.finish()
    res["stream"] = np.concatenate(sp_out)
    dist.barrier()
    if rank == 0:  # the single-GPU references on the union
        pipe = FraudPipeline(forest=forest)
        u = [T(d[k], dt) for k, dt in (("ts", torch.int64), ("customer", torch.int32), ("terminal", torch.int32),
                                       ("amount", torch.float64), ("fraud", torch.uint8))]
        N = len(d["ts"])
        pu = torch.empty(N, dtype=torch.float64, device=dev)
        ru = ops.FeatureTable(N * 11 // 10 + 4096, dev)
        pipe.run_fused(*u, C * world, N_TERMS, pu, rows_out=ru)
        res["ref_proba"] = pu.cpu().numpy()
        res["ref_X"] = table_as_X(ru, pipe.last_slots, d["amount"])
        ref = StreamScorer(forest, C * world, N_TERMS, terminal_ring=1024, max_batch=BATCH)
        outs = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            outs.append(ref.score(T(d["ts"][a:b], torch.int64), T(d["customer"][a:b], torch.int32),
                                  T(d["amount"][a:b], torch.float64), T(d["terminal"][a:b], torch.int32),
                                  T(d["fraud"][a:b], torch.uint8)).cpu().numpy().copy())
        ref.finish()
        res["ref_stream"] = np.concatenate(outs)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_pipeline_and_stream_world2_on_one_gpu(tmp_path):
    if torch.cuda.is_initialized():
        pytest.skip("this process already holds the GPU: the ranks must be spawned before it does")
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], codes
    d = _data()
    r0, r1 = (np.load(tmp_path / f"rank{r}.npz") for r in range(2))
    sel = [(d["customer"] >= C * r) & (d["customer"] < C * (r + 1)) for r in range(2)]
    # every rank sent rows to the other (the exchange crossed ranks), and the shards cover the union
    assert r0["send_rows"][1] > 0 and r1["send_rows"][0] > 0
    assert sel[0].sum() + sel[1].sum() == len(d["ts"])
    for r, res in enumerate((r0, r1)):
        np.testing.assert_array_equal(res["proba"], r0["ref_proba"][sel[r]], err_msg=f"rank {r} proba")
        np.testing.assert_array_equal(res["X"].view(np.int64), r0["ref_X"][sel[r]].view(np.int64),
                                      err_msg=f"rank {r} featurized table")
    # streaming: per micro-batch, each rank's rows in time order
    cuts = np.r_[np.arange(0, len(d["ts"]), BATCH), len(d["ts"])]
    for r, res in enumerate((r0, r1)):
        want = np.concatenate([r0["ref_stream"][a:b][sel[r][a:b]] for a, b in zip(cuts[:-1], cuts[1:])])
        np.testing.assert_array_equal(res["stream"], want, err_msg=f"rank {r} stream")
