"""Multi-GPU featurize + score: customer-sharded rows, one RCCL all-to-all re-key per step.

SURVEY.md §8(e).  One process per GPU (torch.distributed, backend "nccl" = RCCL over
xGMI).  Each rank owns a contiguous range of CUSTOMER_IDs and all their transactions, so
the flags and the customer windows need no communication.  The terminal windows need all
rows of a terminal on one rank: owner(t) = t % world.  Per step

  owner keys -> stable re-key by owner -> pack {ts, term|fraud|row} (16 B/row)
  -> row exchange (splits exchanged first by all_to_all_single, 8 B per peer; the rows by
     batched point-to-point chunks, alltoallv)
  -> owner: unpack, re-key by local terminal id (segments = per-rank time-sorted runs,
     sorted inside the records kernel), terminal windows as count records (W words/row:
     NB | FRAUD << 32) written straight to receive positions
  -> the same exchange back (splits mirrored) -> scatter into the local feature matrix
  -> scale + forest locally.

Ring collectives are the wrong primitive on xGMI's point-to-point links; the all-to-all
sends 1/world of the rows to each peer over its own link.  Results are bitwise identical
to the 1-GPU pipeline (terminal features are tie-order independent, the customer windows
never leave their rank).

The routing logic is written once against a small kernel interface so that the same code
runs with the HIP kernels (GpuKernels, product) and -- in the CPU gloo tests only -- with
numpy stand-ins supplied by the test.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib, ops
from ._lib import check
from .pipeline import check_rows_out


class GpuKernels:
    """The libfdx entry points the exchange uses, on the current HIP stream."""

    owner_keys = staticmethod(lambda term, world: ops.key_map(term, _lib.FDX_KEY_MOD, world))

    rekey = staticmethod(lambda keys, n_keys: ops.rekey(keys, n_keys)[:2])
    gather = staticmethod(ops.gather)
    argsort_i64 = staticmethod(ops.argsort_i64)

    @staticmethod
    def exchange_pack(ts, term, fraud, perm):
        rec = torch.empty((perm.numel(), 2), dtype=torch.int64, device=ts.device)
        check(_lib.load().fdx_exchange_pack(ops._ptr(ts), ops._ptr(term), ops._ptr(fraud), ops._ptr(perm),
                                            perm.numel(), ops._ptr(rec), ops._s()), "fdx_exchange_pack")
        return rec

    @staticmethod
    def exchange_unpack(rec, world):
        m = rec.shape[0]
        ts = torch.empty(m, dtype=torch.int64, device=rec.device)
        tl = torch.empty(m, dtype=torch.int32, device=rec.device)
        fr = torch.empty(m, dtype=torch.uint8, device=rec.device)
        check(_lib.load().fdx_exchange_unpack(ops._ptr(rec), m, world, ops._ptr(ts), ops._ptr(tl), ops._ptr(fr),
                                              ops._s()), "fdx_exchange_unpack")
        return ts, tl, fr

    terminal_windows = staticmethod(ops.terminal_windows)

    @staticmethod
    def terminal_records_rekey(rts, rterm, rfraud, n_local_terms, delay_days, windows_days, runs=True):
        """owner side: stable re-key of the receive buffer by local terminal id carrying ts
        (and the fraud bit in the perm), then the records of segments made of per-rank
        time-sorted runs (runs=False: one rank -- every segment one run), indexed by receive
        position"""
        perm, seg, gts, _ = ops.rekey_payload(rterm, n_local_terms, rts, flag=rfraud)
        return ops.terminal_windows_grouped(gts, seg, rows=perm, delay_days=delay_days, windows_days=windows_days,
                                            runs=runs)

    @staticmethod
    def reply_assemble(reply, perm, W, X, col0):
        check(_lib.load().fdx_reply_assemble(ops._ptr(reply), ops._ptr(perm), perm.numel(), W, ops._ptr(X),
                                             X.stride(0), col0, ops._s()), "fdx_reply_assemble")


# Largest message of one point-to-point transfer.  RCCL 2.26 (the torch-ROCm wheel's) copies
# only the first half of an all_to_all_single message above 1 GiB (measured on MI355X, world
# 1: every size from 1.1 to 3 GB loses exactly its second half; <= 1 GiB and chunked calls are
# exact -- DESIGN.md §5), and a config-4 rank's exchange is 1.4 GB.  So the row exchange is
# written as batched isend/irecv in chunks of at most this many bytes: both ends of a pair
# derive the same chunking from the same count, so no rank needs another's sizes.
P2P_CHUNK_BYTES = 256 << 20

# Priority of ShardedPipeline's exchange stream.  HIP hands a new stream one of
# GPU_MAX_HW_QUEUES (4) hardware queues per priority level; after RCCL's and torch's own
# streams the normal-priority side stream was measured on the SAME hardware queue as the
# caller's stream (rocprofv3 Queue_Id), which serialises the exchange behind the customer
# half.  A high-priority stream draws from a separate queue pool, so the two halves overlap
# (world-1 step 14.47 -> 13.73 ms).
_SHARD_SIDE_PRIORITY = -1


def all_to_all_split_pairs(out, inp, group=None):
    """The split-size exchange (one [world, 2] int64 tensor each way): RCCL all_to_all_single.
    Module-level, like alltoallv, so that a test can route both through host memory (gloo on
    one GPU, tests/test_gpu_sharded_world2.py)."""
    dist.all_to_all_single(out, inp, group=group)
    return out


def alltoallv(out, inp, out_splits, in_splits, group=None):
    """all_to_all_single(out, inp, out_splits, in_splits) over rows of 2-D tensors: this
    rank's own block is a device copy, every other peer's block goes as point-to-point
    chunks of <= P2P_CHUNK_BYTES (one batched group call)."""
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    row_bytes = max(inp[:1].numel() * inp.element_size(), out[:1].numel() * out.element_size(), 1)
    chunk = max(P2P_CHUNK_BYTES // row_bytes, 1)
    io = [0]
    for c in in_splits:
        io.append(io[-1] + int(c))
    oo = [0]
    for c in out_splits:
        oo.append(oo[-1] + int(c))
    ops = []
    for p in range(world):
        if p == me:
            if io[p + 1] > io[p]:
                out[oo[p]:oo[p + 1]].copy_(inp[io[p]:io[p + 1]])
            continue
        peer = p if group is None else dist.get_global_rank(group, p)
        for a in range(io[p], io[p + 1], chunk):
            ops.append(dist.P2POp(dist.isend, inp[a:min(a + chunk, io[p + 1])], peer, group))
        for a in range(oo[p], oo[p + 1], chunk):
            ops.append(dist.P2POp(dist.irecv, out[a:min(a + chunk, oo[p + 1])], peer, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return out


def exchange_begin(K, term, world, group=None):
    """Phase 1 (enqueue only, no host sync): owner keys, re-key by owner, split exchange."""
    owner = K.owner_keys(term, world)
    send_perm, send_seg = K.rekey(owner, world)
    # peer p gets the pair (send_seg[p], send_seg[p + 1]): the split sizes are differences of
    # the pairs, taken on the host once they are read (exchange_finish) -- no device arithmetic
    send_pairs = send_seg.unfold(0, 2, 1).contiguous()    # [world, 2] int64 (a copy)
    recv_pairs = torch.empty_like(send_pairs)
    all_to_all_split_pairs(recv_pairs, send_pairs, group)
    return send_perm, send_pairs, recv_pairs


def exchange_finish(K, state, ts, term, fraud, world, n_terminals_total, windows_days=(1, 7, 30), delay_days=7,
                    group=None, records=None, mark=None, stats=None):
    """Phase 2: all-to-all of the rows, owner-side terminal records, all-to-all back.
    Returns (reply [n_local, W] count records in send order, send_perm).
    records(rts, rterm_local, rfraud) -> [m, W] count records by receive position replaces
    the owner-side batch windows (the streaming engine passes its incremental update).
    mark(name) is called after each phase is enqueued on the current stream (bench.py records
    HIP events there); stats (a dict) receives the split sizes and bytes per peer."""
    mk = mark or (lambda _name: None)
    send_perm, send_pairs, recv_pairs = state
    sc = [b - a for a, b in send_pairs.tolist()]   # host sync: split sizes
    rc = [b - a for a, b in recv_pairs.tolist()]
    rec = K.exchange_pack(ts, term, fraud, send_perm)
    recv = torch.empty((sum(rc), 2), dtype=torch.int64, device=rec.device)
    mk("exchange_pack")
    alltoallv(recv, rec, rc, sc, group)
    mk("exchange_rows")
    rts, rterm, rfr = K.exchange_unpack(recv, world)
    if records is not None:
        reply = records(rts, rterm, rfr)
    else:
        n_local_terms = (n_terminals_total + world - 1) // world
        # stable re-key by local terminal id: a segment is one time-sorted run per source rank;
        # the records kernel handles such segments itself (no global time sort of the receive buffer)
        reply = K.terminal_records_rekey(rts, rterm, rfr, n_local_terms, delay_days, windows_days,
                                         runs=world > 1)  # by receive index
    mk("owner_windows")
    back = torch.empty((sum(sc), reply.shape[1]), dtype=torch.int64, device=reply.device)
    alltoallv(back, reply, sc, rc, group)
    mk("exchange_back")
    if stats is not None:
        me = dist.get_rank(group)
        row_b, rep_b = rec.element_size() * 2, reply.element_size() * reply.shape[1]
        stats.update(send_rows=sc, recv_rows=rc,
                     bytes_to_peers=sum(c for p, c in enumerate(sc) if p != me) * row_b
                     + sum(c for p, c in enumerate(rc) if p != me) * rep_b,
                     bytes_from_peers=sum(c for p, c in enumerate(rc) if p != me) * row_b
                     + sum(c for p, c in enumerate(sc) if p != me) * rep_b,
                     row_bytes=row_b, reply_bytes=rep_b)
    return back, send_perm


def exchange_terminal_features(K, ts, term, fraud, world, n_terminals_total, windows_days=(1, 7, 30),
                               delay_days=7, group=None):
    """Runs the re-key exchange and the owner-side terminal windows.  Returns
    (reply [n_local, W] count records in send order, send_perm [n_local] send position ->
    local row)."""
    state = exchange_begin(K, term, world, group)
    return exchange_finish(K, state, ts, term, fraud, world, n_terminals_total, windows_days, delay_days, group)


def customer_shards(tx_per_customer, world: int):
    """Contiguous CUSTOMER_ID ranges, one per rank, balanced by transaction count (SURVEY.md
    §8(e)): rank k owns [base_k, base_k + count_k) with base_0 = 0 and the cut points at the
    customers whose cumulative tx count first reaches k/world of the total.  Any remainder
    (uneven customer or tx totals) lands on the ranks it falls to -- every customer is owned
    exactly once.  -> list of (customer_base, n_customers_local)."""
    import numpy as np

    c = np.asarray(tx_per_customer, dtype=np.int64)
    n_cust = len(c)
    if world < 1:
        raise ValueError("world must be >= 1")
    cum = np.cumsum(c)
    total = int(cum[-1]) if n_cust else 0
    cuts = [0]
    for k in range(1, world):
        if total:  # smallest j with rows(customers [0, j)) >= ceil(k * total / world)
            j = int(np.searchsorted(cum, -(-total * k // world), side="left")) + 1
        else:
            j = n_cust * k // world
        cuts.append(min(max(j, cuts[-1]), n_cust))
    cuts.append(n_cust)
    return [(cuts[k], cuts[k + 1] - cuts[k]) for k in range(world)]


class ShardedPipeline:
    """FraudPipeline over `world` GPUs (this process = `rank`).  The rank owns the customers
    [customer_base, customer_base + n_customers_local) -- pass each rank's range explicitly
    (customer_shards balances them by tx count); its rows are exactly those customers'."""

    def __init__(self, pipe, world: int, rank: int, n_terminals_total: int, customer_base: int | None = None,
                 group=None, n_customers_local: int | None = None):
        self.pipe, self.world, self.rank = pipe, world, rank
        self.n_terminals_total = n_terminals_total
        self.customer_base = customer_base
        self.n_customers_local = n_customers_local
        self.group = group

    def _range(self, n_customers_local=None):
        n = self.n_customers_local if n_customers_local is None else int(n_customers_local)
        if n is None:
            raise _lib.FdxError("ShardedPipeline needs this rank's n_customers_local")
        base = self.rank * n if self.customer_base is None else int(self.customer_base)
        return base, n

    def featurize(self, ts, customer, terminal, amount, fraud, n_customers_local: int | None = None):
        """customer: global ids of this rank's customers, dense in
        [customer_base, customer_base + n_customers_local)."""
        p = self.pipe
        W = len(p.windows_days)
        we, ni = ops.time_flags(ts, p.flags_mode)
        base, n_local = self._range(n_customers_local)
        cust = ops.key_map(customer, _lib.FDX_KEY_SUB, base) if base else customer
        bad = torch.empty(1, dtype=torch.int32, device=ts.device)
        cperm, cseg, gts, gamt = ops.rekey_payload(cust, n_local, ts, amount, bad=bad)
        rc = ops.KeyRangeCheck.from_count(bad, n_local, "customer ids of this shard")
        if p.avg_mode == "scan":
            cnb, cavg = ops.customer_windows_scan(gts, gamt, cseg, p.windows_days)
        else:
            cnb, cavg = ops.customer_windows(gts, gamt, cseg, p.windows_days)
        n = ts.numel()
        ld = 16 if p.n_features <= 16 else p.n_features
        X = torch.empty((n, ld), dtype=torch.float64, device=ts.device)
        P = ops._ptr
        check(_lib.load().fdx_assemble_features(n, W, P(amount), P(we), P(ni), P(cperm), P(cnb), P(cavg), None,
                                                None, None, P(X), ld, ops._s()), "fdx_assemble_features")
        back, send_perm = exchange_terminal_features(GpuKernels, ts, terminal, fraud, self.world,
                                                     self.n_terminals_total, p.windows_days, p.delay_days,
                                                     self.group)
        GpuKernels.reply_assemble(back, send_perm, W, X, 3 + 2 * W)
        rc.check()
        return X[:, : p.n_features]

    def run(self, ts, customer, terminal, amount, fraud, proba, ws, events=None, n_customers_local: int | None = None,
            mark=None, stats=None, rows_out=None):
        """featurize + score this rank's rows: the single-GPU scoring path (interleaved
        customer layout, FraudPipeline.run_fused) for the customer half; the terminal half
        comes back from the owners as packed count records in send order.  mark(stage, stream)
        after each stage is enqueued on its stream (bench.py's HIP events: the customer stages
        on the caller's stream, the exchange phases on the side stream); stats: the split sizes
        and bytes per peer of this step's exchange (exchange_finish)."""
        mk = mark or (lambda _name, _st: None)
        p = self.pipe
        W = len(p.windows_days)
        check_rows_out(rows_out, ts)
        base, n_local = self._range(n_customers_local)
        # The terminal exchange (RCCL all-to-all there and back + the owner-side windows)
        # runs on a side stream, overlapped with the customer half on the main stream; the
        # two meet at the scoring-row assembly.
        main = torch.cuda.current_stream()
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=ts.device, priority=_SHARD_SIDE_PRIORITY)
        side = self._side
        mk("start", main)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            mk("start", side)
            state = exchange_begin(GpuKernels, terminal, self.world, self.group)
            mk("exchange_splits", side)
        cust = ops.key_map(customer, _lib.FDX_KEY_SUB, base) if base else customer
        # the customer half's intermediates in the pipeline's arena (as FraudPipeline.run_fused; they
        # are used on this stream only, so stream order is the reuse order)
        if getattr(p, "_arena", None) is None or p._arena.device != ts.device:
            p._arena = ops.Arena(ts.device)
        ar = p._arena if p.use_arena else None
        A = (lambda name: ar.scope("sh." + name)) if ar is not None else (lambda name: None)
        bad = torch.empty(1, dtype=torch.int32, device=ts.device)  # counted in the re-key's first pass
        cperm, cseg, gts, gamt = ops.rekey_payload(cust, n_local, ts, amount, bad=bad, alloc=A("cust"))
        rc = ops.KeyRangeCheck.from_count(bad, n_local, "customer ids of this shard")  # read after the layout's sync
        mk("rekey_customer", main)
        scan = p.avg_mode == "scan"
        walk = W >= 3
        # the walk's layout plan right behind the re-key (no host wait): it runs while the host
        # waits for the exchange's split sizes below
        pending = ops.customer_layout_plan_async(cseg, W, alloc=A("plan")) if (walk and not scan) else None
        # the exchange's split-size sync waits only for the (short) owner re-key on the side
        # stream; enqueueing the whole exchange before the layout's host sync keeps the side
        # stream busy while the customer re-key runs
        with torch.cuda.stream(side):
            back, send_perm = exchange_finish(GpuKernels, state, ts, terminal, fraud, self.world,
                                              self.n_terminals_total, p.windows_days, p.delay_days, self.group,
                                              mark=lambda name: mk(name, side), stats=stats)
            sinv = ops.invert_perm(send_perm)   # local row -> send position (= reply record)
        if pending is not None:
            lay = ops.customer_layout_fill(pending.result(p.plan_spin_s), cseg, cperm, gts, gamt, p.windows_days,
                                           alloc=A("lay"))
        else:
            lay = ops.customer_layout(cseg, cperm, gts, gamt, W, None, p._slots_hint,
                                      p.windows_days if walk else None, grouped=True)  # (host sync on main)
        mk("customer_layout", main)
        rc.check()
        p._slots_hint = lay.its.numel()
        p.last_slots = lay.n_slots  # (the FeatureTable's slots, as FraudPipeline.run_fused)
        if scan:
            inb, isum = ops.customer_windows_scan(gts, gamt, cseg, p.windows_days, lay=lay)
        elif walk:
            inb, isum = ops.customer_windows_walk(lay, cseg, alloc=A("walk"))
        else:
            inb, isum = ops.customer_windows_interleaved(lay, cseg, p.windows_days)
        mk("customer_walk", main)
        main.wait_stream(side)
        back.record_stream(main)
        sinv.record_stream(main)
        ws = p._forest_ws(lay.n_slots, ws, ts.device)
        ops.forest_prepare_grouped(p.forest, p.flags_mode, lay.its, lay.iamt, inb, isum, lay.irow, sinv, back, ws,
                                   n=lay.n_slots, val_is_sum=True, rows_out=rows_out)
        mk("assemble_rows", main)
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
        ops.forest_traverse_perm(p.forest, lay.n_slots, ws, proba, lay.irow)
        mk("forest_traverse", main)
        if events is not None:
            b.record()
            events.append((a, b))
        return proba
