"""Whole-table featurize (+ score) pipeline on device tensors.

One call replaces the notebook's whole featurization sequence
(feature_transformation.ipynb:278, :319, :1092-1093, :2435-2436) and, with a forest, the
scoring UDF body (pyspark/scripts/fraud_detection.py:183-195):

    flags -> re-key by CUSTOMER_ID -> customer windows -> re-key by TERMINAL_ID
          -> terminal windows -> assemble the 15 input_features -> scale + forest

Input rows are in time order (the reference's order: read_from_files sorts by
TRANSACTION_ID, which the generator assigns in TX_DATETIME order,
shared_functions.py:74-90, data_generator.ipynb:1364-1369); ``time_sort=True`` first
sorts them on the GPU.  All outputs are returned in input row order.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from . import _lib, ops
from ._lib import check


@dataclass
class Features:
    weekend: torch.Tensor        # uint8 [n]
    night: torch.Tensor          # uint8 [n]
    cust_perm: torch.Tensor      # int32 [n] grouped position -> row
    cust_seg: torch.Tensor       # int64 [n_customers+1]
    cust_nb: torch.Tensor        # int32 [W, n] grouped order
    cust_avg: torch.Tensor       # float64 [W, n] grouped order
    term_perm: torch.Tensor
    term_seg: torch.Tensor
    term_nb: torch.Tensor        # int32 [W, n] grouped order
    term_risk: torch.Tensor      # float64 [W, n] grouped order
    X: Optional[torch.Tensor] = None  # float64 [n, ld] input_features in row order


class FraudPipeline:
    """avg_mode: "exact" -- the customer averages bit for bit as pandas' roll_sum (the
    sequential Kahan add/remove recurrence, k_customer_walk) -- or "scan" -- float64 prefix
    sums, fully parallel, within ~1e-13 relative of pandas (the counts
    and every other feature stay exact)."""

    # run_fused: the terminal half starts once the customer re-key is done on the device, so that
    # re-key has the GPU to itself (started together, the two re-keys took 0.90 and 1.00 ms in step
    # instead of 0.56 and 0.46 alone), and then runs at the HIGHER stream priority (lower number):
    # the customer walk's one-wave blocks take 22 KB of LDS each, 7 per CU fill a CU's LDS, and
    # dispatched first they left the terminal scatter (37-42 KB blocks) no CU until the walk's
    # queue drained (1.2 ms for a 0.2 ms pass, profiles/r05am trace).  Front half + assembly:
    # 3.84 (both at the start, customer high) -> 3.74 (terminal after the customer re-key) ->
    # 3.58-3.60 ms (and at high priority); profiles/r05ak_stream_order_ab.txt, r05an_priority_ab.txt.
    crit_priority = 0
    side_priority = -1
    terminal_after_customer_rekey = True
    # the terminal re-key's first histogram pass (+ scan, + the terminal id-range count) runs on
    # the side stream at the step's start, beside the customer re-key, instead of after it on the
    # critical chain (fdx_rekey_hist0 / fdx_rekey_payload_hist0)
    terminal_hist_ahead = 1
    # the assembly and the forest on the terminal half's stream (the half that ends last), the NaN
    # flag cleared on the main stream beforehand (tools/step_ab.py measures it against 0)
    tail_on_side = 1
    # the step's intermediates in the pipeline's own arena (ops.Arena; 0: torch's caching allocator
    # per call, as before round 6 -- tools/step_ab.py measures the two)
    use_arena = 1
    # how long the host polls for the layout plan's slot count before a blocking wait: the plan of
    # step k lands only after step k - 1's forest (6.6 ms at configs[1]) when steps are queued back
    # to back, and a blocking hipEventSynchronize woke up ~150 us after it (profiles/r06t trace: plan
    # done at 0.64 ms, layout fill at 0.81 ms)
    plan_spin_s = 0.05

    def __init__(self, windows_days: Sequence[int] = (1, 7, 30), delay_days: int = 7,
                 flags_mode: int = _lib.FDX_FLAGS_NOTEBOOK, forest: Optional[ops.Forest] = None,
                 avg_mode: str = "exact", compact_records: bool = True):
        if avg_mode not in ("exact", "scan"):
            raise ValueError("avg_mode must be 'exact' or 'scan'")
        self.avg_mode = avg_mode
        # the scoring path's terminal count records in the 16-byte compact form (3 windows): one
        # 16-byte store / load per row at random instead of two for the 24-byte record
        # (terminal windows 0.65 -> 0.41 ms alone, profiles/r03ac_compact_records_ab.txt)
        self.compact_records = bool(compact_records)
        self.windows_days = tuple(int(w) for w in windows_days)
        self.delay_days = int(delay_days)
        self.flags_mode = flags_mode
        self.forest = forest
        self.n_features = 3 + 4 * len(self.windows_days)
        self._ws = None
        self._slots_hint = None

    def featurize(self, ts_ns, customer, terminal, amount, fraud, n_customers: int, n_terminals: int,
                  assemble: bool = True, time_sort: bool = False, stream=None) -> Features:
        """ts_ns int64, customer/terminal int32 (dense ids in [0, n_*)), amount float64,
        fraud uint8 -- all GPU tensors of length n in time order (see time_sort)."""
        if time_sort:
            tperm = ops.argsort_i64(ts_ns, stream)
            f = self.featurize(ops.gather(ts_ns, tperm, stream), ops.gather(customer, tperm, stream),
                               ops.gather(terminal, tperm, stream), ops.gather(amount, tperm, stream),
                               ops.gather(fraud, tperm, stream), n_customers, n_terminals, False,
                               False, stream)
            f = _to_caller_order(f, tperm, stream)
            if assemble:
                f.X = self.assemble(f, amount, stream)
            return f
        n = ts_ns.numel()
        we, ni = ops.time_flags(ts_ns, self.flags_mode, stream)
        # the re-keys carry the columns the window kernels read (grouped, sequential)
        cperm, cseg, gts, gamt = ops.rekey_payload(customer, n_customers, ts_ns, amount, stream=stream)
        if self.avg_mode == "scan":
            cnb, cavg = ops.customer_windows_scan(gts, gamt, cseg, self.windows_days, stream=stream)
        else:
            cnb, cavg = ops.customer_windows(gts, gamt, cseg, self.windows_days, stream)
        tperm, tseg, tgts, _ = ops.rekey_payload(terminal, n_terminals, ts_ns, stream=stream)
        tnb, trisk = ops.terminal_windows_grouped(tgts, tseg, gfraud=ops.gather(fraud, tperm, stream),
                                                  delay_days=self.delay_days, windows_days=self.windows_days,
                                                  records=False, stream=stream)
        f = Features(we, ni, cperm, cseg, cnb, cavg, tperm, tseg, tnb, trisk)
        if assemble:
            f.X = self.assemble(f, amount, stream)
        return f

    def assemble(self, f: Features, amount: torch.Tensor, stream=None) -> torch.Tensor:
        n = amount.numel()
        ld = 16 if self.n_features <= 16 else self.n_features
        X = torch.empty((n, ld), dtype=torch.float64, device=amount.device)
        W = len(self.windows_days)
        p = ops._ptr
        check(_lib.load().fdx_assemble_features(n, W, p(amount), p(f.weekend), p(f.night), p(f.cust_perm),
                                                p(f.cust_nb), p(f.cust_avg), p(f.term_perm), p(f.term_nb),
                                                p(f.term_risk), p(X), ld, ops._s(stream)),
              "fdx_assemble_features")
        return X[:, : self.n_features]

    def score(self, X: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        if self.forest is None:
            raise _lib.FdxError("FraudPipeline has no forest")
        need = self.forest.workspace_size(X.shape[0])
        if self._ws is None or self._ws.numel() < need or self._ws.device != X.device:
            self._ws = ops.workspace(need, X.device)
        return self.forest.predict(X, ws=self._ws, out=out, stream=stream)

    def run(self, ts_ns, customer, terminal, amount, fraud, n_customers, n_terminals, stream=None):
        """featurize (with the float64 feature matrix) + score; returns (Features, proba)."""
        f = self.featurize(ts_ns, customer, terminal, amount, fraud, n_customers, n_terminals, True,
                           False, stream)
        return f, self.score(f.X, stream=stream)

    def run_fused(self, ts_ns, customer, terminal, amount, fraud, n_customers, n_terminals,
                  proba: torch.Tensor, ws: Optional[torch.Tensor] = None, stream=None, mark=None,
                  validate: bool = True, overlap: bool = True, rows_out=None):
        """The scoring path of bench.py: no float64 feature matrix.  The customer half is
        computed in the interleaved (lane-major) layout and the scoring rows follow that
        layout (customer features already in place, the terminal half one count record per
        row, read through the layout's irow); the last forest launch writes proba back in
        input row order.

        Streams: the terminal half (re-key + windows) runs on a side stream, concurrently with
        the customer half's layout plan, layout and walk (it waits for the customer re-key:
        terminal_after_customer_rekey) -- the customer walk is a latency-bound recurrence with one
        lane per (customer, window) that leaves most SIMDs idle; the two meet at the row assembly.  The
        customer half, assembly and forest run on a stream of the pipeline's own, the terminal half
        on a higher-priority one (crit_priority / side_priority), ordered after the caller's stream
        on entry and before it on return.
        mark(stage, stream) is called after each stage is enqueued on its stream (bench.py
        records a HIP event there).  validate: the customer / terminal ids must lie in
        [0, n_customers) / [0, n_terminals) (counted on the device, read once everything is
        enqueued -- no extra stall).  overlap=False runs everything on the caller's stream
        (bench.py's isolated per-stage timings).  rows_out: the featurized table -- the 14
        feature columns the reference's featurization writes, with each transaction's input
        row -- from the same assembly pass: an ops.FeatureRecords(n) (one record per input row,
        time order: one random 80-byte write per row) or an ops.FeatureTable (columns by
        scoring slot, written coalesced; capacity >= self.last_slots, which a caller can size
        as n * 11 // 10 -- the layout pads < 1 %; padding slots' rows are -1)."""
        W = len(self.windows_days)
        mk = mark or (lambda _name, _st: None)
        caller = stream or torch.cuda.current_stream()
        check_rows_out(rows_out, ts_ns)
        if ts_ns.numel() == 0:  # an empty table: nothing to score
            return proba
        if getattr(self, "_side", None) is None or self._side.device != ts_ns.device:
            self._side = torch.cuda.Stream(device=ts_ns.device, priority=self.side_priority)
            # two streams of the pipeline's own; their priorities: crit_priority / side_priority
            self._crit = torch.cuda.Stream(device=ts_ns.device, priority=self.crit_priority)
        main = self._crit if overlap else caller
        side = self._side if overlap else caller
        # the step's intermediates live in an arena of the pipeline's own (ops.Arena): a repeated
        # step allocates nothing; its buffers are reused by the next step, which the joins below
        # order after every use (main waits for the caller and for the side stream's last step)
        if getattr(self, "_arena", None) is None or self._arena.device != ts_ns.device:
            self._arena = ops.Arena(ts_ns.device)
        ar = self._arena if self.use_arena else _NoArena(ts_ns.device)
        # the two re-keys' scratch is one buffer when the terminal re-key starts after the customer one
        rk_shared = ("rekey_ws",) if self.terminal_after_customer_rekey else ()
        if main is not caller:
            main.wait_stream(caller)
            main.wait_stream(side)
            for t in (ts_ns, customer, terminal, amount, fraud, proba) + ((ws,) if ws is not None else ()) + \
                ((rows_out.buf,) if rows_out is not None else ()):
                t.record_stream(main)
        # an error raised after work was enqueued (a layout refused, an undersized feature table,
        # ids out of range) still joins the streams back to the caller's before it propagates
        try:
            with torch.cuda.stream(main):
                mk("start", main)
                side.wait_stream(main)
                # customer half first (the critical path): the re-key carries ts and amount into
                # grouped order
                scan = self.avg_mode == "scan"
                walk = W >= 3  # the two-kernel walk serves >= 3 windows; fewer use the one-pass ring kernel
                # the id range checks ride on the re-keys' first histogram pass (bad counts), read once
                # everything is enqueued (out-of-range ids cannot make the re-keys write out of bounds)
                bad = ar("bad", 2, torch.int32) if validate else None
                th0 = None
                # (overlapped mode only: on one stream it would just run first, and the per-stage
                # times bench.py takes in that mode would book it to the customer re-key)
                if self.terminal_hist_ahead and self.terminal_after_customer_rekey and main is not caller:
                    with torch.cuda.stream(side):
                        th0 = ops.rekey_hist0(terminal, n_terminals, side, bad=bad[1:2] if validate else None,
                                              alloc=ar.scope("th0"))
                        if validate:  # (the count's copy here too, off the terminal chain)
                            rc_t = ops.KeyRangeCheck.from_count(bad[1:2], n_terminals, "terminal ids", side)
                cperm, cseg, gts, gamt = ops.rekey_payload(customer, n_customers, ts_ns, amount, stream=main,
                                                           bad=bad[0:1] if validate else None,
                                                           alloc=ar.scope("cust", rk_shared))
                mk("rekey_customer", main)
                if self.terminal_after_customer_rekey:
                    side.wait_stream(main)
                # the walk's layout plan goes right behind the re-key; its slot count is read only
                # after the terminal half is enqueued (no host wait between the two)
                pending = ops.customer_layout_plan_async(cseg, W, main, alloc=ar.scope("plan")) \
                    if (walk and not scan) else None
                if validate:  # (its pinned copy behind the plan, not in front of it: up to 38 us)
                    rc = [ops.KeyRangeCheck.from_count(bad[0:1], n_customers, "customer ids", main)]
                # terminal half (side stream): the re-key carries ts (and TX_FRAUD in bit 31 of the
                # perm); the records come out in input row order, read by the row assembly through irow.
                # Allocated under the side stream's context, so that the caching allocator hands
                # these buffers to nothing on the main stream while the side stream still uses them.
                compact = self.compact_records and W == 3
                with torch.cuda.stream(side):
                    mk("start", side)
                    tperm, tseg, tgts, _ = ops.rekey_payload(terminal, n_terminals, ts_ns, flag=fraud, stream=side,
                                                             bad=bad[1:2] if validate and th0 is None else None,
                                                             alloc=ar.scope("term", rk_shared), hist0=th0)
                    if validate:
                        rc.append(rc_t if th0 is not None else
                                  ops.KeyRangeCheck.from_count(bad[1:2], n_terminals, "terminal ids", side))
                    mk("rekey_terminal", side)
                    if compact:
                        trec = ops.terminal_windows_compact(tgts, tseg, rows=tperm, delay_days=self.delay_days,
                                                            windows_days=self.windows_days, stream=side,
                                                            alloc=ar.scope("trec"))
                    else:
                        trec = ops.terminal_windows_grouped(tgts, tseg, rows=tperm, delay_days=self.delay_days,
                                                            windows_days=self.windows_days, stream=side)
                    mk("terminal_windows", side)
                for t in (ts_ns, customer, terminal, fraud) + ((bad,) if validate else ()):
                    t.record_stream(side)  # inputs in use on the side stream
                try:
                    if pending is not None:
                        lay = ops.customer_layout_fill(pending.result(self.plan_spin_s), cseg, cperm, gts, gamt,
                                                       self.windows_days, main,
                                                       alloc=ar.scope("lay"))
                    else:
                        lay = ops.customer_layout(cseg, cperm, gts, gamt, W, main, self._slots_hint,
                                                  self.windows_days if walk else None, grouped=True)
                except _lib.FdxError:
                    if validate:  # ids outside the range are the likelier cause: report them
                        for c in rc:
                            c.check()
                    raise
                mk("customer_layout", main)
                self._slots_hint = lay.its.numel()
                self.last_slots = lay.n_slots
                if scan:  # the windows straight from the grouped rows into the layout's slots
                    inb, isum = ops.customer_windows_scan(gts, gamt, cseg, self.windows_days, lay=lay, stream=main)
                elif walk:
                    inb, isum = ops.customer_windows_walk(lay, cseg, main, alloc=ar.scope("walk"))
                else:
                    inb, isum = ops.customer_windows_interleaved(lay, cseg, self.windows_days, main)
                mk("customer_walk", main)
                ws = self._forest_ws(lay.n_slots, ws, amount.device)
                # the assembly and the forest run on the stream that finishes its half LAST -- the
                # terminal half since round 5's reorder (it ends ~0.3 ms after the walk,
                # profiles/r05br_step_timeline.txt) -- so that no cross-stream wait (~20 us) sits
                # on the critical path; the workspace's NaN flag is cleared here, off it (5 us)
                tail = side if overlap and self.tail_on_side else main
                if tail is not main:
                    ops.forest_clear_flag(self.forest, lay.n_slots, ws, main)
                    tail.wait_stream(main)
                    for t in (lay.its, lay.iamt, lay.irow, inb, isum, ws, proba, amount) + \
                            ((rows_out.buf,) if rows_out is not None else ()):
                        t.record_stream(tail)
                else:
                    main.wait_stream(side)
                    trec.record_stream(main)
                with torch.cuda.stream(tail):
                    ops.forest_prepare_grouped(self.forest, self.flags_mode, lay.its, lay.iamt, inb, isum, lay.irow,
                                               None, trec, ws, tail, n=lay.n_slots, val_is_sum=True,
                                               term_compact=compact, rows_out=rows_out, flag_cleared=tail is not main)
                    mk("assemble_rows", tail)
                    ops.forest_traverse_perm(self.forest, lay.n_slots, ws, proba, lay.irow, tail)
                    mk("forest_traverse", tail)
                if validate:  # read once everything is enqueued (the counts ran in the re-keys)
                    for c in rc:
                        c.check()
        finally:
            if main is not caller:
                main.wait_stream(side)
                caller.wait_stream(main)
        return proba

    def _forest_ws(self, n_rows, ws, device):
        need = self.forest.workspace_size(n_rows)
        if ws is not None and ws.numel() >= need:
            return ws
        if self._ws is None or self._ws.numel() < need:
            self._ws = ops.workspace(need, device)
        return self._ws


class _NoArena:
    """use_arena = 0: every alloc() a fresh tensor from torch's caching allocator."""

    def __init__(self, device):
        self.device = device

    def __call__(self, _name, numel, dtype):
        return torch.empty(max(int(numel), 1), dtype=dtype, device=self.device)[:int(numel)]

    def scope(self, _prefix, _shared=()):
        return None  # (the ops allocate fresh tensors themselves)


def check_rows_out(rows_out, ts_ns: torch.Tensor) -> None:
    """rows_out of run_fused / ShardedPipeline.run, checked before anything is enqueued: an
    ops.FeatureRecords of >= n records or an ops.FeatureTable of >= n slots (the layout's slot
    count is >= n; its exact value is checked by the assembly), on the inputs' device."""
    if rows_out is None:
        return
    if not isinstance(rows_out, (ops.FeatureRecords, ops.FeatureTable)):
        raise TypeError("rows_out must be an ops.FeatureRecords or an ops.FeatureTable")
    if rows_out.buf.device != ts_ns.device:
        raise ValueError("rows_out must be on the inputs' device")
    if rows_out.cap < ts_ns.numel():
        raise ValueError(f"rows_out holds {rows_out.cap} rows / slots < n = {ts_ns.numel()}")


def _to_caller_order(f: Features, tperm: torch.Tensor, stream) -> Features:
    """Outputs computed on time-sorted rows -> the caller's row order (tperm[j] = caller row
    of sorted row j).  Grouped outputs keep their order; only the perms are composed."""
    return Features(ops.scatter(f.weekend, tperm, stream=stream), ops.scatter(f.night, tperm, stream=stream),
                    ops.gather(tperm, f.cust_perm, stream), f.cust_seg, f.cust_nb, f.cust_avg,
                    ops.gather(tperm, f.term_perm, stream), f.term_seg, f.term_nb, f.term_risk)
