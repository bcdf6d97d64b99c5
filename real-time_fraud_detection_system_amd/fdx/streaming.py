"""BASELINE.json config 5: streaming micro-batches with incremental window state + scoring.

The reference's streaming job (pyspark/scripts/fraud_detection.py:88-201) reads Debezium
micro-batches from Kafka, LEFT JOINs them against feature snapshot tables written by the
batch notebooks, scales and scores them in a pandas UDF.  Config 5 asks for the real-time
version of that: each micro-batch updates the customer / terminal window state and is
scored on fresh features.  The state lives in HBM (csrc/fdx_stream.hip) and is exactly the
batch recurrences' state at each key's last row, so streaming a history batch by batch gives
the same 15 features, bit for bit, as the batch path over the whole history
(get_customer_spending_behaviour_features feature_transformation.ipynb:601-628,
get_count_risk_rolling_window :1495-1522, tests/test_gpu_stream.py).

  StreamState          device state + fdx_stream_update (features of a batch)
  StreamScorer         StreamState + the forest (scale + predict_proba) per batch
  ShardedStreamScorer  one process per GPU: customers sharded by id range, terminals owned
                       by id % world, one RCCL all-to-all there and back per batch (the
                       exchange of fdx.distributed, with the owner running its incremental
                       terminal state instead of the batch windows)
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, ops
from ._lib import FdxError, FdxUnsupported, check

_STATUS = {1: "customer ring overflow (raise customer_ring)", 2: "terminal ring overflow (raise terminal_ring)",
           4: "customer or terminal id outside the state's capacity", 8: "a key's rows went back in time"}


class StreamState:
    """Per-customer and per-terminal window state on the current GPU."""

    def __init__(self, n_customers: int, n_terminals: int, windows_days=(1, 7, 30), delay_days=7,
                 customer_ring=256, terminal_ring=256, max_batch=65536, flags_mode=_lib.FDX_FLAGS_NOTEBOOK,
                 stream=None):
        self.device = ops.require_gpu()
        self.windows_days = tuple(int(d) for d in windows_days)
        self.W = len(self.windows_days)
        self.max_batch = int(max_batch)
        h = ctypes.c_void_p()
        check(_lib.load().fdx_stream_create(int(n_customers), int(n_terminals), int(customer_ring), int(terminal_ring),
                                            self.W, ops._win_ns(self.windows_days), int(delay_days) * ops.NS_PER_DAY,
                                            int(flags_mode), self.max_batch, ctypes.byref(h), ops._s(stream)),
              "fdx_stream_create")
        self._h = h
        b = ctypes.c_size_t()
        check(_lib.load().fdx_stream_memory(h, ctypes.byref(b)), "fdx_stream_memory")
        self.memory_bytes = b.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.fdx_stream_destroy(h)
            self._h = None

    def reset(self, stream=None):
        check(_lib.load().fdx_stream_reset(self._h, ops._s(stream)), "fdx_stream_reset")

    def update(self, ts, customer=None, amount=None, terminal=None, fraud=None, X=None, term_col0=-1,
               term_records=None, cust_nb=None, cust_sum=None, stream=None):
        """One micro-batch (device tensors; int64 ns, int32 ids, f64, int32 ids, u8).  Writes and
        returns X [n, >= 3 + 4W] float64 (columns in `input_features` order) unless the
        terminal half goes to term_records [n, W] int64 (count records) and the customer half
        to the planes cust_nb [W, n] int32 / cust_sum [W, n] float64 (rolling SUM; the scoring
        layout of ops.forest_prepare_grouped with val_is_sum) -- then X is None."""
        ops._dev(ts, torch.int64, "ts")
        n = ts.numel()
        if n > self.max_batch:
            raise FdxError(f"batch of {n} rows > max_batch {self.max_batch}")
        for t, dt, name in ((customer, torch.int32, "customer"), (amount, torch.float64, "amount"),
                            (terminal, torch.int32, "terminal"), (fraud, torch.uint8, "fraud")):
            if t is not None:
                ops._dev(t, dt, name)
                if t.numel() != n:
                    raise FdxError(f"{name} has {t.numel()} rows, ts has {n}")
        W = self.W
        if (cust_nb is None) != (cust_sum is None):
            raise FdxError("cust_nb and cust_sum go together")
        if cust_nb is not None:
            ops._dev(cust_nb, torch.int32, "cust_nb")
            ops._dev(cust_sum, torch.float64, "cust_sum")
            if cust_nb.numel() < W * n or cust_sum.numel() < W * n or not (cust_nb.is_contiguous()
                                                                           and cust_sum.is_contiguous()):
                raise FdxError(f"cust_nb / cust_sum need {W} x {n} contiguous elements")
        cust_planes = customer is not None and cust_nb is not None
        if X is None and ((customer is not None and not cust_planes) or (terminal is not None
                                                                         and term_records is None)):
            X = torch.empty((n, 3 + 4 * W), dtype=torch.float64, device=ts.device)
        if X is not None and (X.dtype != torch.float64 or X.stride(1) != 1):
            raise FdxError("X must be float64 with unit column stride")
        check(_lib.load().fdx_stream_update(self._h, ops._ptr(ts), ops._ptr(customer), ops._ptr(amount),
                                            ops._ptr(terminal), ops._ptr(fraud), n, ops._ptr(X),
                                            X.stride(0) if X is not None else 0, int(term_col0),
                                            ops._ptr(cust_nb), ops._ptr(cust_sum), ops._ptr(term_records),
                                            ops._s(stream)), "fdx_stream_update")
        return X

    def check(self, stream=None):
        """Synchronise and raise if a kernel reported a problem since the last check."""
        f = ctypes.c_int32()
        check(_lib.load().fdx_stream_status(self._h, ctypes.byref(f), ops._s(stream)), "fdx_stream_status")
        if f.value:
            raise FdxUnsupported("stream state: " + "; ".join(m for b, m in _STATUS.items() if f.value & b))

    def watch(self, stream=None):
        """Enqueue a non-blocking copy of the status bits (pinned host memory + event); the
        next poll() raises if the batch that preceded this call reported a problem."""
        if getattr(self, "_pin", None) is None:
            self._pin = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._ev = torch.cuda.Event()
        check(_lib.load().fdx_stream_status_async(self._h, ctypes.c_void_p(self._pin.data_ptr()), ops._s(stream)),
              "fdx_stream_status_async")
        self._ev.record(stream or torch.cuda.current_stream())
        self._watching = True

    def poll(self, block: bool = False):
        """Raise (and clear the bits) if the last watch() saw a problem.  Non-blocking unless
        block: a copy still in flight is looked at by a later poll()."""
        if not getattr(self, "_watching", False):
            return
        if not block and not self._ev.query():
            return
        self._ev.synchronize()
        self._watching = False
        if int(self._pin.item()):
            self.check()  # synchronises, clears and raises with the decoded bits


class StreamScorer:
    """Features + scaler + forest per micro-batch on one GPU (config 5 at N = 1)."""

    def __init__(self, forest: ops.Forest, n_customers: int, n_terminals: int, windows_days=(1, 7, 30),
                 delay_days=7, customer_ring=256, terminal_ring=256, max_batch=65536,
                 flags_mode=_lib.FDX_FLAGS_NOTEBOOK, fused=True):
        self.forest = forest
        self.state = StreamState(n_customers, n_terminals, windows_days, delay_days, customer_ring, terminal_ring,
                                 max_batch, flags_mode)
        W = self.state.W
        if forest.n_features != 3 + 4 * W:
            raise FdxError(f"forest has {forest.n_features} features, the stream makes {3 + 4 * W}")
        dev = self.state.device
        self.flags_mode = int(flags_mode)
        self.fused = fused
        if fused:  # state kernels -> NB / SUM planes + count records -> scoring rows (no X matrix)
            self.cnb = torch.empty(W * max_batch, dtype=torch.int32, device=dev)
            self.csum = torch.empty(W * max_batch, dtype=torch.float64, device=dev)
            self.trec = torch.empty(max_batch * W, dtype=torch.int64, device=dev)
        else:
            self.X = torch.empty((max_batch, 3 + 4 * W), dtype=torch.float64, device=dev)
        self.ws = ops.workspace(forest.workspace_size_max(max_batch), dev)
        self.proba = torch.empty(max_batch, dtype=torch.float64, device=dev)

    def score(self, ts, customer, amount, terminal, fraud):
        """-> predict_proba[:, 1] of the batch (device view, valid until the next call).
        Ring overflows, ids out of range and rows that go back in time are flagged by the
        kernels; every batch enqueues a non-blocking copy of those bits and the next score()
        (or finish()) raises FdxUnsupported for the batch that set them."""
        self.state.poll()
        n = ts.numel()
        if not self.fused:
            X = self.state.update(ts, customer, amount, terminal, fraud, X=self.X[:n])
            out = self.forest.predict(X, ws=self.ws, out=self.proba[:n])
            self.state.watch()
            return out
        W = self.state.W
        cnb, csum = self.cnb[:W * n].view(W, n), self.csum[:W * n].view(W, n)
        trec = self.trec[:n * W].view(n, W)
        self.state.update(ts, customer, amount, terminal, fraud, term_records=trec, cust_nb=cnb, cust_sum=csum)
        # flags (from ts), averages = SUM / NB, risks = FRAUD / NB, scaling, threshold ranks
        ops.forest_prepare_grouped(self.forest, self.flags_mode, ts, amount, cnb, csum, None, None, trec, self.ws,
                                   n=n, val_is_sum=True)
        out = ops.forest_traverse(self.forest, n, self.ws, self.proba[:n])
        self.state.watch()
        return out

    def finish(self):
        """Wait for the last batch's status bits and raise if it reported a problem."""
        self.state.poll(block=True)

    def score_graph(self, ts, customer, amount, terminal, fraud, out_host=None, replay: bool = True):
        """score() replayed from a HIP graph: the batch's kernels (state update, row assembly,
        forest walk, tree sums), its status-word copy and -- with out_host (pinned, float64,
        >= n) -- the probabilities' copy to the host are captured once per (batch size, buffer
        addresses) and then launched as ONE graph per batch, so the host enqueues one call
        instead of ~10 (fused mode only).  Inputs must live at the same addresses on every call
        with that size (a consumer's staging buffers).  Same results and status semantics as
        score(); -> the device view of the probabilities.  replay=False: capture only (a consumer
        that knows its batch sizes captures them before the first batch arrives)."""
        if not self.fused:
            raise FdxError("score_graph needs the fused scorer")
        if replay:
            self.state.poll()
        n = ts.numel()
        key = (n, self.forest.epoch) + tuple(t.data_ptr() for t in (ts, customer, amount, terminal, fraud)) + \
            ((out_host.data_ptr(),) if out_host is not None else ())
        graphs = self.__dict__.setdefault("_graphs", {})
        g = graphs.get(key)
        if g is None:
            for k in [k for k in graphs if k[1] != self.forest.epoch]:
                del graphs[k]  # captured over a forest layout that no longer exists
            st = self.state
            if getattr(st, "_pin", None) is None:  # watch()'s pinned status word, captured below
                st._pin = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                st._ev = torch.cuda.Event()
            W = st.W
            cnb, csum = self.cnb[:W * n].view(W, n), self.csum[:W * n].view(W, n)
            trec = self.trec[:n * W].view(n, W)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st.update(ts, customer, amount, terminal, fraud, term_records=trec, cust_nb=cnb, cust_sum=csum)
                ops.forest_prepare_grouped(self.forest, self.flags_mode, ts, amount, cnb, csum, None, None, trec,
                                           self.ws, n=n, val_is_sum=True)
                ops.forest_traverse(self.forest, n, self.ws, self.proba[:n])
                check(_lib.load().fdx_stream_status_async(st._h, ctypes.c_void_p(st._pin.data_ptr()), ops._s()),
                      "fdx_stream_status_async")
                if out_host is not None:
                    out_host[:n].copy_(self.proba[:n], non_blocking=True)
            graphs[key] = g
        if not replay:
            return None
        g.replay()
        self.state._ev.record(torch.cuda.current_stream())
        self.state._watching = True
        return self.proba[:n]

    def score_cdc(self, tx_id, customer_id, terminal_id, amount_bytes, amount_offsets, tx_datetime_us, kafka_ts,
                  fraud=None):
        """One Debezium micro-batch scored from its wire columns, device-resident end to end --
        the reference's sink (pyspark/scripts/kafka_s3_sink_transactions.py) decodes tx_amount
        DECIMAL(10,2) bytes (:64-71), truncates tx_datetime microseconds to seconds (:167) and
        keeps the latest record per tx_id by Kafka timestamp (:180); then the scoring job scores
        the rows (fraud_detection.py:183-201).  Here: fdx_cdc_decode -> fdx_dedup_latest ->
        fdx_cdc_compact (kept records, batch order) -> score().  Inputs are device tensors:
        tx_id / customer_id / terminal_id / tx_datetime_us / kafka_ts int64 [n], amount_bytes
        uint8 (the records' bytes back to back), amount_offsets int64 [n + 1], fraud uint8 [n]
        or None (the CDC topic carries no label: zeros).  One host read per batch (the kept
        count).  -> (proba [m] device view, rows int32 [m] = batch position of each kept record)."""
        L = _lib.load()
        n = tx_id.numel()
        dev = tx_id.device
        for t, nm in ((tx_id, "tx_id"), (customer_id, "customer_id"), (terminal_id, "terminal_id"),
                      (tx_datetime_us, "tx_datetime_us"), (kafka_ts, "kafka_ts")):
            ops._dev(t, torch.int64, nm)
            if t.numel() != n:
                raise FdxError(f"{nm} has {t.numel()} rows, tx_id has {n}")
        ops._dev(amount_bytes, torch.uint8, "amount_bytes")
        ops._dev(amount_offsets, torch.int64, "amount_offsets")
        if amount_offsets.numel() != n + 1:
            raise FdxError("amount_offsets needs n + 1 entries")
        if fraud is not None:
            ops._dev(fraud, torch.uint8, "fraud")
        if n > self.state.max_batch:
            raise FdxError(f"batch of {n} records > max_batch {self.state.max_batch}")
        c = getattr(self, "_cdc", None)
        if c is None:  # per-scorer buffers for max_batch records
            m = self.state.max_batch
            c = self._cdc = dict(
                amt=torch.empty(m, dtype=torch.float64, device=dev), ts=torch.empty(m, dtype=torch.int64, device=dev),
                keep=torch.empty(m, dtype=torch.uint8, device=dev), cust=torch.empty(m, dtype=torch.int32, device=dev),
                term=torch.empty(m, dtype=torch.int32, device=dev), ts_k=torch.empty(m, dtype=torch.int64, device=dev),
                amt_k=torch.empty(m, dtype=torch.float64, device=dev), fr_k=torch.empty(m, dtype=torch.uint8, device=dev),
                rows=torch.empty(m, dtype=torch.int32, device=dev),
                status=torch.zeros(2, dtype=torch.int64, device=dev),  # [count, bad]
                ws=ops.workspace(max(L.fdx_dedup_latest_workspace_size(m), L.fdx_cdc_compact_workspace_size(m)), dev),
                host=torch.zeros(2, dtype=torch.int64, pin_memory=True))
        st = torch.cuda.current_stream()
        P, S = ops._ptr, ops._s()
        bad = c["status"][1:].view(torch.int32)[:1]  # low word of status[1]
        c["status"].zero_()
        if n:
            check(L.fdx_cdc_decode(P(amount_bytes), P(amount_offsets), P(tx_datetime_us), n, None, P(c["amt"]),
                                   P(c["ts"]), P(bad), S), "fdx_cdc_decode")
            check(L.fdx_dedup_latest(P(tx_id), P(kafka_ts), n, P(c["keep"]), P(bad), P(c["ws"]), c["ws"].numel(), S),
                  "fdx_dedup_latest")
        check(L.fdx_cdc_compact(P(c["keep"]), n, P(customer_id), P(terminal_id), P(c["ts"]), P(c["amt"]), P(fraud),
                                P(c["cust"]), P(c["term"]), P(c["ts_k"]), P(c["amt_k"]), P(c["fr_k"]), P(c["rows"]),
                                P(c["status"]), P(c["ws"]), c["ws"].numel(), S), "fdx_cdc_compact")
        c["host"].copy_(c["status"], non_blocking=True)
        st.synchronize()
        m, b = int(c["host"][0]), int(c["host"][1])
        if b:
            raise FdxUnsupported("CDC batch: a tx_amount field of 0 or > 8 bytes, or tx_id -1 (reserved)")
        out = self.score(c["ts_k"][:m], c["cust"][:m], c["amt_k"][:m], c["term"][:m], c["fr_k"][:m])
        return out, c["rows"][:m]


def stream_terminal_exchange(K, records, ts, terminal, fraud, world, n_terminals_total, windows_days=(1, 7, 30),
                             delay_days=7, group=None):
    """The per-batch terminal exchange of the sharded stream: rows to their terminal's owner
    (RCCL all-to-all), the owner's incremental update `records(rts, rterm_local, rfraud)`,
    count records back.  -> (records [n, W] in send order, send_perm).  K: the kernel set
    (fdx.distributed.GpuKernels; the CPU tests pass numpy stand-ins)."""
    from . import distributed as D

    st = D.exchange_begin(K, terminal, world, group)
    return D.exchange_finish(K, st, ts, terminal, fraud, world, n_terminals_total, windows_days, delay_days, group,
                             records=records)


class ShardedStreamScorer:
    """Config 5 over `world` GPUs (this process = `rank`).  Each rank receives the rows of its
    customers [customer_base, customer_base + n_customers_local) (Kafka partitions keyed by
    customer); terminal t's state lives on rank t % world as local id t // world."""

    def __init__(self, forest: ops.Forest, world: int, rank: int, n_customers_local: int, customer_base: int,
                 n_terminals_total: int, windows_days=(1, 7, 30), delay_days=7, customer_ring=256,
                 terminal_ring=256, max_batch=65536, max_recv=None, flags_mode=_lib.FDX_FLAGS_NOTEBOOK,
                 group=None):
        self.forest, self.world, self.rank, self.group = forest, world, rank, group
        self.customer_base = int(customer_base)
        self.n_terminals_total = int(n_terminals_total)
        n_term_local = (self.n_terminals_total + world - 1) // world
        # the owner side sees up to every rank's rows of its terminals in one batch
        self.state = StreamState(n_customers_local, n_term_local, windows_days, delay_days, customer_ring,
                                 terminal_ring, max(max_batch, max_recv or max_batch * world), flags_mode)
        self.windows_days, self.delay_days = self.state.windows_days, int(delay_days)
        W = self.state.W
        dev = self.state.device
        self.flags_mode = int(flags_mode)
        self.cnb = torch.empty(W * max_batch, dtype=torch.int32, device=dev)
        self.csum = torch.empty(W * max_batch, dtype=torch.float64, device=dev)
        self.ws = ops.workspace(forest.workspace_size_max(max_batch), dev)
        self.proba = torch.empty(max_batch, dtype=torch.float64, device=dev)

    def _owner_records(self, rts, rterm, rfr):
        rec = torch.empty((rts.numel(), self.state.W), dtype=torch.int64, device=rts.device)
        self.state.update(rts, terminal=rterm, fraud=rfr, term_records=rec)
        return rec

    def score(self, ts, customer, amount, terminal, fraud):
        from . import distributed as D

        self.state.poll()
        n = ts.numel()
        W = self.state.W
        K = D.GpuKernels
        cust = ops.key_map(customer, _lib.FDX_KEY_SUB, self.customer_base) if self.customer_base else customer
        cnb, csum = self.cnb[:W * n].view(W, n), self.csum[:W * n].view(W, n)
        self.state.update(ts, cust, amount, cust_nb=cnb, cust_sum=csum)  # customer half, local
        back, send_perm = stream_terminal_exchange(K, self._owner_records, ts, terminal, fraud, self.world,
                                                   self.n_terminals_total, self.windows_days, self.delay_days,
                                                   self.group)
        # row r's count record is back[inv[r]] (send order -> row order through the inverse)
        inv = ops.invert_perm(send_perm)
        ops.forest_prepare_grouped(self.forest, self.flags_mode, ts, amount, cnb, csum, None, inv, back, self.ws,
                                   n=n, val_is_sum=True)
        out = ops.forest_traverse(self.forest, n, self.ws, self.proba[:n])
        self.state.watch()
        return out

    def finish(self):
        self.state.poll(block=True)
