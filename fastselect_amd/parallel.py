"""Multi-GPU Relief scoring over one process per GPU (torch.distributed).

The reference is single-device; this is the MI355X-native
multi-GPU path of §8e: the upper-triangle pair tiles are dealt round-robin to
the ranks (tile t -> rank t % world), every rank holds all of X, and the path
has exactly three exchange points, each a SUM all-reduce of a small float64
vector (RCCL over xGMI with the 'nccl' backend, gloo on CPU):

    pass1  -> rowstats[3n]  (sum D, sum D^2, mean-correction share per sample)
    select -> counts[2n]    (near hits, near misses)
    pass2  -> scores[p]     (per-feature score sums)

With world == 1 no collective is issued and the result equals
``MultiSURF.fit`` on one device.

ReliefF and SURF shard the focal samples instead (§8e "same row sharding"):
their neighbour selection is row-local (ReliefF's k nearest per class, SURF's
float32 sequential per-sample mean, which needs whole distance rows), so each
rank scores a slice of the samples (``shard_rows``) and one SUM all-reduce of
the p per-feature sums combines them (``relieff_scores`` / ``surf_scores``).
A rank computes every distance tile touching its 128-sample blocks.

Getting X onto the GPUs (``resident_x``): with RCCL each rank copies only its
own n/N rows over PCIe and the rows of the other ranks arrive by one
all-gather over xGMI, instead of N full host-to-device copies; the gathered
copy is registered for the column statistics and the plan
(``fs_stage_x_device``), so neither uploads X again.
"""
from __future__ import annotations

import contextlib

import numpy as np

from . import _base, _lib


def _dist():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


def row_chunk(n: int, rank: int, world: int):
    """Rows [lo, hi) that ``rank`` uploads for the all-gather of X: equal
    chunks of ceil(n / world) rows (the last one short or empty)."""
    rows = -(-n // world)
    return min(n, rank * rows), min(n, (rank + 1) * rows), rows


class GatherFailed(RuntimeError):
    """Raised on EVERY rank when some rank could not set up the all-gather of
    X, so that all of them take the per-rank upload together."""


def gather_rows(x, device=None, force=False):
    """All of the float32 / float64 host matrix ``x`` in one tensor on
    ``device`` (a CUDA ordinal; None = host tensors, the gloo rehearsal), with
    this rank copying only its ``row_chunk`` from the host and the rest
    all-gathered from the other ranks.  Returns a (world * rows, p) tensor of
    x's dtype whose first n rows are x."""
    import torch
    dist, rank, world = _dist()
    n, p = x.shape
    tdt = torch.float64 if x.dtype == np.float64 else torch.float32
    if dist is None or (world == 1 and not force):
        dev = "cpu" if device is None else torch.device("cuda", device)
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    lo, hi, rows = row_chunk(n, rank, world)
    dev = torch.device("cpu") if device is None else torch.device("cuda", device)
    # The buffer and this rank's rows are set up first and every rank learns
    # whether all of them managed it before anyone enters the all-gather: a
    # rank that failed alone (out of memory) would otherwise leave its peers
    # blocked in the collective while it went on to the next one.
    err = None
    try:
        buf = torch.empty((rows * world, p), dtype=tdt, device=dev)
        mine = buf[rank * rows:(rank + 1) * rows]
        if hi > lo:
            mine[:hi - lo].copy_(torch.from_numpy(x[lo:hi]))
    except RuntimeError as e:
        err = e
    ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        raise GatherFailed(f"rank {rank}: {err}" if err else "another rank could not stage its rows")
    if dev.type == "cuda":
        dist.all_gather_into_tensor(buf, mine)          # in place, RCCL over xGMI
        # the library reads buf on its own streams (column statistics): the
        # gather must have landed, not merely be ordered on torch's stream
        torch.cuda.current_stream(dev).synchronize()
    else:
        parts = list(buf.split(rows))
        dist.all_gather(parts, mine.clone())
    return buf


@contextlib.contextmanager
def resident_x(x, backend="gpu", device=0, gather=None):
    """X on the GPU for the calls inside the block.  Multi-GPU with RCCL:
    per-rank rows + all-gather (``gather_rows``), registered as the staged
    copy of ``x`` (fs_stage_x_device); the block receives the gathered
    device tensor (n first rows = x).  One GPU (or gloo): one host-to-device
    copy (fs_stage_x), and the block receives None.  ``x`` must be
    C-contiguous float32 or float64 (SURF's dtype).  gather=True takes the
    all-gather path at any world size with an 'nccl' group (tests)."""
    dist, _, world = _dist()
    if backend != "gpu":
        yield None
        return
    if gather is None:
        gather = dist is not None and world > 1
    if not gather or dist is None or dist.get_backend() != "nccl":
        with _lib.staged_x(backend, x, device):
            yield None
        return
    try:
        buf = gather_rows(x, device, force=True)
    except GatherFailed as e:
        # the all-gather only saves host-to-device copies: without it every
        # rank uploads X itself (same result), and says so.  Only the
        # collective decision falls back; an error inside the all-gather
        # itself propagates on the ranks that see it.
        import sys
        print(f"fastselect_amd: RCCL all-gather of X failed ({e}); uploading X per rank",
              file=sys.stderr, flush=True)
        with _lib.staged_x(backend, x, device):
            yield None
        return
    try:
        with _lib.staged_device_x(x, buf.data_ptr(), device):
            yield buf
    finally:
        import torch
        torch.cuda.current_stream(device).synchronize()
        del buf


def prepare_inputs(X, y, discrete_limit: int = 10, backend: str = "cpu", device: int = 0):
    """The preprocessing of ``MultiSURF.fit`` (MultiSURF.py:384-420), with the
    column statistics computed on ``backend`` (GPU: on ``device``, the rank's
    own GPU)."""
    x = np.ascontiguousarray(X, dtype=np.float32)
    isd, mn, mx = _base.column_preprocess(x, discrete_limit, backend, device)
    ranges = (mx - mn).astype(np.float32)
    ranges[ranges == 0] = 1
    recip = (1.0 / ranges).astype(np.float32)
    return x, np.asarray(y), recip, isd


class ShardedMultiSURF:
    """One rank's share of a MultiSURF scoring job.

    backend 'gpu': buffers are CUDA tensors on ``device``, and the plan's
    kernels, the torch ops on the exchange buffers and the collectives all run
    on one stream (``self.stream``: torch's current stream, or a stream of the
    job's own when that is the default stream, whose handle 0 would give the
    plan a stream unordered with torch's work), so each stage waits for the
    all-reduce before it without a host synchronisation.  backend 'cpu': host
    tensors (use the gloo backend).
    """

    def __init__(self, x, y, recip, is_discrete, use_star=False, backend="gpu", device=0,
                 shard=True, rows=None, shards=None, accumulation="fast"):
        import torch
        self.dist, self.rank, self.world = _dist() if shard else (None, 0, 1)
        _lib.accumulation_code(accumulation)
        if accumulation == "reference" and self.world > 1 and backend != "gpu":
            raise ValueError("accumulation='reference' over world > 1 ranks runs on the GPU "
                             "backend (fs_plan_ref_masks / fs_plan_ref_pass2)")
        # reference order over ranks (_step_reference): pass 2 is the masks'
        # all-reduce, every rank's chains, then the float32 column sums handed
        # from rank to rank
        self.ref_chain = accumulation == "reference" and self.world > 1
        self.n, self.p = x.shape
        self.backend = backend
        # tile shards per device (n beyond HBM): the device holds the distance
        # tiles of one shard at a time (fs_plan_set_shard, three rounds a step)
        if shards is None:
            shards = (_lib.multisurf_shards(self.n, self.p, self.world, device)
                      if backend == "gpu" else 1)
        if backend == "gpu":
            torch.cuda.set_device(device)
            self.tdev = torch.device("cuda", device)
            cur = torch.cuda.current_stream(self.tdev)
            self.stream = cur if cur.cuda_stream != 0 else torch.cuda.Stream(self.tdev)
            stream = self.stream.cuda_stream
        else:
            self.tdev = torch.device("cpu")
            self.stream = None
            stream = 0
        # Every rank must use the same shard count: ownership is tile t ->
        # shard t % (world * V), so ranks with different V would score some
        # tiles twice and others never.  Each rank sizes V from its own free
        # memory; the largest V fits on every rank.
        self.shards = self._agree_max(max(1, int(shards)))
        if accumulation == "reference" and self.ref_chain and self.shards > 1:
            # the rank step keeps all of a rank's tiles resident (its masks
            # are written once, then reduce-scattered): a job that needs V > 1
            # tile shards per device does not fit it
            raise MemoryError(
                f"accumulation='reference' over {self.world} ranks needs each rank's pair "
                f"tiles resident, but the devices hold only 1/{self.shards} of them; use more "
                "ranks, or one rank (the one-shot call shards by itself)")
        if accumulation == "reference":
            # one plan per rank holding all of its tiles (the one-shot calls
            # shard by themselves)
            self.shards = 1
        with self._on_stream(), _lib.accumulation(accumulation):  # plans keep their mode
            self.plan = _lib.Plan(backend, x, y, recip, is_discrete, use_star=use_star,
                                  rank=self.rank, world=self.world * self.shards, device=device,
                                  stream=stream)
        if rows is not None:  # focal-sample slice: pass 2 sums those samples only
            self.plan.set_rows(*rows)
        if self.ref_chain:
            # equal blocks of R focal rows per rank (the last ones short or
            # empty), so that each rank's rows of the decision masks are one
            # equal chunk of the buffer: a reduce-scatter, not an all-reduce
            f0, f1 = rows if rows is not None else (0, self.n)
            self.ref_R = -(-(f1 - f0) // self.world)
            lo = min(f1, f0 + self.rank * self.ref_R)
            self.ref_rows = (lo, min(f1, lo + self.ref_R))
            self.ref_f0 = f0
            self.masks = None
        f64 = torch.float64
        with self._on_stream():
            self.rowstats = torch.zeros(3 * self.n, dtype=f64, device=self.tdev)
            self.counts = torch.zeros(2 * self.n, dtype=f64, device=self.tdev)
            self.scores = torch.zeros(self.p, dtype=f64, device=self.tdev)

    @contextlib.contextmanager
    def _on_stream(self):
        """Run the block on the job's stream, ordered after the caller's
        stream on entry and before it on exit."""
        if self.stream is None:
            yield
            return
        import torch
        caller = torch.cuda.current_stream(self.tdev)
        if caller == self.stream:
            yield
            return
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            yield
        caller.wait_stream(self.stream)

    def _agree_max(self, v: int) -> int:
        """MAX of an integer over the ranks (no collective without a group)."""
        if self.dist is None or self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.int64, device=self.tdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return int(t.item())

    def set_features(self, feat_idx):
        """Score another feature subset of the resident samples from the next
        step on (fs_plan_set_features: X stays on the device)."""
        import torch
        with self._on_stream():
            self.plan.set_features(feat_idx)
            n_kept = self.plan.n_kept
            if self.scores.numel() != n_kept:
                self.scores = torch.zeros(n_kept, dtype=torch.float64, device=self.tdev)

    def _allreduce(self, t):
        # issued whenever a process group is up, world 1 included (one RCCL
        # call per exchange point; a plain single-process job has none).  The
        # ordering is explicit: RCCL runs the collective on its own internal
        # stream after the job's stream (torch's current stream here, see
        # _on_stream) reaches the call, and work.wait() makes the job's
        # stream wait for its completion before the next plan stage reads t
        # (no host synchronisation; gloo completes on the host)
        if self.dist is not None:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, async_op=True).wait()

    def _mask_words_per_row(self):
        return self.plan.ref_mask_words() // self._n_pad()

    def _n_pad(self):
        return -(-self.n // ROW_BLOCK) * ROW_BLOCK

    def _masks_of_my_rows(self):
        """The rank's pair-tile decisions (``fs_plan_ref_masks``) summed over
        the ranks for this rank's focal rows only: every (row, word) is
        written by exactly one rank, so the SUM of the buffers is the whole
        triangle's masks.  With RCCL a reduce-scatter over equal chunks of
        R rows (each rank receives 1/N of the n_pad^2/2 bytes: 202 MB / N at
        cfg4, where an all-reduce moved all of it); gloo has no
        reduce-scatter, so it all-reduces and slices the same chunk.  Returns
        (buffer, device address of row 0 in it): the chains read only rows
        ref_rows, so the address may lie before the chunk."""
        import torch
        wpr = self._mask_words_per_row()
        R, f0 = self.ref_R, self.ref_f0
        if R == 0:
            return 0
        rows_total = max(self._n_pad(), f0 + self.world * R)
        if self.masks is None:
            # whole-matrix buffer (rows past n_pad stay zero) and the chunk
            self.masks = torch.zeros(rows_total * wpr, dtype=torch.int64, device=self.tdev)
            self.mask_chunk = torch.empty(R * wpr, dtype=torch.int64, device=self.tdev)
        self.plan.ref_masks(self.masks.data_ptr(), self.plan.ref_mask_words())
        src = self.masks[f0 * wpr:(f0 + self.world * R) * wpr]
        if self.dist.get_backend() == "nccl":
            self.dist.reduce_scatter_tensor(self.mask_chunk, src, op=self.dist.ReduceOp.SUM,
                                            async_op=True).wait()
        else:
            self.dist.all_reduce(src, op=self.dist.ReduceOp.SUM, async_op=True).wait()
            self.mask_chunk.copy_(src[self.rank * R * wpr:(self.rank + 1) * R * wpr])
        lo = f0 + self.rank * R
        return self.mask_chunk.data_ptr() - lo * wpr * 8

    def _shard(self, v):
        self.plan.set_shard(self.rank + self.world * v, self.world * self.shards)

    def _step_shards(self):
        """step() with V tile shards per device: three rounds over the shards
        (row moments; thresholds + counts; weights + pass 2), each shard's
        distances recomputed per round, the shards' partial vectors summed
        before each all-reduce."""
        import torch
        V = self.shards
        tmp3 = torch.zeros_like(self.rowstats)
        tmp2 = torch.zeros_like(self.counts)
        tmps = torch.zeros_like(self.scores)
        self.rowstats.zero_()
        for v in range(V):
            self._shard(v)
            self.plan.pass1(tmp3.data_ptr())
            self.rowstats += tmp3
        self._allreduce(self.rowstats)
        self.counts.zero_()
        for v in range(V):
            self._shard(v)
            self.plan.pass1(tmp3.data_ptr())
            self.plan.select(self.rowstats.data_ptr(), tmp2.data_ptr())
            self.counts += tmp2
        self._allreduce(self.counts)
        self.scores.zero_()
        for v in range(V):
            self._shard(v)
            self.plan.pass1(tmp3.data_ptr())
            self.plan.select(self.rowstats.data_ptr(), tmp2.data_ptr())
            self.plan.pass2(self.counts.data_ptr(), tmps.data_ptr())
            self.scores += tmps
        self._allreduce(self.scores)
        return (self.scores / self.n).float()

    def _p2p(self, t):
        """``t`` as the process group moves it point to point (gloo: host)."""
        return t.cpu() if self.dist.get_backend() == "gloo" else t

    def _step_reference(self):
        """Reference-order step over world > 1 ranks (fs_plan_ref_masks,
        fs_plan_ref_pass2, fs_plan_ref_sums).  The reference sums every focal
        sample's float32 temp row into one sequential float32 column sum
        (MultiSURF.py:231-253, np.sum(temp, axis=0)), which no all-reduce of
        partials reproduces.  So: the ranks' pair-tile decisions as bit masks,
        combined by a SUM all-reduce (each word is written by one rank);
        every rank's chains for its contiguous block of focal rows at once;
        then the column sums continue from rank to rank in sample order --
        n_kept float64 values per hop -- and the last rank's are broadcast."""
        import torch
        self.plan.pass1(self.rowstats.data_ptr())
        self._allreduce(self.rowstats)
        self.plan.select(self.rowstats.data_ptr(), self.counts.data_ptr())
        self._allreduce(self.counts)
        base = self._masks_of_my_rows()
        self.plan.ref_pass2(base, self.counts.data_ptr(), *self.ref_rows)
        init = None
        if self.rank > 0:
            buf = self._p2p(torch.empty_like(self.scores))
            self.dist.recv(buf, src=self.rank - 1)
            init = buf.to(self.tdev)
        self.plan.ref_sums(init.data_ptr() if init is not None else 0, self.scores.data_ptr())
        if self.rank < self.world - 1:
            self.dist.send(self._p2p(self.scores), dst=self.rank + 1)
        last = self._p2p(self.scores)
        self.dist.broadcast(last, src=self.world - 1)
        if last is not self.scores:
            self.scores.copy_(last)
        return (self.scores / self.n).float()

    def _step_once(self):
        if self.ref_chain:
            return self._step_reference()
        if self.shards > 1:
            return self._step_shards()
        self.plan.pass1(self.rowstats.data_ptr())
        self._allreduce(self.rowstats)
        self.plan.select(self.rowstats.data_ptr(), self.counts.data_ptr())
        self._allreduce(self.counts)
        self.plan.pass2(self.counts.data_ptr(), self.scores.data_ptr())
        self._allreduce(self.scores)
        return (self.scores / self.n).float()

    def step(self):
        """One full scoring pass; returns float32 scores (device tensor).

        With 16-bit pass-1 operands the step ends with the decision check of
        the one-shot call (``fs_plan_decision_guard`` on the all-reduced
        vectors, so every rank decides alike): above its bound the plan moves
        to 32-bit operands for good and the step runs again.  ``last_guard``
        holds (risk, re-run) of the last step."""
        with self._on_stream():
            s = self._step_once()
            risk, switched = self.plan.decision_guard(self.rowstats.data_ptr(),
                                                      self.counts.data_ptr(),
                                                      self.scores.data_ptr())
            if switched:
                s = self._step_once()
        if self.stream is not None:  # s is consumed on the caller's stream
            import torch
            s.record_stream(torch.cuda.current_stream(self.tdev))
        self.last_guard = (risk, switched)
        return s

    def info(self):
        return self.plan.info()

    def weighted_pairs(self) -> int:
        return self.plan.weighted_pairs()

    def kernel_ms(self, which: int) -> float:
        return self.plan.kernel_ms(which)

    def close(self, release_cache=True):
        """Free the plan and hand its device blocks back to the device:
        torch's caching allocator shares the GPU with this job and cannot
        reclaim blocks held in the library's cache (fs_device_cache_release).
        release_cache=False keeps them for the next job (repeated fits)."""
        if self.stream is not None:
            self.stream.synchronize()
        self.plan.close()
        if self.backend == "gpu" and release_cache:
            _lib.release_device_cache()


def multisurf_scores(X, y, use_star=False, discrete_limit=10, backend="gpu", device=0,
                     release_cache=True, accumulation="fast"):
    """Score X on this rank's share of the tiles and return the full float32
    score vector (identical on every rank).  X reaches the GPUs once
    (``resident_x``: per-rank rows + an RCCL all-gather when sharded)."""
    x = _base.to_float32(np.asarray(X), pinned=backend == "gpu")
    with resident_x(x, backend, device):
        x, yv, recip, isd = prepare_inputs(x, y, discrete_limit, backend, device)
        job = ShardedMultiSURF(x, yv, recip, isd, use_star=use_star, backend=backend,
                               device=device, accumulation=accumulation)
        try:
            s = job.step()
            return s.cpu().numpy()
        finally:
            job.close(release_cache)


# ---- row-sharded ReliefF / SURF ------------------------------------------

ROW_BLOCK = 128   # the distance tile edge of the GPU plan


def shard_rows(n: int, rank: int, world: int):
    """Focal samples [begin, end) of ``rank``: whole 128-sample blocks dealt
    contiguously, so every rank touches the same number of distance tiles
    (up to one block)."""
    nb = (n + ROW_BLOCK - 1) // ROW_BLOCK
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    return min(n, b0 * ROW_BLOCK), min(n, b1 * ROW_BLOCK)


def _allreduce_sums(sums, backend, device):
    """SUM all-reduce of a float64 host vector across the ranks (RCCL on the
    GPU with the 'nccl' backend, gloo on the CPU); unchanged when world == 1."""
    dist, _, world = _dist()
    if dist is None or world == 1:
        return sums
    import torch
    on_gpu = dist.get_backend() == "nccl"
    t = torch.from_numpy(np.ascontiguousarray(sums))
    if on_gpu:
        t = t.to(torch.device("cuda", device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


@contextlib.contextmanager
def resident_cast(xd, x32, device=0):
    """The float32 copy ``x32`` of a host matrix whose float64 rows are
    already on the GPU (``xd``, the tensor resident_x yields: RCCL-gathered)
    made there by one device cast -- round to nearest even, the rounding of
    numpy's astype, so the copy is bit-identical to x32 -- and registered as
    x32's staged copy (fs_stage_x_device) for the calls inside the block.
    xd None (no gather: one GPU, gloo, the CPU backend): nothing to do, the
    calls upload x32 themselves."""
    if xd is None:
        yield
        return
    import torch
    n = x32.shape[0]
    buf = xd[:n].to(torch.float32).contiguous()
    torch.cuda.current_stream(device).synchronize()   # the library reads it on its own streams
    try:
        with _lib.staged_device_x(x32, buf.data_ptr(), device):
            yield
    finally:
        torch.cuda.current_stream(device).synchronize()
        del buf


def _chain_column_sums(plan, p, device):
    """Reference order over the ranks: rank r continues the float32 column
    sums of rank r - 1 over its temp rows (``fs_plan_ref_sums``) and hands
    them to rank r + 1; every rank returns the last rank's sums (float64
    host vector).  ``plan`` runs on its own stream and synchronises the host
    after each call."""
    import torch
    dist, rank, world = _dist()
    dev = torch.device("cuda", device)
    host = dist.get_backend() == "gloo"
    sums = torch.zeros(p, dtype=torch.float64, device=dev)
    init = None
    if rank > 0:
        buf = torch.empty(p, dtype=torch.float64, device="cpu" if host else dev)
        dist.recv(buf, src=rank - 1)
        init = buf.to(dev)
    torch.cuda.current_stream(dev).synchronize()   # init has landed (the plan's own stream)
    plan.ref_sums(init.data_ptr() if init is not None else 0, sums.data_ptr())
    out = sums.cpu() if host else sums
    if rank < world - 1:
        dist.send(out, dst=rank + 1)
    dist.broadcast(out, src=world - 1)
    return out.cpu().numpy()


def relieff_scores(X, y, n_neighbors=3, discrete_limit=10, backend="gpu", device=0, n_jobs=-1,
                   gather=None, accumulation="fast"):
    """ReliefF feature scores with the focal samples sharded over the ranks:
    this rank scores ``shard_rows(n, rank, world)``, one all-reduce sums the
    slices.  Returns the full float32 score vector (identical on every rank)
    -- ``ReliefF(n_neighbors=...).fit(X, y).feature_importances_`` up to
    float64 summation order.  X crosses the host link once over all ranks
    (``resident_x``: each rank uploads its n/N float64 rows, RCCL all-gathers
    the rest; the column statistics read that copy, and the float32 copy
    the plan scores is cast from it on the device, ``resident_cast``).

    accumulation='reference': the reference's float32 scores bit for bit.
    Its column sum is one sequential float32 sum over the focal samples
    (ReliefF.py:219-220), so over N ranks every rank forms its float32 temp
    rows at once (``fs_plan_ref_temp``) and the running sums then pass from
    rank to rank (``fs_plan_ref_sums``) instead of one all-reduce (GPU
    backend; one rank: the one-shot call)."""
    from .ReliefF import relieff_inputs
    x = np.ascontiguousarray(X, dtype=np.float64)
    yv = np.asarray(y)
    n, p = x.shape
    _lib.accumulation_code(accumulation)
    if np.unique(yv).size < 2:
        return np.zeros(p, dtype=np.float32)
    backend = _base.effective_backend(backend)
    _, rank, world = _dist()
    chain = accumulation == "reference" and world > 1
    if chain and backend != "gpu":
        raise ValueError("accumulation='reference' over world > 1 ranks runs on the GPU "
                         "backend (fs_plan_ref_temp / fs_plan_ref_sums)")
    with resident_x(x, backend, device, gather) as xd:
        x32, y_enc, recip, isd, priors = relieff_inputs(x, yv, discrete_limit, backend, device,
                                                        n_jobs)
        with resident_cast(xd, x32, device), _lib.accumulation(accumulation):
            if not chain:
                sums = _lib.relieff_score(backend, x32, y_enc, recip, isd, n_neighbors, priors,
                                          n_jobs, device=device, rows=shard_rows(n, rank, world))
            else:
                plan = _lib.RowsPlan(backend, "relieff", x32, y_enc, recip, isd, k=n_neighbors,
                                     class_probs=priors, rows=shard_rows(n, rank, world),
                                     n_jobs=n_jobs, device=device)
                try:
                    plan.ref_temp()
                    sums = _chain_column_sums(plan, p, device)
                finally:
                    plan.close()
    if not chain:
        sums = _allreduce_sums(sums, backend, device)
    return (sums / n).astype(np.float32)


def surf_scores(X, y, use_star=False, discrete_limit=10, backend="gpu", device=0, n_jobs=-1,
                gather=None, accumulation="fast"):
    """SURF / SURF* feature scores with the focal samples sharded over the
    ranks (see ``relieff_scores``); X (float64, SURF.py:330-332) reaches the
    GPUs by per-rank rows + one RCCL all-gather of float64 rows.

    accumulation='reference': the reference's float32 scores (its n_jobs=1
    order) bit for bit: every rank forms its float32 temp rows at once
    (``fs_plan_ref_temp``) and the column sums pass from rank to rank in
    sample order (SURF.py:195: one sequential float32 sum)."""
    from .SURF import surf_inputs
    x = np.ascontiguousarray(X, dtype=np.float64)
    n, p = x.shape
    _lib.accumulation_code(accumulation)
    backend = _base.effective_backend(backend)
    _, rank, world = _dist()
    chain = accumulation == "reference" and world > 1
    if chain and backend != "gpu":
        raise ValueError("accumulation='reference' over world > 1 ranks runs on the GPU "
                         "backend (fs_plan_ref_temp / fs_plan_ref_sums)")
    yi = np.asarray(y).astype(np.int32)
    with resident_x(x, backend, device, gather):
        isd, recip = surf_inputs(x, discrete_limit, backend, device)
        with _lib.accumulation(accumulation):
            if not chain:
                sums = _lib.surf_score(backend, x, yi, recip, use_star, isd, n_jobs,
                                       device=device, rows=shard_rows(n, rank, world))
            else:
                plan = _lib.RowsPlan(backend, "surf", x, yi, recip, isd, use_star=use_star,
                                     rows=shard_rows(n, rank, world), n_jobs=n_jobs,
                                     device=device)
                try:
                    plan.ref_temp()
                    sums = _chain_column_sums(plan, p, device)
                finally:
                    plan.close()
    if not chain:
        sums = _allreduce_sums(sums, backend, device)
    return (sums / n).astype(np.float32)
