"""Multi-GPU sweeps: candidate batches sharded over ranks, accepted points
all-gathered (RCCL over xGMI on MI355X, gloo on CPU for tests).

One process per GPU (torch.distributed, backend "nccl" == RCCL on ROCm).
Every candidate's photo test depends only on read-only data (images,
cameras), so a sweep's candidates split into contiguous per-rank slices with
no communication while scoring.  Two exchanges:

* PointsExchange -- the bench's per-sweep exchange: each rank's accepted
  candidates (|V| >= vlb, MVS2.py:256/369) as rows [global index, mask
  words, x, y, z] (40 B at V <= 64: the accepted 3D point itself; or 16 B
  without the point, a candidate's geometry then being regenerated from its
  global index as in the sharded stage) packed on the device
  (mvs_pack_accepted, no host sync) into a fixed-capacity buffer and
  all-gathered on a communication stream while the next sweep scores
  (double-buffered).
* stage_sharded -- the whole DensePointsWithMVS2 stage: every rank computes
  the geometry of every child of a sweep (it depends only on records every
  rank holds), scores its contiguous slice, and the slices' photo-test masks
  (8 B per child at V <= 64) are all-gathered; every rank then runs the
  identical ordered commit (mvs_stage_* in include/mvs_amd.h).
"""
import atexit
import ctypes
import os
import weakref

import numpy as np
import torch
import torch.distributed as dist


class MaskedStream:
    """Owner of a stream of `device` whose kernels run on all CUs but
    `free_cus` of them (hipExtStreamCreateWithCUMask; bit k of the mask = CU
    k as HIP numbers them, the highest free_cus left out), or with
    complement=True on those free_cus CUs only.  `.stream` is the torch
    ExternalStream, `.cus` the CUs in its mask.  The multi-GPU step's `mask`
    layout scores on the first kind, with the scorer's grid at two workgroups
    per CU of the mask (MvsContext.set_scorer_grid), and packs on the second
    (PointsExchange) -- DESIGN.md section 7.

    close() (or the with-block's end, or garbage collection) waits for the
    stream, tells every live MvsContext that it retires (their lazy
    cross-stream ordering must not record an event on it later), then
    destroys it.  Streams still open at interpreter exit are closed by an
    atexit hook, before the HIP runtime and a profiler's tool library tear
    down: a masked stream left to the runtime's own static destructors ended
    a rocprofv3 run in a SIGSEGV inside __cxa_finalize (profiles/r05/,
    DESIGN.md 7)."""

    _live = weakref.WeakSet()

    def __init__(self, device, free_cus, complement=False):
        dev = torch.device(device)
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        free = min(max(int(free_cus), 1), ncu - 1)
        lo, hi = (ncu - free, ncu) if complement else (0, ncu - free)
        words = []
        for w in range((ncu + 31) // 32):
            v = 0
            for b in range(32):
                if lo <= 32 * w + b < hi:
                    v |= 1 << b
            words.append(v)
        arr = (ctypes.c_uint32 * len(words))(*words)
        handle = ctypes.c_void_p()
        with torch.cuda.device(dev):
            rc = _hip().hipExtStreamCreateWithCUMask(ctypes.byref(handle), ctypes.c_uint32(len(words)), arr)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
        self._handle = handle.value
        self.device = dev
        self.cus = hi - lo
        self.stream = torch.cuda.ExternalStream(handle.value, device=dev)
        MaskedStream._live.add(self)

    @property
    def cuda_stream(self):
        return self._handle

    def close(self):
        h, self._handle = getattr(self, "_handle", None), None
        if not h:
            return
        MaskedStream._live.discard(self)
        self.stream.synchronize()
        from . import _lib
        _lib.stream_retiring(h)
        rc = _hip().hipStreamDestroy(ctypes.c_void_p(h))
        if rc != 0:
            raise RuntimeError(f"hipStreamDestroy failed ({rc})")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@atexit.register
def _close_masked_streams():
    # registered after _lib's context hook (this module imports later), so
    # it runs first: streams retire while their contexts are still open
    for ms in list(MaskedStream._live):
        try:
            ms.close()
        except Exception:
            pass


def cu_masked_stream(device, free_cus, complement=False):
    """A MaskedStream (see there); release it with close() or destroy_stream()."""
    return MaskedStream(device, free_cus, complement)


def destroy_stream(stream):
    """Release a MaskedStream (after its work has completed)."""
    if not isinstance(stream, MaskedStream):
        raise TypeError("destroy_stream takes a MaskedStream (cu_masked_stream)")
    stream.close()


_HIP = None


def _hip():
    """The HIP runtime this process already runs (the libamdhip64 that torch
    loaded), opened without loading anything: a second copy of the runtime
    would hand out streams that torch and libmvs_amd do not know."""
    global _HIP
    if _HIP is None:
        path = None
        with open("/proc/self/maps") as f:
            for ln in f:
                p = ln.split()[-1] if len(ln.split()) >= 6 else ""
                if os.path.basename(p).startswith("libamdhip64.so"):
                    path = p
                    break
        if path is None:
            raise RuntimeError("the HIP runtime (libamdhip64) is not loaded in this process; import torch first")
        try:
            _HIP = ctypes.CDLL(path, mode=os.RTLD_NOLOAD)
        except OSError as e:
            raise RuntimeError(f"cannot open the loaded HIP runtime {path}: {e}") from e
        _HIP.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        _HIP.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return _HIP


def shard_range(n, rank, world):
    """Contiguous slice [begin, end) of n items for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def points_width(words, points=True):
    """int64 columns of an exchange row: global index, mask words, and the
    accepted 3D point's x, y, z (binary64 bits) when points."""
    return 1 + words + (3 if points else 0)


def sort_rows(rows):
    """Exchange rows (k, width) int64 ordered by their global index (column
    0): mvs_pack_accepted leaves its chunks in reservation order."""
    if rows.shape[0] == 0:
        return rows
    return rows[torch.argsort(rows[:, 0], stable=True)]


def pack_accepted_reference(offset, count, mask, vlb, out, c=None):
    """mvs_pack_accepted's layout from torch ops, for CPU tensors only (the
    gloo process groups of the CPU tests): header [accepted, n, 0...], then
    up to cap rows in index order (with c: the points' bits after the mask
    words).  Device tensors never come here."""
    if mask.is_cuda:
        raise RuntimeError("pack_accepted_reference is for CPU tensors; device slices use mvs_pack_accepted")
    cap = out.shape[0] - 1
    if count is None:        # records [mask words, avg bits]: |V| = popcount
        mask = mask[:, :-1]
        count = torch.from_numpy(np.bitwise_count(mask.contiguous().numpy().view(np.uint64)).sum(axis=1)
                                 .astype(np.int32))
    words = mask.shape[1]
    idx = torch.nonzero(count >= vlb).squeeze(1)
    out.zero_()
    out[0, 0] = idx.numel()
    out[0, 1] = count.numel()
    idx = idx[:cap]
    k = idx.numel()
    out[1:1 + k, 0] = idx + offset
    out[1:1 + k, 1:1 + words] = mask[idx].view(torch.int64)
    if c is not None:
        out[1:1 + k, 1 + words:4 + words] = c[idx].contiguous().view(torch.int64)


class PointsExchange:
    """Per-sweep all-gather of the accepted points as
    [global index, mask words, x, y, z] rows, in chunk order (result() sorts
    them by index) (points=False: without the
    point, which then follows from the index), pipelined: post() packs this
    rank's accepted rows on the scoring stream (no host sync) and starts the
    all-gather on a communication stream that waits only for that pack, so
    the next sweep scores while it runs.  The two send / receive buffers
    alternate; a pack waits for the all-gather that used its buffer two
    sweeps before.  cap = rows per rank (the bench takes the first sweep's
    accepted count plus a margin); a rank with more than cap accepted
    candidates shows it in its header (check() and result() raise).

    ctx = the rank's MvsContext (its pack kernel); on CPU tensors (gloo) the
    torch reference pack is used and the all-gather is synchronous."""

    def __init__(self, ctx, words, cap, device, group=None, points=True, pack_on_comm=False, comm_stream=None):
        self.ctx, self.words, self.cap, self.group = ctx, words, int(cap), group
        self.points = bool(points)
        # pack_on_comm: the pack runs on the communication stream as well (after
        # the scoring stream's sweep), overlapping the next sweep's scoring;
        # the caller then leaves the sweep's outputs alone until consumed(b)
        self.pack_on_comm = bool(pack_on_comm)
        self.read = [None, None]
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.width = points_width(words, self.points)
        self.device = torch.device(device)
        cuda = self.device.type == "cuda"
        self.send = [torch.zeros((self.cap + 1, self.width), dtype=torch.int64, device=device) for _ in range(2)]
        self.recv = [torch.zeros((self.world * (self.cap + 1), self.width), dtype=torch.int64, device=device)
                     for _ in range(2)]
        # comm_stream: e.g. a MaskedStream(complement=True) of the CUs the
        # scoring stream leaves out (held here, so that it outlives the exchange)
        self._comm_owner = comm_stream if isinstance(comm_stream, MaskedStream) else None
        if self._comm_owner is not None:
            comm_stream = self._comm_owner.stream
        self.comm = comm_stream if comm_stream is not None else (
            torch.cuda.Stream(self.device) if cuda and (self.world > 1 or self.pack_on_comm) else None)
        self.done = [None, None]
        self._held = [None, None]
        self.posted = 0

    def post(self, offset, count, mask, vlb, stream=None, c=None):
        """Pack this rank's accepted rows of a scored slice (c: its (n, 3)
        float64 centres, required when points) and start the all-gather;
        returns the buffer index for result()."""
        if self.points and c is None:
            raise RuntimeError("PointsExchange(points=True).post needs the slice's centres c")
        cc = c if self.points else None
        b = self.posted & 1
        self.posted += 1
        if mask.is_cuda:
            cur = stream if stream is not None else torch.cuda.current_stream(self.device)
            if cur.cuda_stream == 0:
                # the C-ABI reads stream 0 as "the library's own stream": the pack
                # would not be ordered with this stream's events
                raise RuntimeError("PointsExchange.post needs a non-default stream")
            if self.pack_on_comm:
                scored = torch.cuda.Event()
                scored.record(cur)
                self.comm.wait_event(scored)          # send[b]'s last gather ran on comm itself
                # the pack reads the slice's outputs on the comm stream: they
                # are held until the next post into buffer b, which orders the
                # scoring stream after this pack first (a record_stream on the
                # comm stream instead would leave the caching allocator an event
                # to record on it after a MaskedStream comm stream is destroyed)
                if self.read[b] is not None and not self.read[b].query():
                    cur.wait_event(self.read[b])
                self._held[b] = (count, mask, cc)
                self.ctx.pack_accepted(offset, count, mask, vlb, self.send[b], stream=self.comm.cuda_stream, c=cc)
                rd = torch.cuda.Event()
                rd.record(self.comm)
                self.read[b] = rd
                if self.world == 1:
                    self.done[b] = rd
                    return b
                with torch.cuda.stream(self.comm):
                    work = dist.all_gather_into_tensor(self.recv[b], self.send[b], group=self.group, async_op=True)
                    work.wait()
                    ev = torch.cuda.Event()
                    ev.record(self.comm)
                self.done[b] = ev
                return b
            if self.done[b] is not None:
                cur.wait_event(self.done[b])          # the all-gather two sweeps back has read send[b]
            self.ctx.pack_accepted(offset, count, mask, vlb, self.send[b], stream=cur.cuda_stream, c=cc)
            packed = torch.cuda.Event()
            packed.record(cur)
            if self.world == 1:
                self.done[b] = packed                 # result()/check() wait for the pack itself
                return b
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(packed)
                work = dist.all_gather_into_tensor(self.recv[b], self.send[b], group=self.group, async_op=True)
                work.wait()                           # the comm stream (not the host) waits for RCCL
                ev = torch.cuda.Event()
                ev.record(self.comm)
            self.done[b] = ev
            return b
        pack_accepted_reference(offset, count, mask, vlb, self.send[b], cc)
        if self.world > 1:
            dist.all_gather_into_tensor(self.recv[b], self.send[b], group=self.group)
        return b

    def consumed(self, b):
        """pack_on_comm: the event after which the sweep posted into buffer b
        no longer reads its outputs (None before the first post)."""
        return self.read[b]

    def blocks(self, b):
        """(world, cap + 1, width) view of buffer b's gathered rows (device);
        the caller orders its stream after the gather (wait_done)."""
        src = self.recv[b] if self.world > 1 else self.send[b]
        return src.view(self.world, self.cap + 1, self.width)

    def wait_done(self, b, stream=None):
        if self.done[b] is not None:
            (stream or torch.cuda.current_stream(self.device)).wait_event(self.done[b])

    def result(self, b):
        """The gathered accepted rows of every rank, concatenated in rank order
        (host sync; a consumer of the exchange, not the timed loop):
        (global index, mask (k, words) int64 view[, points (k, 3) float64])."""
        blk = self.check(b)
        # every rank's rows in index order (the pack orders them per chunk only)
        rows = torch.cat([sort_rows(blk[r, 1:1 + int(blk[r, 0, 0])]) for r in range(blk.shape[0])])
        if self.points:
            pts = rows[:, 1 + self.words:4 + self.words].contiguous().view(torch.float64)
            return rows[:, 0], rows[:, 1:1 + self.words], pts
        return rows[:, 0], rows[:, 1:1 + self.words]

    def check(self, b=None):
        """Wait for buffer b's exchange (default: the last posted) and raise if
        any rank's header is not a row count (a buffer no pack wrote) or
        accepted more candidates than the capacity; -> the (world, cap + 1,
        width) gathered block."""
        b = (self.posted - 1) & 1 if b is None else b
        if self.done[b] is not None:
            self.done[b].synchronize()
        blk = self.blocks(b)
        acc = blk[:, 0, 0].tolist()
        if min(acc) < 0:
            raise RuntimeError(f"PointsExchange: rank(s) {[r for r, a in enumerate(acc) if a < 0]} "
                               f"sent a negative row count (corrupt buffer)")
        if max(acc) > self.cap:
            raise RuntimeError(f"PointsExchange capacity {self.cap} < accepted {max(acc)}")
        return blk

    def accepted(self, b=None):
        """Accepted rows per rank of buffer b (after check())."""
        return self.check(b)[:, 0, 0].tolist()


def gather_slices(out, group=None):
    """All-gather equal-size slice blocks (slice_max, width) -> (world, slice_max, width)."""
    world = dist.get_world_size(group)
    # concatenated along dim 0 (the layout every backend accepts), viewed per rank
    flat = torch.empty((world * out.shape[0],) + tuple(out.shape[1:]), dtype=out.dtype,
                       device=out.device)
    dist.all_gather_into_tensor(flat, out.contiguous(), group=group)
    return flat.view((world,) + tuple(out.shape))


def stage_sharded(ctx, track_off, obs_view, obs_xy, cell_size=2, scale=1.0, wid=5,
                  max_pops=100000, group=None, device=None, filter_outliers=False):
    """DensePointsWithMVS2 minus IO on every rank of `group` (one GPU each).

    Returns the same (initial, all, stats) on every rank as MvsContext.stage()
    returns on one GPU."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if device is None:
        device = torch.device("cuda", int(ctx.device))
    if hasattr(ctx, "set_stage_options"):      # applied by every rank's finish (identical records)
        ctx.set_stage_options(filter_outliers)
    elif filter_outliers:
        raise RuntimeError("this context has no stage options")
    st = ctx.stage_begin(track_off, obs_view, obs_xy, cell_size, scale, wid, max_pops, rank, world)
    try:
        while True:
            nj = st.plan()
            if nj == 0:
                break
            if world == 1:
                st.score_slice(None)
                st.ingest(None)
                continue
            out = torch.empty((st.slice_max(nj), st.width), dtype=torch.int64, device=device)
            st.score_slice(out)          # synchronous on the library's stream
            allbuf = gather_slices(out, group)
            if allbuf.is_cuda:
                torch.cuda.current_stream(device).synchronize()
            st.ingest(allbuf)
        return st.finish()
    finally:
        st.close()
