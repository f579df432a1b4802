"""Multi-GPU sweeps: candidate batches sharded over ranks, accepted records
all-gathered (RCCL over xGMI on MI355X, gloo on CPU for tests).

One process per GPU (torch.distributed, backend "nccl" == RCCL on ROCm).
Every candidate's photo test depends only on read-only data (images,
cameras), so a sweep's candidates split into contiguous per-rank slices with
no communication while scoring.  The only exchange is at the end of the
sweep: each rank packs the candidates it accepted (|V| >= vlb,
MVS2.py:256/369) as fixed-width int64 records and all-gathers them, so every
rank holds the sweep's accepted set -- the input of the replicated,
order-deterministic commit.

Record layout (int64 columns): [global index, count, mask words..., x bits, y bits].

stage_sharded() runs the whole DensePointsWithMVS2 stage this way: every
expansion sweep (the children of a block of queued patches, MVS2.py:329-369)
is split into contiguous per-rank slices, each rank scores its slice on its
GPU, the packed records are all-gathered, and every rank runs the identical
ordered commit (mvs_stage_* in include/mvs_amd.h).
"""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous slice [begin, end) of n items for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def record_width(words):
    return 2 + words + 2


def pack_accepted(offset, count, mask, xy, vlb):
    """Accepted candidates of this rank's slice as int64 records (k, record_width)."""
    acc = torch.nonzero(count >= vlb).squeeze(1)
    words = mask.shape[1]
    rec = torch.empty((acc.numel(), record_width(words)), dtype=torch.int64, device=count.device)
    if acc.numel():
        rec[:, 0] = acc + offset
        rec[:, 1] = count[acc].to(torch.int64)
        rec[:, 2:2 + words] = mask[acc].view(torch.int64)
        rec[:, 2 + words:] = xy[acc].contiguous().view(torch.int64)
    return rec


def all_gather_records(rec, group=None):
    """All-gather variable-length record blocks; returns them concatenated in rank order."""
    world = dist.get_world_size(group)
    if world == 1:
        return rec
    k = torch.tensor([rec.shape[0]], dtype=torch.int64, device=rec.device)
    ks = [torch.empty_like(k) for _ in range(world)]
    dist.all_gather(ks, k, group=group)
    sizes = [int(x.item()) for x in ks]
    kmax = max(max(sizes), 1)
    buf = torch.zeros((kmax, rec.shape[1]), dtype=rec.dtype, device=rec.device)
    buf[:rec.shape[0]] = rec
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return torch.cat([o[:s] for o, s in zip(outs, sizes)], 0)


def unpack_records(rec, words):
    """-> (index, count, mask (k, words) uint64 view as int64, xy (k, 2) float64)."""
    idx = rec[:, 0]
    count = rec[:, 1].to(torch.int32)
    mask = rec[:, 2:2 + words]
    xy = rec[:, 2 + words:].contiguous().view(torch.float64)
    return idx, count, mask, xy


# Compact form of a rank's accepted set (the bench's per-sweep exchange): one
# int64 block [k, accept bitmap (ceil(n/64) words, bit i = candidate i),
# masks of the k accepted candidates (k*words)].  count = popcount(mask) and
# the candidates' centroids / projections are known to every rank (the
# sweep's candidate list is), so the bitmap and the masks are the whole
# accepted set at 8 B per accepted candidate plus n/8 B -- 5x less than the
# explicit records above, which matters on xGMI at N = 8.
def pack_compact(count, mask, vlb):
    n = count.numel()
    words = mask.shape[1]
    nbw = (n + 63) // 64
    acc = count >= vlb
    a = acc.to(torch.int64)
    if nbw * 64 != n:
        a = torch.cat([a, a.new_zeros(nbw * 64 - n)])
    sh = torch.arange(64, dtype=torch.int64, device=count.device)
    bits = (a.view(nbw, 64) << sh).sum(1)            # distinct bits: the sum is their OR
    masks = mask[acc].reshape(-1)
    k = masks.numel() // max(words, 1)
    head = torch.full((1,), k, dtype=torch.int64, device=count.device)
    return torch.cat([head, bits, masks.view(torch.int64)])


def all_gather_compact(block, group=None):
    """All-gather the ranks' compact blocks -> list of blocks in rank order."""
    world = dist.get_world_size(group)
    if world == 1:
        return [block]
    k = torch.tensor([block.numel()], dtype=torch.int64, device=block.device)
    ks = torch.empty(world, dtype=torch.int64, device=block.device)
    dist.all_gather_into_tensor(ks, k, group=group)
    sizes = ks.tolist()
    kmax = max(sizes)
    buf = torch.zeros(kmax, dtype=torch.int64, device=block.device)
    buf[:block.numel()] = block
    flat = torch.empty(world * kmax, dtype=torch.int64, device=block.device)
    dist.all_gather_into_tensor(flat, buf, group=group)
    return [flat[r * kmax: r * kmax + sizes[r]] for r in range(world)]


def exchange_accepted(count, mask, vlb, group=None):
    """pack_compact + all_gather_compact with ONE host synchronisation: the
    accepted counts travel first (a tiny all-gather), their host copy sizes
    both the static-size compaction (nonzero_static, no sync of its own) and
    the padded data all-gather.  Returns the ranks' compact blocks."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    n = count.numel()
    words = mask.shape[1]
    nbw = (n + 63) // 64
    acc = count >= vlb
    k = acc.sum().to(torch.int64).reshape(1)
    if world > 1:
        ks = torch.empty(world, dtype=torch.int64, device=count.device)
        dist.all_gather_into_tensor(ks, k, group=group)
    else:
        ks = k
    a = acc.to(torch.int64)
    if nbw * 64 != n:
        a = torch.cat([a, a.new_zeros(nbw * 64 - n)])
    sh = torch.arange(64, dtype=torch.int64, device=count.device)
    bits = (a.view(nbw, 64) << sh).sum(1)
    sizes = ks.tolist()                               # the one host sync
    rank = dist.get_rank(group) if world > 1 else 0
    kmax = max(sizes)
    buf = torch.zeros(1 + nbw + kmax * words, dtype=torch.int64, device=count.device)
    buf[0] = k[0]
    buf[1:1 + nbw] = bits
    if sizes[rank]:
        idx = torch.nonzero_static(acc, size=sizes[rank]).squeeze(1)
        buf[1 + nbw:1 + nbw + sizes[rank] * words] = mask[idx].reshape(-1).view(torch.int64)
    if world == 1:
        return [buf[:1 + nbw + sizes[0] * words]]
    flat = torch.empty(world * buf.numel(), dtype=torch.int64, device=count.device)
    dist.all_gather_into_tensor(flat, buf, group=group)
    L = buf.numel()
    return [flat[r * L: r * L + 1 + nbw + sizes[r] * words] for r in range(world)]


def exchange_accepted_points(offset, count, mask, c, vlb, group=None):
    """The sweep's exchange step: every rank's accepted
    candidates (|V| >= vlb, MVS2.py:256/369) as int64 records
    [global index, count, mask words..., x, y, z (float64 bits)] -- the 3D
    points included -- all-gathered over the group (RCCL over xGMI for the
    nccl backend) with one host synchronisation (the record counts travel
    first).  offset = global index of this rank's candidate 0.
    Returns the records of all ranks, concatenated in rank order."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    words = mask.shape[1]
    width = 2 + words + 3
    acc = count >= vlb
    k = acc.sum().to(torch.int64).reshape(1)
    if world > 1:
        ks = torch.empty(world, dtype=torch.int64, device=count.device)
        dist.all_gather_into_tensor(ks, k, group=group)
    else:
        ks = k
    sizes = ks.tolist()                               # the one host sync
    rank = dist.get_rank(group) if world > 1 else 0
    kmax = max(max(sizes), 1)
    buf = torch.zeros((kmax, width), dtype=torch.int64, device=count.device)
    if sizes[rank]:
        idx = torch.nonzero_static(acc, size=sizes[rank]).squeeze(1)
        buf[:sizes[rank], 0] = idx + offset
        buf[:sizes[rank], 1] = count[idx].to(torch.int64)
        buf[:sizes[rank], 2:2 + words] = mask[idx].view(torch.int64)
        buf[:sizes[rank], 2 + words:] = c[idx].contiguous().view(torch.int64)
    if world == 1:
        return buf[:sizes[0]]
    flat = torch.empty((world * kmax, width), dtype=torch.int64, device=count.device)
    dist.all_gather_into_tensor(flat, buf, group=group)
    return torch.cat([flat[r * kmax: r * kmax + sizes[r]] for r in range(world)])


def unpack_points(rec, words):
    """-> (global index, count, mask (k, words) int64 view, points (k, 3) float64)."""
    return rec[:, 0], rec[:, 1].to(torch.int32), rec[:, 2:2 + words], \
        rec[:, 2 + words:].contiguous().view(torch.float64)


_POP8 = None


def unpack_compact(blocks, n, words):
    """Compact blocks of ranks 0..world-1 (slices of n candidates each, rank r's
    candidate i = global index r*n + i) -> (index, count, mask) in global order."""
    global _POP8
    idx, cnt, msk = [], [], []
    nbw = (n + 63) // 64
    for r, b in enumerate(blocks):
        k = int(b[0].item())
        bits = b[1:1 + nbw]
        sh = torch.arange(64, dtype=torch.int64, device=b.device)
        flags = ((bits.unsqueeze(1) >> sh) & 1).reshape(-1)[:n].bool()
        ii = torch.nonzero(flags).squeeze(1) + r * n
        m = b[1 + nbw:1 + nbw + k * words].reshape(k, words)
        if _POP8 is None or _POP8.device != b.device:
            _POP8 = torch.tensor([bin(v).count("1") for v in range(256)], dtype=torch.int32,
                                 device=b.device)
        c = _POP8[m.contiguous().view(torch.uint8).long()].reshape(k, -1).sum(1).to(torch.int32)
        idx.append(ii)
        cnt.append(c)
        msk.append(m)
    return torch.cat(idx), torch.cat(cnt), torch.cat(msk)


def sharded_sweep(score_fn, c, ref, vlb, words, group=None):
    """Score the sweep [c, ref] (all ranks pass the same full batch) by slices and
    exchange the accepted records.  score_fn(c_slice, ref_slice) -> (xy, mask, count)
    as tensors.  Returns (index, count, mask, xy) of every accepted candidate of the
    sweep, in global index order, identical on every rank."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    b, e = shard_range(len(ref), rank, world)
    xy, mask, count = score_fn(c[b:e], ref[b:e])
    rec = pack_accepted(b, count, mask, xy, vlb)
    allrec = all_gather_records(rec, group) if world > 1 else rec
    return unpack_records(allrec, words)


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
