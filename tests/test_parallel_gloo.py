"""The multi-rank sweep path (parallel.py) with world_size 2 and 3 on the gloo
backend, CPU only.  The photo test inside each rank is the oracle here (the
stand-in scorer for a CPU-only process; on the GPU box the same function runs
with the HIP scorer over RCCL).  Checked: slices cover the batch exactly once,
records round-trip, and every rank ends with the same accepted set as one
process scoring the whole batch."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import DATA, GOLDEN, PKG_NAME, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_dir):
    import importlib
    sys.path.insert(0, REPO)
    sys.path.insert(0, GOLDEN)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par = importlib.import_module(PKG_NAME + ".parallel")
    syn = importlib.import_module(PKG_NAME + ".synthetic")
    from make_seeds import load_dino
    from oracle import oracle as orc
    imgs, K, R, t = load_dino(DATA)
    sc = orc.Scene(np.stack(imgs), K, R, t)
    c, ref = syn.candidates(n, K, R, t, seed=17)

    def score_fn(cs, rs):
        xy, mask, count, _ = sc.score_batch(cs.numpy(), rs.numpy(), 0.4, 5)
        return torch.from_numpy(xy), torch.from_numpy(mask.view(np.int64)), torch.from_numpy(count)

    idx, count, mask, xy = par.sharded_sweep(score_fn, torch.from_numpy(c), torch.from_numpy(ref),
                                             vlb=3, words=1)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), idx=idx.numpy(), count=count.numpy(),
             mask=mask.numpy(), xy=xy.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    import importlib
    par = importlib.import_module(PKG_NAME + ".parallel")
    for n in (0, 1, 7, 100, 1001):
        for world in (1, 2, 3, 8):
            cover = []
            for r in range(world):
                b, e = par.shard_range(n, r, world)
                assert 0 <= b <= e <= n
                cover += list(range(b, e))
            assert cover == list(range(n))


@pytest.mark.parametrize("world,n", [(2, 600), (3, 401)])
def test_sharded_sweep_gloo(tmp_path, orc, dino, world, n):
    import importlib
    syn = importlib.import_module(PKG_NAME + ".synthetic")
    mp.spawn(_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True)
    rgb, K, R, t = dino
    sc = orc.Scene(rgb, K, R, t)
    c, ref = syn.candidates(n, K, R, t, seed=17)
    xy, mask, count, _ = sc.score_batch(c, ref, 0.4, 5)
    exp = np.nonzero(count >= 3)[0]
    assert len(exp) > 0
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(z["idx"], exp)
        assert np.array_equal(z["count"], count[exp])
        assert np.array_equal(z["mask"].view(np.uint64), mask[exp])
        assert np.array_equal(z["xy"], xy[exp])


class _FakeStage:
    """Duck-typed _lib.Stage: three sweeps of known sizes; each slice row holds
    (job index, scoring rank, sweep, 7).  ingest() checks that every rank's
    rows arrive in rank order at the documented slice bounds."""

    def __init__(self, rank, world, par):
        self.rank, self.world, self.par = rank, world, par
        self.sizes = [5, 8, 3, 1]
        self.k = -1
        self.width = 4
        self.seen = []

    def plan(self):
        self.k += 1
        return self.sizes[self.k] if self.k < len(self.sizes) else 0

    def slice_max(self, nj):
        return -(-nj // self.world)

    def score_slice(self, out):
        nj = self.sizes[self.k]
        b, e = self.par.shard_range(nj, self.rank, self.world)
        out.fill_(-1)
        for q, job in enumerate(range(b, e)):
            out[q] = torch.tensor([job, self.rank, self.k, 7])

    def ingest(self, allbuf):
        nj = self.sizes[self.k]
        assert allbuf.shape == (self.world, self.slice_max(nj), self.width)
        jobs = []
        for r in range(self.world):
            b, e = self.par.shard_range(nj, r, self.world)
            rows = allbuf[r, : e - b]
            assert (rows[:, 1] == r).all() and (rows[:, 2] == self.k).all()
            jobs += rows[:, 0].tolist()
        assert jobs == list(range(nj))
        self.seen.append(nj)

    def finish(self):
        return np.zeros((0, 6)), np.zeros((0, 6)), {"ingested": self.seen}

    def close(self):
        pass


class _FakeCtx:
    device = 0

    def __init__(self, par):
        self.par = par

    def stage_begin(self, *a):
        rank, world = a[-2], a[-1]
        return _FakeStage(rank, world, self.par)


def _stage_worker(rank, world, port, out_dir):
    import importlib
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par = importlib.import_module(PKG_NAME + ".parallel")
    _, _, st = par.stage_sharded(_FakeCtx(par), None, None, None, device=torch.device("cpu"))
    np.save(os.path.join(out_dir, f"s{rank}.npy"), np.array(st["ingested"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_stage_sharded_driver_gloo(tmp_path, world):
    """parallel.stage_sharded's plan / score_slice / all-gather / ingest loop
    over gloo: every sweep's slices reach every rank, complete and in order."""
    mp.spawn(_stage_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert np.load(tmp_path / f"s{r}.npy").tolist() == [5, 8, 3, 1]


def _compact_worker(rank, world, port, n, words, out_dir):
    import importlib
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par = importlib.import_module(PKG_NAME + ".parallel")
    rng = np.random.default_rng(100 + rank)          # this rank's own sweep slice (seed = rank)
    mask = rng.integers(0, 2**63, (n, words), dtype=np.int64)
    mask[rng.random((n, words)) < 0.5] = 0
    mask[:, 0] |= np.int64(-2**63) * (rng.random(n) < 0.3)   # bit 63 set on some masks
    cnt = np.array([sum(bin(int(w) & (2**64 - 1)).count("1") for w in row) for row in mask], np.int32)
    blk = par.pack_compact(torch.from_numpy(cnt), torch.from_numpy(mask), 3)
    blocks = par.all_gather_compact(blk)
    idx, count, m = par.unpack_compact(blocks, n, words)
    # the single-sync form the bench uses delivers the same blocks
    blocks2 = par.exchange_accepted(torch.from_numpy(cnt), torch.from_numpy(mask), 3)
    assert len(blocks2) == len(blocks)
    for b1, b2 in zip(blocks, blocks2):
        assert torch.equal(b1, b2)
    np.savez(os.path.join(out_dir, f"c{rank}.npz"), idx=idx.numpy(), count=count.numpy(),
             mask=m.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,words", [(2, 1000, 1), (3, 130, 4)])
def test_compact_exchange_gloo(tmp_path, world, n, words):
    """The bench's per-sweep exchange (bitmap + masks of accepted candidates):
    every rank rebuilds every rank's accepted (index, count, mask)."""
    mp.spawn(_compact_worker, args=(world, _free_port(), n, words, str(tmp_path)), nprocs=world,
             join=True)
    exp_i, exp_c, exp_m = [], [], []
    for r in range(world):
        rng = np.random.default_rng(100 + r)
        mask = rng.integers(0, 2**63, (n, words), dtype=np.int64)
        mask[rng.random((n, words)) < 0.5] = 0
        mask[:, 0] |= np.int64(-2**63) * (rng.random(n) < 0.3)
        cnt = np.array([sum(bin(int(w) & (2**64 - 1)).count("1") for w in row) for row in mask])
        acc = np.nonzero(cnt >= 3)[0]
        exp_i.append(acc + r * n)
        exp_c.append(cnt[acc])
        exp_m.append(mask[acc])
    exp_i, exp_c, exp_m = np.concatenate(exp_i), np.concatenate(exp_c), np.concatenate(exp_m)
    assert len(exp_i) > 0
    for r in range(world):
        z = np.load(tmp_path / f"c{r}.npz")
        assert np.array_equal(z["idx"], exp_i)
        assert np.array_equal(z["count"], exp_c)
        assert np.array_equal(z["mask"], exp_m)


def _points_worker(rank, world, port, n, strong, out_dir):
    import importlib
    sys.path.insert(0, REPO)
    sys.path.insert(0, GOLDEN)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par = importlib.import_module(PKG_NAME + ".parallel")
    syn = importlib.import_module(PKG_NAME + ".synthetic")
    from make_seeds import load_dino
    from oracle import oracle as orc
    imgs, K, R, t = load_dino(DATA)
    sc = orc.Scene(np.stack(imgs), K, R, t)
    if strong:      # one queue of n candidates, rank r scores its shard_range slice
        c, ref = syn.candidates(n, K, R, t, seed=17)
        b, e = par.shard_range(n, rank, world)
        c, ref, off = c[b:e], ref[b:e], b
    else:           # weak: block r of a queue of world * n candidates
        c, ref = syn.candidates(n, K, R, t, seed=17 + rank)
        off = rank * n
    _, mask, count, _ = sc.score_batch(c, ref, 0.4, 5)
    rec = par.exchange_accepted_points(off, torch.from_numpy(count), torch.from_numpy(mask.view(np.int64)),
                                       torch.from_numpy(np.ascontiguousarray(c)), 3)
    idx, cnt, m, pts = par.unpack_points(rec, 1)
    np.savez(os.path.join(out_dir, f"p{rank}.npz"), idx=idx.numpy(), count=cnt.numpy(), mask=m.numpy(),
             pts=pts.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,strong", [(2, 500, False), (3, 401, True)])
def test_accepted_points_exchange_gloo(tmp_path, orc, dino, world, n, strong):
    """The bench's sweep exchange (bench.py, parallel.exchange_accepted_points):
    the candidate queue split over the ranks -- per-rank blocks (weak) or
    shard_range slices of one queue (strong) -- and every rank ends with the
    whole sweep's accepted records, 3D points included, as one process
    scoring the whole queue would produce them."""
    import importlib
    syn = importlib.import_module(PKG_NAME + ".synthetic")
    mp.spawn(_points_worker, args=(world, _free_port(), n, strong, str(tmp_path)), nprocs=world, join=True)
    rgb, K, R, t = dino
    sc = orc.Scene(rgb, K, R, t)
    if strong:
        c, ref = syn.candidates(n, K, R, t, seed=17)
    else:
        parts = [syn.candidates(n, K, R, t, seed=17 + r) for r in range(world)]
        c = np.concatenate([p[0] for p in parts])
        ref = np.concatenate([p[1] for p in parts])
    _, mask, count, _ = sc.score_batch(c, ref, 0.4, 5)
    exp = np.nonzero(count >= 3)[0]
    assert len(exp) > 0
    for r in range(world):
        z = np.load(tmp_path / f"p{r}.npz")
        assert np.array_equal(z["idx"], exp)
        assert np.array_equal(z["count"], count[exp])
        assert np.array_equal(z["mask"].view(np.uint64), mask[exp])
        assert np.array_equal(z["pts"], c[exp])
