"""The multi-rank sweep path (parallel.py) with world_size 2 and 3 on the gloo
backend, CPU only.  The photo test inside each rank is the oracle here (the
stand-in scorer for a CPU-only process; on the GPU box the HIP scorer and the
device pack run over RCCL).  Checked: slices cover the batch exactly once,
the stage driver delivers every rank's slice in order, and every rank ends
each sweep with the same accepted set as one process scoring the whole
batch."""
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


def _points_worker(rank, world, port, n, strong, sweeps, out_dir):
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
    out = {}
    ex = None
    for k in range(sweeps):              # consecutive sweeps through the double buffers
        seed = 17 + 100 * k
        if strong:      # one queue of n candidates, rank r scores its shard_range slice
            c, ref = syn.candidates(n, K, R, t, seed=seed)
            b, e = par.shard_range(n, rank, world)
            c, ref, off = c[b:e], ref[b:e], b
        else:           # weak: block r of a queue of world * n candidates
            c, ref = syn.candidates(n, K, R, t, seed=seed + rank)
            off = rank * n
        _, mask, count, _ = sc.score_batch(c, ref, 0.4, 5)
        if ex is None:
            ex = par.PointsExchange(None, 1, n, torch.device("cpu"))
        bi = ex.post(off, torch.from_numpy(count), torch.from_numpy(mask.view(np.int64)), 3,
                     c=torch.from_numpy(np.ascontiguousarray(c)))
        idx, m, pts = ex.result(bi)
        # the rows carry the accepted 3D points themselves
        out[f"idx{k}"], out[f"mask{k}"], out[f"pts{k}"] = idx.numpy(), m.numpy(), pts.numpy()
    # capacity overflow is reported, not silently truncated
    small = par.PointsExchange(None, 1, 2, torch.device("cpu"), points=False)
    bi = small.post(0, torch.full((10,), 5, dtype=torch.int32), torch.ones((10, 1), dtype=torch.int64), 3)
    try:
        small.result(bi)
        out["overflow_raised"] = np.array(False)
    except RuntimeError:
        out["overflow_raised"] = np.array(True)
    np.savez(os.path.join(out_dir, f"p{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,strong", [(2, 500, False), (3, 401, True)])
def test_accepted_points_exchange_gloo(tmp_path, orc, dino, world, n, strong):
    """The bench's sweep exchange (bench.py, parallel.PointsExchange: device
    pack layout, double-buffered all-gather): the candidate queue split over
    the ranks -- per-rank blocks (weak) or shard_range slices of one queue
    (strong) -- over three consecutive sweeps, and every rank ends each sweep
    with the whole sweep's accepted candidates (|V| >= 3) and masks in index
    order with their 3D points (40-B records), as one process scoring the
    whole queue finds them."""
    import importlib
    syn = importlib.import_module(PKG_NAME + ".synthetic")
    sweeps = 3
    mp.spawn(_points_worker, args=(world, _free_port(), n, strong, sweeps, str(tmp_path)), nprocs=world,
             join=True)
    rgb, K, R, t = dino
    sc = orc.Scene(rgb, K, R, t)
    for k in range(sweeps):
        seed = 17 + 100 * k
        if strong:
            c, ref = syn.candidates(n, K, R, t, seed=seed)
        else:
            parts = [syn.candidates(n, K, R, t, seed=seed + r) for r in range(world)]
            c = np.concatenate([p[0] for p in parts])
            ref = np.concatenate([p[1] for p in parts])
        _, mask, count, _ = sc.score_batch(c, ref, 0.4, 5)
        exp = np.nonzero(count >= 3)[0]
        assert len(exp) > 0
        for r in range(world):
            z = np.load(tmp_path / f"p{r}.npz")
            assert np.array_equal(z[f"idx{k}"], exp)
            assert np.array_equal(z[f"mask{k}"].view(np.uint64), mask[exp])
            assert np.array_equal(z[f"pts{k}"], c[exp])
            assert bool(z["overflow_raised"])
