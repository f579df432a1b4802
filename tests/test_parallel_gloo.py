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
