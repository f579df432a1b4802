"""The bench's multi-rank step on the GPU: two ranks on one
MI355X (gloo: RCCL refuses two ranks on one device; the 8-GPU RCCL run is the
driver's), each scoring its block of the global candidate queue with the HIP
scorer and posting it to parallel.PointsExchange -- device pack (k_acc_pack,
40-B rows with the accepted 3D points) on the scoring stream, all-gather on
the exchange's communication stream, double-buffered over two sweeps.  Every
rank's gathered rows must equal the oracle's accepted set of the whole queue:
global indices, view masks and points, for both blocks and both sweeps."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import DATA, GOLDEN, PKG_NAME, REPO

pytestmark = pytest.mark.gpu

N_BLOCK = 1 << 15
SWEEPS = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _seed(k, rank):
    return 1000 + 10 * k + rank


def _worker(rank, world, port, out_dir):
    import importlib
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sys.path.insert(0, GOLDEN)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module(PKG_NAME)
    par = importlib.import_module(PKG_NAME + ".parallel")
    from make_seeds import load_dino
    imgs, K, R, t = load_dino(DATA)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ctx = pkg.MvsContext(np.stack(imgs), K, R, t, device=0)
    stream = torch.cuda.Stream(dev)
    ex = par.PointsExchange(ctx, 1, N_BLOCK, dev)
    out = {}
    bufs = []
    with torch.cuda.stream(stream):
        for k in range(SWEEPS):
            c, ref = pkg.synthetic.candidates(N_BLOCK, K, R, t, seed=_seed(k, rank))
            tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
            xy = torch.empty((N_BLOCK, 2), dtype=torch.float64, device=dev)
            mask = torch.empty((N_BLOCK, 1), dtype=torch.int64, device=dev)
            count = torch.empty(N_BLOCK, dtype=torch.int32, device=dev)
            ctx.score_device(tc, tr, xy, mask, count, None, 0.7, 5, stream=stream.cuda_stream)
            # the pack reads the sweep's outputs on the scoring stream; the
            # tensors stay alive until the exchange has completed
            bufs.append((tc, tr, xy, mask, count))
            ex.post(rank * N_BLOCK, count, mask, 3, stream=stream, c=tc)
        # both sweeps are in flight (double buffer); collect them in order
        for k in range(SWEEPS):
            idx, m, pts = ex.result(k & 1)
            out[f"idx{k}"], out[f"mask{k}"], out[f"pts{k}"] = (idx.cpu().numpy(), m.cpu().numpy(),
                                                               pts.cpu().numpy())
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


def test_points_exchange_two_ranks_one_gpu(tmp_path, pkg, orc, dino):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rgb, K, R, t = dino
    sc = orc.Scene(rgb, K, R, t)
    for k in range(SWEEPS):
        parts = [pkg.synthetic.candidates(N_BLOCK, K, R, t, seed=_seed(k, r)) for r in range(world)]
        c = np.concatenate([p[0] for p in parts])
        ref = np.concatenate([p[1] for p in parts])
        _, mask, count, _ = sc.score_batch(c, ref, 0.7, 5, nthreads=8)
        exp = np.nonzero(count >= 3)[0]
        assert len(exp) > 1000
        for r in range(world):
            z = np.load(tmp_path / f"g{r}.npz")
            assert np.array_equal(z[f"idx{k}"], exp), (k, r)
            assert np.array_equal(z[f"mask{k}"].view(np.uint64), mask[exp]), (k, r)
            assert np.array_equal(z[f"pts{k}"], c[exp]), (k, r)
