"""C-ABI library: loads, exports every symbol of include/mvs_amd.h, and its
host-side geometry matches the oracle (no GPU needed for these)."""
import os
import re

import numpy as np
import pytest

from conftest import REPO


def header_symbols():
    src = open(os.path.join(REPO, "include", "mvs_amd.h")).read()
    return sorted(set(re.findall(r"\b(mvs_[a-z_]+)\s*\(", src)))


def test_library_exports_header(pkg):
    lib = pkg._lib.load()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    declared = {n for n, _, _ in pkg._lib.SIGNATURES}
    assert set(syms) == declared


def test_version(pkg):
    assert b"gfx950" in pkg._lib.load().mvs_version()


def test_rodrigues_roundtrip_matches_oracle(pkg, orc, dino):
    _, K, R, t = dino
    for v in range(len(R)):
        assert np.array_equal(pkg.rodrigues_roundtrip(R[v]), orc.rodrigues_roundtrip(R[v]))
    # near-identity / 180-degree special cases of cvRodrigues2
    rng = np.random.default_rng(0)
    for M in [np.eye(3), np.diag([1.0, -1.0, -1.0]), np.diag([-1.0, 1.0, -1.0])]:
        assert np.array_equal(pkg.rodrigues_roundtrip(M), orc.rodrigues_roundtrip(M))
    for _ in range(200):
        q, _r = np.linalg.qr(rng.normal(size=(3, 3)))
        q *= np.sign(np.linalg.det(q))
        q += rng.normal(scale=1e-7, size=(3, 3))
        assert np.array_equal(pkg.rodrigues_roundtrip(q), orc.rodrigues_roundtrip(q))


def test_triangulate_matches_oracle(pkg, orc):
    rng = np.random.default_rng(1)
    for _ in range(300):
        P1, P2 = rng.normal(size=(3, 4)), rng.normal(size=(3, 4))
        x1, x2 = rng.uniform(0, 640, 2), rng.uniform(0, 480, 2)
        assert np.array_equal(pkg.triangulate(P1, P2, x1, x2), orc.triangulate(P1, P2, x1, x2))


def test_create_without_device_fails_loudly(pkg, dino):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    rgb, K, R, t = dino
    with pytest.raises(RuntimeError):
        pkg.MvsContext(rgb[:3], K[:3], R[:3], t[:3])


def test_ply_roundtrip(pkg, tmp_path):
    rng = np.random.default_rng(0)
    pts, col = rng.normal(size=(50, 3)), rng.integers(0, 256, (50, 3)).astype(np.uint8)
    p = str(tmp_path / "x")
    pkg.export2ply(pts, col, path=p)
    back = pkg.read_ply(p + ".ply")
    assert np.array_equal(back, np.hstack([pts, col.astype(np.float64)]))
