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


def test_filter_outliers_crafted_vs_reference(pkg):
    """filter_out_outlier (MVS2.py:132-158) where it does remove patches: the
    host core the stage's opt-in filter runs (mvs_filter_outliers) on the 60
    crafted patch sets of tests/golden/filter_crafted.npz, recorded from the
    reference's own CellTable (gen_golden.py --filter-crafted): the same
    survivors, the same "remove a outlier" line count, ZeroDivisionError where
    the reference raised it, and the survivors in reconstruct_from_Q's order
    (MVS2.py:159-173: first sight in the (view, ci, cj) key walk = a stable
    sort by (min view of V, cell))."""
    g = dict(np.load(os.path.join(REPO, "tests", "golden", "filter_crafted.npz")))
    cs, H, W = int(g["cs"]), int(g["H"]), int(g["W"])
    nci, ncj = -(-(W - 1) // cs), -(-(H - 1) // cs)
    n_rem = n_dz = 0
    for k in range(int(g["n_cases"])):
        mask, xy = g[f"c{k}_mask"], g[f"c{k}_xy"]
        cell = np.floor(xy / cs).astype(np.int32)
        count = np.array([bin(int(m)).count("1") for m in mask], np.int32)
        args = (cell, mask.reshape(-1, 1), count, g[f"c{k}_avg"], g[f"c{k}_c"], g[f"c{k}_n"], nci, ncj)
        if bool(g[f"c{k}_divzero"]):
            with pytest.raises(ZeroDivisionError):
                pkg._lib.filter_outliers(*args)
            n_dz += 1
            continue
        alive, removed, lines = pkg._lib.filter_outliers(*args)
        assert lines == int(g[f"c{k}_lines"]), k
        assert removed == len(mask) - alive.sum()
        minv = np.array([(int(m) & -int(m)).bit_length() - 1 for m in mask])
        ids = np.nonzero(alive)[0]
        order = sorted(ids, key=lambda e: (minv[e], cell[e, 0], cell[e, 1]))   # stable: fill order
        assert order == g[f"c{k}_survivors"].tolist(), k
        n_rem += removed > 0
    assert n_rem >= 40 and n_dz >= 1


def test_filter_outliers_bad_arguments(pkg):
    with pytest.raises(RuntimeError):
        pkg._lib.filter_outliers(np.zeros((1, 2)), np.ones(1, np.uint64), [1], [0.5], np.zeros(3), np.zeros(3), 0, 4)


def test_sanitizer_builds_when_requested(pkg, orc):
    """Under tools/asan_cpu.sh (MVS_LIB / MVS_ORACLE_LIB name the ASan + UBSan
    builds) the process really runs them: both libraries and the sanitizer
    runtime are mapped."""
    if "asan" not in os.environ.get("MVS_LIB", "") and "asan" not in os.environ.get("MVS_ORACLE_LIB", ""):
        pytest.skip("not a sanitizer run")
    pkg._lib.load()
    orc.lib()
    maps = open("/proc/self/maps").read()
    assert "libmvs_amd_asan.so" in maps and "libmvs_oracle_asan.so" in maps
    assert "libclang_rt.asan" in maps
