"""The oracle (CPU restatement, oracle/mvs_oracle.c) against the vectors the
reference itself produced (tests/golden/gen_golden.py).  CPU only."""
import numpy as np
import pytest

from conftest import stage_golden


@pytest.mark.parametrize("wid", [5, 3])
def test_ctncc_bit_exact(orc, func_golden, wid):
    A, B, S = (func_golden[f"ncc_{k}_w{wid}"] for k in "abs")
    got = np.array([orc.ctncc(a, b) for a, b in zip(A, B)])
    same = (got == S) | (np.isnan(got) & np.isnan(S))
    assert same.all(), np.nonzero(~same)[0][:10]
    assert np.isnan(S).any()   # constant windows are covered


def test_projection_bit_exact(orc, oracle_scene, func_golden):
    sc = oracle_scene
    xy = np.array([orc.project(sc.K[v], sc.Rp[v], sc.t[v], c)
                   for c, v in zip(func_golden["proj_c"], func_golden["proj_v"])])
    assert np.array_equal(xy, func_golden["proj_xy"])


def test_desc_window_edges(orc, func_golden):
    for y, x, ok in func_golden["desc_edge"]:
        out = np.empty(121, np.uint8)
        g = np.zeros((480, 640), np.uint8)
        r = orc.lib().or_get_desc(g.ctypes.data_as(orc._u8p), 480, 640, float(y), float(x), 5,
                                  out.ctypes.data_as(orc._u8p))
        assert bool(r) == bool(ok), (y, x)


def test_photo_test_bit_exact(oracle_scene, func_golden):
    f = func_golden
    for thr in (0.7, 0.4):
        sel = f["pt_thr"] == thr
        xy, mask, count, avg = oracle_scene.score_batch(f["pt_c"][sel], f["pt_R"][sel], thr)
        assert np.array_equal(mask, f["pt_mask"][sel])
        assert np.array_equal(count, f["pt_count"][sel])
        assert np.array_equal(avg, f["pt_avg"][sel])
        assert np.array_equal(xy, f["pt_xy"][sel])
    assert f["pt_count"].sum() > 100


@pytest.mark.parametrize("cap", [200, 2000])
def test_stage_bit_exact(oracle_scene, seeds, cap):
    g = stage_golden(cap)
    ini, allp, st = oracle_scene.mvs_stage(seeds["track_off"], seeds["obs_view"], seeds["obs_xy"],
                                           scale=10.0, max_pops=cap)
    assert st["pops"] == cap
    assert np.array_equal(ini, g["initial_patches"])
    assert np.array_equal(allp, g["all_patches"])


def test_rayplane_and_neighbor_formula(func_golden):
    """ray_plane_intersection / is_patch_neighbor (MVS2.py:298-306) with the
    OpenBLAS FMA-chain dot the oracle and the HIP kernel use."""
    def dot3(a, b):
        import math
        return math.fma(a[2], b[2], math.fma(a[1], b[1], a[0] * b[0])) if hasattr(math, "fma") \
            else _fma3(a, b)
    rp = func_golden["rayplane"]
    for row in rp:
        o, d, pc, pn, X, xn, nb = row[0:3], row[3:6], row[6:9], row[9:12], row[12:15], row[15:18], row[18]
        t = _fma3(pc - o, pn) / _fma3(d, pn)
        assert np.array_equal(o + t * d, X)
        pm = pc - X
        assert (abs(_fma3(pm, pn) + _fma3(pm, xn)) < 0.1) == bool(nb)


def _fma3(a, b):
    from fractions import Fraction as F
    x = float(F(a[0]) * F(b[0]))
    x = float(F(a[1]) * F(b[1]) + F(x))
    return float(F(a[2]) * F(b[2]) + F(x))
