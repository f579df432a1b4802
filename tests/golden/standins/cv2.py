"""Stand-in for the `cv2` module, used ONLY by tests/golden/gen_golden.py to run
the reference's own MVS2.py in this container (OpenCV is not installed).

Each function restates the OpenCV 4.x algorithm the reference calls, through
the CPU restatement in oracle/mvs_oracle.c.  Results are therefore pinned to
these restatements, not to a real OpenCV build (unpinned: the reference names
no OpenCV version).  Call sites: HarrisFeatures.py:125 (cvtColor),
utils.py:242-243 (Rodrigues, projectPoints), utils.py:239 (triangulatePoints),
HarrisFeatures.py:139-144 (cornerHarris, dilate; tests/golden/gen_sfm_golden.py).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
from oracle import oracle as _or  # noqa: E402

COLOR_BGR2GRAY = 6
COLOR_BGR2RGB = 4
COLOR_RGB2BGR = 4

_gray_cache = {}


def cvtColor(img, code):
    if code == COLOR_BGR2GRAY:
        # memoised on content: the reference converts the whole frame on every
        # getDescFeatures call (HarrisFeatures.py:124-125); the result only
        # depends on the bytes.
        import xxhash
        key = (img.shape, xxhash.xxh3_128_hexdigest(np.ascontiguousarray(img).tobytes()))
        g = _gray_cache.get(key)
        if g is None:
            g = _or.gray_from_rgb(img)
            _gray_cache[key] = g
        return g.copy()
    if code == COLOR_BGR2RGB:
        return np.ascontiguousarray(img[..., ::-1])
    raise NotImplementedError(code)


def Rodrigues(src):
    src = np.asarray(src, np.float64)
    if src.size == 9:
        return _or.rodrigues_m2v(src.reshape(3, 3)).reshape(3, 1), None
    return _or.rodrigues_v2m(src.reshape(3)), None


def projectPoints(objectPoints, rvec, tvec, cameraMatrix, distCoeffs):
    # computed in double; the image points take the object points' depth
    # (float32 points from SFM.py:74 give float32 projections)
    assert distCoeffs is None
    dt = np.float32 if np.asarray(objectPoints).dtype == np.float32 else np.float64
    pts = np.asarray(objectPoints, np.float64).reshape(-1, 3)
    Rp = _or.rodrigues_v2m(np.asarray(rvec, np.float64).reshape(3))
    out = np.stack([_or.project(cameraMatrix, Rp, tvec, p) for p in pts])
    return out.reshape(-1, 1, 2).astype(dt), None


def triangulatePoints(P1, P2, pts1, pts2):
    # OpenCV computes in double and creates the output with the points' type:
    # float32 points (SFM.py:67) give a float32 4xN result
    dt = np.float32 if np.asarray(pts1).dtype == np.float32 else np.float64
    pts1 = np.asarray(pts1, np.float64).reshape(2, -1)
    pts2 = np.asarray(pts2, np.float64).reshape(2, -1)
    out = np.stack([_or.triangulate(P1, P2, pts1[:, i], pts2[:, i]) for i in range(pts1.shape[1])], 1)
    return out.astype(dt)


def cornerHarris(src, blockSize, ksize, k):
    # OpenCV 4.x cornerEigenValsVecs + calcHarris (scalar path), restated in
    # oracle/sfm_oracle.c; src is np.float32(gray) (HarrisFeatures.py:139-141)
    assert blockSize == 2 and ksize == 3
    g = np.asarray(src)
    assert g.ndim == 2 and np.array_equal(g, np.rint(g)) and g.min() >= 0 and g.max() <= 255
    return _or.harris_response(g.astype(np.uint8), k)


def dilate(src, kernel):
    # default 3x3 rectangle, anchor at the centre, one iteration; the constant
    # border (morphologyDefaultBorderValue) never wins the max
    assert kernel is None
    a = np.asarray(src)
    p = np.pad(a, 1, constant_values=-np.inf).astype(a.dtype)
    out = a.copy()
    H, W = a.shape
    for u in (0, 1, 2):
        for v in (0, 1, 2):
            out = np.maximum(out, p[u:u + H, v:v + W])
    return out


def circle(img, *a, **k):
    return img


def imread(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"))[..., ::-1].copy()
