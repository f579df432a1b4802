"""Stand-in for pyntcloud (absent), used ONLY by tests/golden/gen_golden.py.
`PyntCloud(df).to_file(path)` (utils.py:250-251) records the DataFrame that
the reference would have written as PLY."""
import numpy as np

written = {}


class PyntCloud:
    def __init__(self, points):
        self.points = points

    def to_file(self, path):
        written[path] = np.asarray(self.points.values, np.float64).copy()
