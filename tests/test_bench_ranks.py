"""bench.py's rank handling (the driver's multi-GPU SCALE run goes through it).

`python bench.py --gpus N` without a launcher must start N ranks itself (as
children, before any GPU call), and under a launcher the number of ranks must
equal --gpus.  The GPU case runs two ranks on one MI355X over gloo (RCCL
refuses two ranks on one device) and checks that the line reports two ranks
and that the all-gathered rows are every rank's accepted candidates."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def test_launcher_world_must_match_gpus():
    """Under a launcher with one rank, --gpus 2 is refused before the GPU is used."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "--gpus 2 but the launcher started 1 rank" in p.stderr


def test_gpus_must_be_positive():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "0"], cwd=REPO, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode != 0 and "--gpus must be >= 1" in p.stderr


@pytest.mark.gpu
def test_bench_two_ranks_self_launch():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "-u", BENCH, "--gpus", "2", "--backend", "gloo", "--n", "32768", "--steps", "3",
           "--warmup", "1", "--no-stage", "--no-ring", "--no-overlap", "--no-cpu-baseline", "--secondary-wid", "0"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["ranks_seen"] == 2
    assert sorted(r["rank"] for r in d["ranks"]) == [0, 1]
    assert d["backend"] == "gloo"
    assert d["config"]["global_batch"] == 2 * 32768
    assert len(d["accepted_per_rank"]) == 2 and min(d["accepted_per_rank"]) > 1000
    assert d["gathered_records"] == sum(d["accepted_per_rank"])
