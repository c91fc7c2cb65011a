"""bench.py's N-rank launch without a launcher (`python3 bench.py --gpus N`
with no WORLD_SIZE spawns its rank processes itself, before any GPU call) and
the N>1 line's per-rank telemetry, on CPU: gloo ranks with synthetic times."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3])
def test_bench_spawns_its_ranks_and_reports_each(world):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--launch-selftest"],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == world
    assert [p["rank"] for p in d["per_rank_ms"]] == list(range(world))
    assert [p["render_span_ms"] for p in d["per_rank_ms"]] == [1.0 + r for r in range(world)]
    assert d["slowest_rank"] == world - 1
    assert d["gather_ms"]["max"] == 0.25 * world
    assert d["max_wall"] == 2.0 + world - 1 and d["sum_rays"] == 10.0 * world


def test_bench_rank_failure_stops_the_launch():
    """A rank that cannot start (bad argument) makes the launch fail, not hang."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "nope"],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode != 0


def test_inflight_default():
    """Frames in flight when --inflight is not given: 2, and 3 for the C3
    scenes' strong-scaling shares at >= 4 ranks (bench.inflight_default)."""
    import argparse
    sys.path.insert(0, ROOT)
    import bench

    def ns(**kw):
        d = dict(config="c3", rows=None, accel="bvh", scaling="strong")
        d.update(kw)
        return argparse.Namespace(**d)

    assert bench.inflight_default(ns(), 1) == 2
    assert bench.inflight_default(ns(), 2) == 2
    assert bench.inflight_default(ns(), 4) == 3
    assert bench.inflight_default(ns(), 8) == 3
    assert bench.inflight_default(ns(config="c3cone"), 8) == 3
    assert bench.inflight_default(ns(config="c4"), 8) == 2
    assert bench.inflight_default(ns(config="c4csg"), 8) == 2
    assert bench.inflight_default(ns(scaling="weak"), 8) == 2
    assert bench.inflight_default(ns(accel="none"), 8) == 2
