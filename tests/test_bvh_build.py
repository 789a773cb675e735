"""The scene commit's BVH build on host threads (scheme-raytrace_amd/csrc/rt_bvh.h, round 6) against the
serial build: the same tree bit for bit — node array, primitive order, BVH2 layout, BVH4 collapse — on C5's
curve generator (points->bezier polylines, points.scm:28-50) and on a sphere cloud.  Host only: the build
is compiled with g++ from the library's own header (tests/csrc/bvh_check.cpp); no GPU."""
import json
import os
import subprocess

import numpy as np
import pytest

from rtamd import scenes

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def bvh_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bvh") / "bvh_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-ffp-contract=off", "-o", exe,
                           os.path.join(HERE, "csrc", "bvh_check.cpp")])
    return exe


def _curve_boxes(n, width):
    """commit_scene's curve boxes: control points +- width / 2 (bezier.scm:88-98), type LEAF_BEZIER (5)."""
    cp = np.asarray(scenes.random_polyline_curves(n), dtype=np.float64).reshape(n, 4, 3)
    w1 = abs(width / 2)
    out = np.zeros((n, 7))
    out[:, 0:3] = cp.min(axis=1) - w1
    out[:, 3:6] = cp.max(axis=1) + w1
    out[:, 6] = 5
    return out


def _run(exe, boxes, path, threads, sweep=None):
    boxes.astype(np.float64).tofile(path)
    args = [exe, str(path), str(threads)] + ([str(sweep)] if sweep is not None else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    print(r.stdout.strip())
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout)


def test_threaded_curve_bvh_equals_serial(bvh_check, tmp_path):
    """2^18 curves: binned top levels over sweep levels with the centroid orders passed down, and a BVH2
    large enough (>= 65 536 inner nodes) for the threaded BVH4 collapse."""
    res = _run(bvh_check, _curve_boxes(1 << 18, 0.5), tmp_path / "c.bin", 8)
    assert res["nodes"] >= 2 * 65536
    assert res["same_nodes"] and res["same_order"] and res["same_bvh2"] and res["same_bvh4"]


def test_threaded_build_binned_top_and_spheres(bvh_check, tmp_path):
    """Binned SAH above a small sweep threshold (so the threads split binned levels too), and spheres with
    duplicated centres (ties in the sweep's stable sort)."""
    _run(bvh_check, _curve_boxes(1 << 15, 3.0), tmp_path / "c.bin", 5, sweep=4096)
    rs = np.random.default_rng(7)
    c = rs.uniform(-50, 50, size=(20000, 3))
    c[10000:] = c[:10000]                                # every sphere twice
    r = rs.uniform(0.1, 2.0, size=(20000, 1))
    boxes = np.concatenate([c - r, c + r, np.zeros((20000, 1))], axis=1)
    res = _run(bvh_check, boxes, tmp_path / "s.bin", 3)
    assert res["same_nodes"] and res["same_order"] and res["same_bvh2"] and res["same_bvh4"]


def test_sweep_orders_with_ties_below_binned_levels(bvh_check, tmp_path):
    """Every centroid three times (ties on all axes) and centroids on a coarse grid (ties on one axis at a
    time), binned above 4096 primitives: the sweep roots sort, their subtrees split the sorted orders and
    re-order tied runs by position — the stable sort's order at every node."""
    rs = np.random.default_rng(11)
    c = np.round(rs.uniform(-40, 40, size=(50000, 3)) * 4) / 4
    c = np.concatenate([c, c, c])
    r = rs.uniform(0.1, 1.0, size=(150000, 1))
    boxes = np.concatenate([c - r, c + r, np.zeros((150000, 1))], axis=1)
    res = _run(bvh_check, boxes, tmp_path / "t.bin", 6, sweep=4096)
    assert res["same_nodes"] and res["same_order"] and res["same_bvh2"] and res["same_bvh4"]
