"""The device's sin / cos (scheme-raytrace_amd/csrc/rt_libm.h) against the C
library the reference runtime and the oracle use, bit for bit, on the host:
the same header compiled by g++ ("libm")."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_sin_cos_restatement_matches_host_libm(tmp_path):
    exe = str(tmp_path / "libm_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin", "-o", exe,
                           os.path.join(HERE, "csrc", "libm_check.cpp"), "-lm"])
    out = subprocess.run([exe, "3000000"], capture_output=True, text=True, check=True).stdout.strip().splitlines()
    total, bad_sin, bad_cos = (int(x) for x in out[-1].split())
    print("\n".join(out[-4:]))
    assert total > 9000000
    assert bad_sin == 0 and bad_cos == 0, out


def _depth_cases():
    """Ray-space curves whose depth estimate z = sqrt(2) n (n-1) l0 / (8 eps) (bezier.scm:179-192, n = 4)
    lands exactly on a power of 4 and on its neighbours: p0 = p1 = 0, p2 = (l0, 0), p3 = (2 l0, 0) give
    l0 exactly, and l0 is searched ulp by ulp so that the f64 expression the kernels evaluate (the same
    operation order, no contraction) yields 4^k, or the doubles just below / above it.  Plus random l0
    over 40 decades and a flat curve (l0 = 0: log -inf, depth 0)."""
    import math

    import numpy as np
    c = (1.4142135623730951 * 4.0) * 3.0
    cps, eps, kinds = [], [], []

    def add(l0, e8, kind):
        cps.append([0, 0, 1, 0, 0, 1, l0, 0, 1, 2 * l0, 0, 1])
        eps.append(e8)
        kinds.append(kind)

    for e8 in (1.0, 0.4, 8 * (0.5 / 20)):
        for k in range(-60, 27):
            target = 4.0 ** k
            l0 = target * e8 / c
            for _ in range(64):
                l0 = math.nextafter(l0, -math.inf)
            for _ in range(128):
                z = (c * l0) / e8
                if z == target:
                    add(l0, e8, "4^%d" % k)
                elif z == math.nextafter(target, -math.inf) or z == math.nextafter(target, math.inf):
                    add(l0, e8, "4^%d +- 1 ulp" % k)
                l0 = math.nextafter(l0, math.inf)
    rng = np.random.default_rng(5)
    for l0 in np.exp(rng.uniform(-40.0, 40.0, 50000)):
        add(float(l0), 1.0, "random")
    add(0.0, 1.0, "flat")
    return np.array(cps, dtype=np.float64), np.array(eps), kinds


def _host_depth(cps, e8):
    """bez_maxd's result with the C library's log: ceiling((log z) / (log 4)), 0 at -inf, saturated at 25."""
    import math
    l0 = max(abs(cps[0] - 2 * cps[3] + cps[6]), abs(cps[1] - 2 * cps[4] + cps[7]),
             abs(cps[3] - 2 * cps[6] + cps[9]), abs(cps[4] - 2 * cps[7] + cps[10]))
    z = (((1.4142135623730951 * 4.0) * 3.0) * l0) / e8
    if z == 0.0:
        return 0
    md = math.log(z) / math.log(4.0)
    return 25 if md > 25.0 else math.ceil(md)


def test_depth_cases_cover_powers_of_four():
    """The probe's inputs (CPU): for most k the search finds an l0 whose z is exactly 4^k, and the host
    library's quotient is then exactly k ("libm")."""
    cps, eps, kinds = _depth_cases()
    exact = [i for i, k in enumerate(kinds) if k.startswith("4^") and "ulp" not in k]
    assert len(exact) > 150
    for i in exact:
        k = int(kinds[i][2:])
        assert _host_depth(cps[i], eps[i]) == min(k, 25), kinds[i]


@pytest.mark.gpu
def test_curve_depth_estimate_matches_host_libm(gpu_ctx):
    """The curve kernels' own depth estimate (bez_maxd, through rt_curve_depth_probe) against
    ceiling((log z) / (log 4)) with the host's C library (the reference runtime's log), at exact powers of
    4, their 1-ulp neighbours and random flatness: the device's log (OCML) must give the same ceiling in
    every case (bezier.scm:179-192)."""
    from rtamd import gpu
    cps, eps, kinds = _depth_cases()
    dev = gpu.curve_depth_probe(cps, eps, ctx=gpu_ctx)
    host = [_host_depth(cps[i], eps[i]) for i in range(len(kinds))]
    bad = [(kinds[i], int(dev[i]), host[i]) for i in range(len(kinds)) if int(dev[i]) != host[i]]
    print("depth estimate: %d cases (%d at powers of 4 or their neighbours), %d differ: %s"
          % (len(kinds), sum(1 for k in kinds if k.startswith("4^")), len(bad), bad[:8]))
    assert not bad
