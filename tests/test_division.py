"""The correctly rounded quotient the closest-hit kernels use for sphere roots.

rt_kernels.hip div_ia computes x / a from ia = RN(1/a) (one true division
per ray) with two fma residual steps (Markstein); sphere_test relies on it
being the IEEE quotient of geometry.scm:160-170's `(/ (- (- b) sq) a)`.
This host build of the same operations (tests/csrc/div_ia_check.c, gcc,
-ffp-contract=off) checks it against x / a on random operands across the
exponent range, including near-1 and all-ones-significand divisors.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("div") / "div_ia_check")
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                           os.path.join(HERE, "csrc", "div_ia_check.c"), "-lm"])
    return exe


@pytest.mark.parametrize("seed", ["0x9E3779B97F4A7C15", "0x5EED0002", "0x123456789"])
def test_div_ia_is_the_ieee_quotient(checker, seed):
    r = subprocess.run([checker, "4000000", seed], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0 of 4000000" in r.stdout
