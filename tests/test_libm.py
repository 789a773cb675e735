"""The device's sin / cos (scheme-raytrace_amd/csrc/rt_libm.h) against the C
library the reference runtime and the oracle use, bit for bit, on the host:
the same header compiled by g++ ("libm")."""
import os
import subprocess

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
