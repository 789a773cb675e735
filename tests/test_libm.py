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


@pytest.mark.gpu
def test_depth_estimate_log_at_powers_of_four():
    """bez_maxd (rt_kernels.hip) takes ceiling((log z) / (log 4)) with the device's log (OCML), the
    reference (bezier.scm:179-192) with the C library's.  At exact powers of 4 both quotients must sit on
    the integer for every depth the walk supports ("libm"); elsewhere the two logs may
    differ by an ulp, and the test reports how often.  torch's f64 log on ROCm is the same OCML function
    the kernels call."""
    import math

    import numpy as np
    import torch
    ks = list(range(-200, 29))
    z = torch.tensor([4.0 ** k for k in ks], dtype=torch.float64, device="cuda")
    l4 = torch.log(torch.tensor([4.0], dtype=torch.float64, device="cuda"))
    assert float(l4.item()) == math.log(4.0)
    q = (torch.log(z) / l4).cpu().numpy()
    assert [math.ceil(v) for v in q] == ks
    assert [math.ceil(math.log(4.0 ** k) / math.log(4.0)) for k in ks] == ks
    rng = np.random.default_rng(7)
    x = np.exp(rng.uniform(-30.0, 30.0, 200000))
    dev = torch.log(torch.from_numpy(x).cuda()).cpu().numpy()
    host = np.array([math.log(v) for v in x])
    print("log: %d of %d arguments differ from the host library" % (int((dev != host).sum()), x.size))
    assert np.all(np.abs(dev - host) <= 2.0 * np.spacing(np.abs(host)))
