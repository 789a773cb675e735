import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "scheme-raytrace_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def host_threads():
    """Threads for the oracle on this host: the process's CPU share (a GPU box
    gives a one-GPU job 16 CPUs of a much larger machine; os.cpu_count()
    reports the machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 64))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    from rtamd import gpu
    if gpu.device_count() < 1:
        pytest.fail("no HIP device visible for a gpu-marked test")
    return gpu.default_context(0)


@pytest.fixture
def sched(gpu_ctx):
    """The default context with its render-schedule options (rt_context_set_option)
    at their automatic values, restored after the test."""
    gpu_ctx.reset_options()
    yield gpu_ctx
    gpu_ctx.reset_options()
