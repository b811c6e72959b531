"""The C-ABI under host AddressSanitizer (tests/asan: every library source with its host
side instrumented, driven by capi_asan.cpp). On CPU: argument validation and the
no-device path. On an MI355X (-m gpu): also a FlockingRelative / Flocking-v0 / variant,
Coverage + greedy expert and graph-helper session through the host-pointer entry points,
so ASan checks every host buffer the library reads or writes."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "asan", "capi_asan")


def _run():
    if not os.path.exists(BIN):  # build() makes it; build here only if it is missing
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "asan")], check=True,
                       stdout=subprocess.DEVNULL)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    return subprocess.run([BIN], capture_output=True, text=True, timeout=300, env=env)


def test_capi_host_asan_cpu():
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible: the -m gpu variant runs the full session")
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi_asan: ok" in r.stdout


@pytest.mark.gpu
def test_capi_host_asan_gpu():
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "device present" in r.stdout and "capi_asan: ok" in r.stdout
