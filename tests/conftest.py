import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gym-flock_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_runtest_setup(item):
    if os.environ.get("GF_ABORT_BT") == "1":  # debug aid: native backtrace on SIGABRT
        import ctypes  # (re)installed before every test: the runtimes may install their own
        ctypes.CDLL(os.path.join(ROOT, "scripts", "dbg", "libabort_bt.so")).gf_install_abort_bt()
