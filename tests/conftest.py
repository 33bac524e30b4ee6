import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# specialized-kernel code objects of the policy sets the tests compile: built ahead of time
# on the CPU (tools/jit_warm.sh; hiprtc needs no GPU) and shipped in-tree with libkvgpu.so
os.environ.setdefault("KVGPU_JIT_CACHE", os.path.join(ROOT, "kyverno_amd", "jitcache"))
# every ingest in the suite checks that each 8-byte transfer cell rebuilds its Node bit for bit
# (kvcell.h; the device's kv_expand_rows_kernel decodes the same form)
os.environ.setdefault("KVGPU_CHECK_CELLS", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.build()
    return oracle.get()
