import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "audio-mastering-engine_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_report_header(config):
    """build provenance: the source hash of this tree and the one stamped into the
    libamx.so the tests will load (capi.load refuses a mismatch)"""
    try:
        from amx import build
        return ["amx sources sha256 %s, libamx.so stamp %s" % (build.source_hash(), build.built_hash())]
    except Exception as e:   # noqa: BLE001 -- a header must not break collection
        return ["amx provenance unavailable: %s" % e]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from amx import build
    build.build()
    return torch.device("cuda:0")
