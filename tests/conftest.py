import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libmgpileup.so")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")


@pytest.fixture(scope="session")
def oracle_lib():
    from mgatk2_amd.build import build_oracle

    build_oracle()
    from oracle import oracle

    return oracle


@pytest.fixture(scope="session")
def engine_lib():
    """The HIP engine; the GPU tests fail (not skip) when it cannot load."""
    from mgatk2_amd.build import ENGINE_SO
    from mgatk2_amd import engine

    assert ENGINE_SO.exists(), "libmgpileup.so not built (run __graft_entry__.build())"
    engine.load_library()
    n = engine.device_count()
    assert n >= 1, "no HIP device visible"
    return engine
