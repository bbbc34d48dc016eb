import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def trace_blas_matches():
    """(same, description): whether this host's numpy BLAS is the one tests/golden/gs_trace.npz
    was recorded with (gs_trace_blas.json).  A TRF path is bit-reproducible only under the same
    OpenBLAS kernel choice, so bit-equality against that trace is asserted only then."""
    import json
    import threadpoolctl
    with open(os.path.join(GOLDEN, "gs_trace_blas.json")) as f:
        rec = json.load(f)
    here = [d for d in threadpoolctl.threadpool_info() if d.get("user_api") == "blas"]
    here = here[0] if here else {}
    keys = ("internal_api", "version", "architecture")
    same = all(here.get(k) == rec[k] for k in keys)
    return same, (f"this host: {[here.get(k) for k in keys]}, trace: {[rec[k] for k in keys]}")


@pytest.fixture(scope="session")
def ctx():
    from tsbb15_amd import _ffi
    return _ffi.default_context()
