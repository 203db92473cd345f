import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session", params=["group", "pipeline"])
def ctx(request):
    """A verifier context, once per execution shape of the per-signature
    entry points: "group" = the default (batches of up to CESS_BLS_SMALL_BATCH
    records run k_group, one signature per wave), "pipeline" = the
    one-lane-per-signature six-kernel pipeline for every batch size
    (CESS_BLS_SMALL_BATCH=0, read when the context is created)."""
    from cess_amd import bls
    old = os.environ.get("CESS_BLS_SMALL_BATCH")
    if request.param == "pipeline":
        os.environ["CESS_BLS_SMALL_BATCH"] = "0"
    else:
        os.environ.pop("CESS_BLS_SMALL_BATCH", None)
    try:
        c = bls.Context(max_batch=1 << 16)
    finally:
        if old is None:
            os.environ.pop("CESS_BLS_SMALL_BATCH", None)
        else:
            os.environ["CESS_BLS_SMALL_BATCH"] = old
    yield c
    c.close()
