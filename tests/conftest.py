import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")
    # the oracle is test infrastructure; build it if a fresh checkout lacks it
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session")
def golden():
    import json
    from oracle import jws
    d = os.path.join(ROOT, "tests", "golden")
    keys_raw = json.load(open(os.path.join(d, "keys.json")))
    toks = json.load(open(os.path.join(d, "tokens.json")))
    keys = {k["kid"]: jws.Key.from_fixture(k) for k in keys_raw}
    return {"keys": keys, "keys_raw": keys_raw, "tokens": toks}


def pytest_sessionstart(session):
    """A GPU session (-m gpu) runs with the key-memory lifetime check on
    (include/jg.h jg_debug_lifetime_check): every key generation released
    during the suite must find the work of every stream that used it done;
    tests/test_gpu_zz_lifetime.py (the last GPU module) asserts the count."""
    if (session.config.getoption("markexpr", "") or "").strip() == "gpu":
        from cap_amd import _lib
        _lib.lifetime_check(1)
