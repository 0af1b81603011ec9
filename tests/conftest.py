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
