"""The library's remaining environment knobs that change how work is scheduled
(not tracing, budget or debug checks), each run over the configs[4] pool
against the oracle.  An environment variable is read once
per process, so every case runs the configs[4] tests of test_gpu_edges.py in a
child process started with that environment, before any GPU call of its own:

  CAPJWT_ZC=1, CAPJWT_ZC_MAX   class-major zero-copy plans (jg_set_zero_copy's
                               initial setting; a 4096-job cap forces many plans)
  CAPJWT_TABLES_SYNC=1         key comb tables built at full width inside
                               jg_keys_load (no background widening)
  CAPJWT_CHUNK                 pipeline chunk size (an odd size: ragged chunks)
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    "zero_copy": {"CAPJWT_ZC": "1", "CAPJWT_ZC_MAX": "4096"},
    "tables_sync": {"CAPJWT_TABLES_SYNC": "1"},
    "chunk_1000": {"CAPJWT_CHUNK": "1000"},
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_config5_under_env(case):
    env = dict(os.environ, **CASES[case])
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
           "--timeout", "100", "--timeout-method", "thread",
           os.path.join(ROOT, "tests", "test_gpu_edges.py"), "-k", "config5"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, f"{case}: child failed\n{tail}"
    assert re.search(r"\b2 passed", r.stdout), tail
