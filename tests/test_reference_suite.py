"""The reference repository's own tests/, unmodified, against this rebuild
(``scripts/run_reference_tests.py``).  Runs when a local read-only checkout of
the reference exists (``REFERENCE_DIR``, default /root/reference); skipped
otherwise — nothing is fetched."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("REFERENCE_DIR", "/root/reference")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "tests")), reason="no local reference checkout")
def test_reference_suite_passes_unmodified():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "run_reference_tests.py"), "--reference", REF],
                       capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in tail and "failed" not in tail, tail
