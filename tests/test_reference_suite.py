"""The reference's own Python acceptance suite, run UNCHANGED against this package.

/root/reference/python/tests/test_sdfgen.py:15-1058 (51 tests: shapes, dtypes, signs, error
contracts, CPU vs GPU agreement) imports `sdfgen`; here that name resolves to this repository's
drop-in alias (sdfgen/__init__.py -> sdfgenfast_amd).  The file is read where it lies (never
copied); its conftest is not loaded (--noconftest: it only adds the reference checkout to
sys.path, python/tests/conftest.py:7-13), nothing is written under /root/reference (no bytecode,
no pytest cache), and the reference's pytest configuration is not read (-c /dev/null).  Skipped
where /root/reference is absent (the GPU box).  Without a GPU the suite's GPU tests skip
themselves (python/tests/test_sdfgen.py:268-298 check is_gpu_available()).

The file is third-party code from the reference checkout, so it runs only when its SHA-256 is the
one it was reviewed at (REF_TEST_SHA256): an edited or replaced file is skipped, never executed."""
import hashlib
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_TEST = "/root/reference/python/tests/test_sdfgen.py"
REF_TEST_SHA256 = "7a2d920a16277863d9f3eeb03a020229b5fcb1738af68076e51abf71726917cc"


@pytest.mark.skipif(not os.path.exists(REF_TEST), reason="the reference checkout is not present")
def test_reference_python_suite_passes_unchanged(tmp_path):
    with open(REF_TEST, "rb") as f:
        got = hashlib.sha256(f.read()).hexdigest()
    if got != REF_TEST_SHA256:
        pytest.skip(f"{REF_TEST} is not the reviewed version (sha256 {got[:16]}...): not executed")
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "--noconftest", "-p", "no:cacheprovider",
                        "-c", os.devnull, "--rootdir", str(tmp_path), REF_TEST],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    m = re.search(r"(\d+) passed", out)
    assert m and int(m.group(1)) >= 49, out[-2000:]
    assert "failed" not in out.splitlines()[-1], out[-2000:]
    # the suite imported THIS package under the reference's module name
    probe = subprocess.run([sys.executable, "-c", "import sdfgen, sdfgenfast_amd; "
                            "print(sdfgen.generate_sdf is sdfgenfast_amd.generate_sdf)"],
                           cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
    assert probe.stdout.strip() == "True", probe.stdout + probe.stderr
