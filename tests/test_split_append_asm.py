"""The split append (sweep_sparse.hpp SP_SPLIT_APPEND) issues a returning atomic from inline asm and
waits for it later with a manual s_waitcnt: the compiler's wait-count pass does not see it, so its
safety is checked on the ISA of every build.  tools/check_split_append.py walks every
control-flow path from the asm atomic to the first `s_waitcnt vmcnt(0)` and fails if an instruction
on the way names the atomic's destination VGPRs.  Runs on CPU (hipcc cross-compiles gfx950)."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_split_append as C  # noqa: E402

HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)


def _check_text(asm: str):
    lines = asm.strip("\n").splitlines()
    total, probs = 0, []
    for name, body in C.functions(lines):
        n, p = C.check_function(name, body)
        total += n
        probs += p
    return total, probs


SAFE = """
_Zk:
\t;;#ASMSTART
\tglobal_atomic_add_x2 v[4:5], v[2:3], v[0:1], off sc0
\ts_nop 1
\t;;#ASMEND
.LBB0_1:
\tv_add_u32_e32 v6, 1, v6
\ts_cbranch_vccz .LBB0_1
\ts_waitcnt vmcnt(0)
\tv_mov_b32_e32 v7, v4
\ts_endpgm
.Lfunc_end0:
"""


def test_checker_accepts_a_wait_on_every_path():
    assert _check_text(SAFE) == (1, [])


def test_checker_flags_a_read_before_the_wait():
    n, probs = _check_text(SAFE.replace("\tv_add_u32_e32 v6, 1, v6", "\tv_mov_b32_e32 v6, v5"))
    assert n == 1 and len(probs) == 1 and "v[5]" in probs[0]


def test_checker_flags_a_branch_path_that_skips_the_wait():
    bad = SAFE.replace("\ts_cbranch_vccz .LBB0_1\n\ts_waitcnt vmcnt(0)",
                       "\ts_cbranch_vccz .LBB0_2\n\ts_waitcnt vmcnt(0)\n.LBB0_2:\n\tv_mov_b32_e32 v8, v4")
    n, probs = _check_text(bad)
    assert n == 1 and probs and "v[4]" in probs[0]


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_built_kernels_have_no_split_append_hazard():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sdfgenfast_amd"), "asm"], check=True,
                   capture_output=True, timeout=900)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_split_append.py"),
                        os.path.join(ROOT, "sdfgenfast_amd", "build", "sdfgen_hip.s")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("every path waits") == 2   # k_sp_recheck<false> and <true> (Z-slab)
