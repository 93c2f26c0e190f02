"""tools/asm_audit.py on small hand-written device-asm windows: it must flag a compiler
instruction that touches an outstanding inline-asm ds_read's registers (on either path of a branch), and an
asm rewrite of an MFMA operand too soon after that MFMA, and pass the ordered window."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import asm_audit  # noqa: E402

HEAD = "_Zkernel:\n"
TAIL = ".Lfunc_end0:\n"

# two asm reads, their waits, the MFMAs that use them, and a rewrite of the first set four MFMAs later
ORDERED = """\
\t;;#ASMSTART
\tds_read_b128 v[0:3], v20
\tds_read_b128 v[4:7], v20 offset:1024
\t;;#ASMEND
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(1)
\t;;#ASMEND
\tv_mfma_f64_16x16x4_f64 v[40:47], v[0:1], v[2:3], v[40:47]
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(0)
\t;;#ASMEND
\tv_mfma_f64_16x16x4_f64 v[48:55], v[4:5], v[6:7], v[48:55]
\tv_mfma_f64_16x16x4_f64 v[56:63], v[4:5], v[6:7], v[56:63]
\tv_mfma_f64_16x16x4_f64 v[64:71], v[4:5], v[6:7], v[64:71]
\tv_mfma_f64_16x16x4_f64 v[72:79], v[4:5], v[6:7], v[72:79]
\t;;#ASMSTART
\tds_read_b128 v[0:3], v20 offset:2048
\t;;#ASMEND
\ts_endpgm
"""


def audit(body, tmp_path):
    p = tmp_path / "k.s"
    p.write_text(HEAD + body + TAIL)
    ((_, items),) = list(asm_audit.functions(str(p)))
    nreads, nviol, _, close = asm_audit.audit_fn(items)
    return nreads, nviol, len(close)


def test_ordered_window_passes(tmp_path):
    assert audit(ORDERED, tmp_path) == (3, 0, 0)


def test_copy_before_the_wait_on_one_branch_is_flagged(tmp_path):
    # posterior_cov_big_kernel's round-5 one-word chunk path: a register copy before the asm wait, on one branch
    body = """\
\t;;#ASMSTART
\tds_read_b128 v[0:3], v20
\t;;#ASMEND
\ts_cbranch_scc0 .LBB0_2
; %bb.1:
\tv_mov_b64_e32 v[8:9], v[0:1]
.LBB0_2:
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(0)
\t;;#ASMEND
\ts_endpgm
"""
    assert audit(body, tmp_path)[1] == 1


def test_mfma_before_the_wait_is_flagged(tmp_path):
    body = ORDERED.replace("\t;;#ASMSTART\n\ts_waitcnt lgkmcnt(1)\n\t;;#ASMEND\n", "", 1)
    assert audit(body, tmp_path)[1] >= 1


def test_rewrite_right_after_its_mfma_is_flagged(tmp_path):
    # the second set rewritten right after its own MFMAs (round 5's changed results)
    body = ORDERED.replace("ds_read_b128 v[0:3], v20 offset:2048", "ds_read_b128 v[4:7], v20 offset:2048")
    assert audit(body, tmp_path)[2] == 4  # all four MFMAs reading v[4:7] are within 16 wait states
    # sixteen wait states between (s_nop 7 = 8) make it legal
    fixed = body.replace("\t;;#ASMSTART\n\tds_read_b128 v[4:7], v20 offset:2048",
                         "\ts_nop 7\n\ts_nop 7\n\t;;#ASMSTART\n\tds_read_b128 v[4:7], v20 offset:2048")
    assert audit(fixed, tmp_path)[2] == 0
    # so does a barrier
    barrier = body.replace("\t;;#ASMSTART\n\tds_read_b128 v[4:7], v20 offset:2048",
                           "\ts_barrier\n\t;;#ASMSTART\n\tds_read_b128 v[4:7], v20 offset:2048")
    assert audit(barrier, tmp_path)[2] == 0


def test_loop_back_edge_is_followed(tmp_path):
    # a rewrite at the top of a loop whose last MFMA read the same registers: found through the back edge
    body = """\
.LBB0_1:
\t;;#ASMSTART
\tds_read_b128 v[0:3], v20
\t;;#ASMEND
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(0)
\t;;#ASMEND
\tv_mfma_f64_16x16x4_f64 v[40:47], v[0:1], v[2:3], v[40:47]
\ts_cbranch_scc1 .LBB0_1
\ts_endpgm
"""
    assert audit(body, tmp_path)[2] == 1


def test_cli_exit_codes(tmp_path):
    good = tmp_path / "good.s"
    good.write_text(HEAD + ORDERED + TAIL)
    bad = tmp_path / "bad.s"
    bad.write_text(HEAD + ORDERED.replace("\t;;#ASMSTART\n\ts_waitcnt lgkmcnt(1)\n\t;;#ASMEND\n", "", 1) + TAIL)
    tool = os.path.join(REPO, "tools", "asm_audit.py")
    r = subprocess.run([sys.executable, tool, str(good)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "asm audit: OK" in r.stdout
    r = subprocess.run([sys.executable, tool, str(bad)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
