"""CPU: no LDS read in libmsunet_hip.so has its result registers read, copied, spilled or
overwritten before the s_waitcnt that covers it (tools/lds_hazard_check.py; VERDICT r3 item 6:
the inline-asm ``*_untracked`` reads of csrc/mfma_frag.h rely on the compiler never touching
those VGPRs before ``lds_wait_tie``).  The checker itself is first shown to catch the failure
forms on synthetic instruction streams."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import lds_hazard_check as chk  # noqa: E402


def _fn(*lines):
    return [(4 * i, mn, ops) for i, (mn, ops) in enumerate(lines)]


def test_checker_flags_copy_spill_and_overwrite_before_the_wait():
    read = ("ds_read_b64_tr_b16", " v[10:11], v90 offset:32")
    for bad in ((" v_mov_b32", " v5, v11"), ("scratch_store_dwordx2", " off, v[10:11], s33"),
                ("v_accvgpr_write_b32", " a3, v10"), ("v_add_u32", " v10, v1, v2")):
        f = _fn(read, (bad[0].strip(), bad[1]), ("s_waitcnt", " lgkmcnt(0)"), ("s_endpgm", ""))
        assert chk.check_function("k", f), bad


def test_checker_accepts_covered_reads():
    read = ("ds_read_b64_tr_b16", " v[10:11], v90")
    ok = _fn(read, ("v_mov_b32", " v5, v7"), ("s_waitcnt", " lgkmcnt(0)"), ("v_mov_b32", " v5, v10"),
             ("s_endpgm", ""))
    assert not chk.check_function("k", ok)
    # in-order DS completion: lgkmcnt(1) after one later DS op covers the first read
    ok2 = _fn(read, ("ds_read_b32", " v20, v91"), ("s_waitcnt", " lgkmcnt(1)"), ("v_mov_b32", " v5, v10"),
              ("s_waitcnt", " lgkmcnt(0)"), ("v_mov_b32", " v6, v20"), ("s_endpgm", ""))
    assert not chk.check_function("k", ok2)
    # ... but not lgkmcnt(2) (the read may still be in flight)
    bad = _fn(read, ("ds_read_b32", " v20, v91"), ("s_waitcnt", " lgkmcnt(2)"), ("v_mov_b32", " v5, v10"),
              ("s_endpgm", ""))
    assert chk.check_function("k", bad)


def test_checker_follows_branches():
    read = ("ds_read_b32", " v10, v90")
    # the fall-through path waits, the branch target reads v10 first
    f = _fn(read, ("s_cbranch_scc1", " 2 // <k+0x10>"), ("s_waitcnt", " lgkmcnt(0)"), ("s_endpgm", ""),
            ("v_mov_b32", " v1, v10"), ("s_endpgm", ""))
    assert chk.check_function("k", f)


def test_library_has_no_lds_read_hazards():
    lib = chk.DEFAULT_LIB
    if not os.path.exists(lib) or not os.path.exists(chk.OBJDUMP):
        pytest.skip("library not built / llvm-objdump missing")
    n, bad = chk.check_library(lib)
    assert n > 10000, n  # the disassembly was parsed
    assert not bad, bad[:10]
