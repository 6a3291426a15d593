"""Static check of the gfx950 code in libmsunet_hip.so for LDS reads whose result registers are
touched before the wait that covers them.

The weight-gradient / conv / token-GEMM kernels read LDS-DMA rings with inline-asm ``ds_read*``
(csrc/mfma_frag.h ``*_untracked``): the compiler does not know those registers are still being
written when the asm "returns", so it could copy (``v_mov``, ``v_accvgpr_write``), spill
(``scratch_store``), reuse or overwrite them before the covering ``s_waitcnt lgkmcnt``.  The
round-3 fault of an ablation build that staged global loads the same way
(profiles/r03ad_linbwd_ablation_untracked.txt) is that failure mode.

For EVERY LDS read in the library (tracked reads pass trivially: the compiler waits before
using them) the checker walks the code that can follow it -- fall-through and both sides of
each branch -- until an ``s_waitcnt`` whose ``lgkmcnt(N)`` provably covers the read (N = 0, or
N <= the DS operations issued after it with no scalar-memory load in between: DS operations
complete in order).  Any instruction on the way that names one of the destination registers
(read, write or spill) is reported.

    python tools/lds_hazard_check.py [lib.so]      # prints violations, exit 1 if any
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"
HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(os.path.dirname(HERE), "semantic_segmentation_of_stylegan2_artifacts_amd",
                           "libmsunet_hip.so")

FUNC_RE = re.compile(r"^([0-9a-f]+) <(.+)>:$")
INSN_RE = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-F]+):")
TARGET_RE = re.compile(r"<(.+)\+0x([0-9a-f]+)>")
REG_RANGE_RE = re.compile(r"\b([va])\[(\d+):(\d+)\]")
REG_ONE_RE = re.compile(r"\b([va])(\d+)\b")
LGKM_RE = re.compile(r"lgkmcnt\((\d+)\)")


def extract_code_objects(lib, workdir):
    """The gfx950 code objects bundled in lib, extracted into workdir (objdump writes its
    extracted bundles next to its input, so it runs on a copy)."""
    copy = os.path.join(workdir, "lib.so")
    shutil.copy(lib, copy)
    subprocess.run([OBJDUMP, "--offloading", copy], cwd=workdir, check=True, capture_output=True)
    return sorted(os.path.join(workdir, f) for f in os.listdir(workdir) if f.endswith("gfx950"))


def disassemble(obj):
    r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", obj], check=True, capture_output=True, text=True)
    return r.stdout.splitlines()


def regs(text):
    out = set()
    for kind, a, b in REG_RANGE_RE.findall(text):
        out.update((kind, i) for i in range(int(a), int(b) + 1))
    text = REG_RANGE_RE.sub(" ", text)
    out.update((kind, int(i)) for kind, i in REG_ONE_RE.findall(text))
    return out


def functions(lines):
    """{name: [(addr, mnemonic, operands)]} of every function in a disassembly."""
    funcs, cur = {}, None
    for ln in lines:
        m = FUNC_RE.match(ln)
        if m:
            cur = funcs.setdefault(m.group(2), [])
            continue
        if cur is None:
            continue
        m = INSN_RE.match(ln)
        if m:
            cur.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return funcs


def is_ds(mn):
    return mn.startswith("ds_")


def is_smem(mn):
    return mn.startswith("s_load") or mn.startswith("s_buffer_load") or mn.startswith("s_memtime") or \
        mn.startswith("s_sendmsg") or mn.startswith("s_dcache") or mn.startswith("s_scratch_load")


def is_lds_read(mn):
    return mn.startswith("ds_read") or mn.startswith("ds_load")


def check_function(name, insns, max_steps=4000):
    """Violations [(function, read index, read text, offending index, offending text)]."""
    if not insns:
        return []
    index = {a: i for i, (a, _, _) in enumerate(insns)}
    out = []
    for i, (addr, mn, ops) in enumerate(insns):
        if not is_lds_read(mn):
            continue
        dest = regs(ops.split(",")[0])
        if not dest:
            continue
        # DFS over (insn index, ds ops issued since, smem seen)
        stack = [(i + 1, 0, False)]
        seen = set()
        steps = 0
        while stack:
            j, nds, smem = stack.pop()
            while j < len(insns):
                if (j, nds if nds < 16 else 16, smem) in seen:
                    break
                seen.add((j, nds if nds < 16 else 16, smem))
                steps += 1
                if steps > max_steps:
                    out.append((name, i, f"{mn}{ops}", j, "walk limit reached without a covering wait"))
                    stack = []
                    break
                a2, m2, o2 = insns[j]
                if m2 == "s_waitcnt":
                    mm = LGKM_RE.search(o2)
                    if mm is not None:
                        n = int(mm.group(1))
                        if n == 0 or (not smem and n <= nds):
                            break  # covered on this path
                    j += 1
                    continue
                if regs(o2) & dest:
                    out.append((name, i, f"{mn}{ops}", j, f"{m2}{o2}"))
                    break
                if is_ds(m2):
                    nds += 1
                elif is_smem(m2):
                    smem = True
                if m2 in ("s_endpgm", "s_setpc_b64", "s_trap") or m2.startswith("s_endpgm"):
                    break
                if m2.startswith("s_branch") or m2.startswith("s_cbranch"):
                    # target printed as <symbol+0xOFF>: OFF from the function's first instruction
                    mt = TARGET_RE.search(o2)
                    tgt = None if mt is None else index.get(insns[0][0] + int(mt.group(2), 16))
                    if tgt is not None:
                        stack.append((tgt, nds, smem))
                    if m2.startswith("s_branch"):
                        break
                j += 1
    return out


def check_library(lib=DEFAULT_LIB):
    """(number of LDS reads checked, violations)."""
    work = tempfile.mkdtemp(prefix="msu_lds_")
    try:
        nreads, bad = 0, []
        for obj in extract_code_objects(lib, work):
            for name, insns in functions(disassemble(obj)).items():
                nreads += sum(1 for _, mn, _ in insns if is_lds_read(mn))
                bad += check_function(name, insns)
        return nreads, bad
    finally:
        shutil.rmtree(work, ignore_errors=True)


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB
    n, bad = check_library(lib)
    for name, i, rd, j, what in bad[:50]:
        print(f"{name}: read #{i} `{rd.strip()}` -> insn #{j} `{what.strip()}`")
    print(f"{n} LDS reads checked, {len(bad)} violations")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
