"""CPU check of the shipped machine code: no packed-fp32 broadcast product.

Round 5 localised the deformation backward's co-residency corruption to one instruction form, the
packed fp32 product whose both result halves take A.lo x B.hi,
    v_pk_mul_f32 vD, vA, vB op_sel:[0,1] op_sel_hi:[0,1]
(the SLP vectorizer formed it for the bilinear weights of features_to_lds): every build containing it
was corrupt under two co-resident blocks, every build without it clean.  The containment is that no
shipped unit contains it (deform.o is built with -fno-slp-vectorize; the other units' packed ops are
other forms).  A compiler update or an SLP-on edit could bring the form back silently, so this test
disassembles every gfx950 code object in the built libraries and fails if any packed fp32 op
(v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32) carries that operand selection."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin/llvm-objdump"
LIBS = [os.path.join(ROOT, "4dlangsplat_amd", "build", "liblsr.so"),
        os.path.join(ROOT, "4dlangsplat_amd", "build", "variants", "liblsr_ldspoison.so")]
# both halves of the first operand from its low half, of the second from its high half (omitted fields
# default to op_sel [0,0], op_sel_hi [1,1]); a third (fma) operand's bit may be anything
BROADCAST = re.compile(r"\bv_pk_(mul|add|fma)_f32\b[^\n]*\bop_sel:\[0,1(,[01])?\] op_sel_hi:\[0,1(,[01])?\]")
PACKED = re.compile(r"\bv_pk_(mul|add|fma)_f32\b")


def disassemble(lib, tmp):
    """Every gfx950 code object bundled in `lib`, disassembled: {bundle name: text}."""
    work = tmp / os.path.basename(lib)
    work.mkdir()
    shutil.copy(lib, work / "lib.so")
    subprocess.run([LLVM, "--offloading", "lib.so"], cwd=work, check=True, capture_output=True)
    out = {}
    for f in sorted(os.listdir(work)):
        if f.endswith("gfx950"):
            r = subprocess.run([LLVM, "-d", "--mcpu=gfx950", f], cwd=work, check=True, capture_output=True, text=True)
            out[f] = r.stdout
    return out


@pytest.mark.skipif(not os.path.exists(LLVM), reason="ROCm llvm-objdump not installed")
@pytest.mark.parametrize("lib", LIBS, ids=["liblsr", "ldspoison"])
def test_no_packed_broadcast_product_in_shipped_code(lib, tmp_path):
    assert os.path.exists(lib), f"{lib} not built (run __graft_entry__.build())"
    objs = disassemble(lib, tmp_path)
    assert len(objs) >= 8, sorted(objs)                       # every unit with device code
    assert sum(len(PACKED.findall(t)) for t in objs.values()) > 1000   # the census sees the compositors' ops
    bad = {f: [ln.strip() for ln in t.splitlines() if BROADCAST.search(ln)][:5] for f, t in objs.items()}
    bad = {f: v for f, v in bad.items() if v}
    assert not bad, bad


def test_pattern_matches_the_faulting_form():
    """The regex recognises the disassembler's spelling of the form (and not the shipped forms)."""
    assert BROADCAST.search("v_pk_mul_f32 v[2:3], v[2:3], v[8:9] op_sel:[0,1] op_sel_hi:[0,1]")
    assert BROADCAST.search("v_pk_fma_f32 v[2:3], v[4:5], v[8:9], v[2:3] op_sel:[0,1,0] op_sel_hi:[0,1,1]")
    assert not BROADCAST.search("v_pk_mul_f32 v[2:3], v[4:5], v[8:9] op_sel_hi:[1,0]")
    assert not BROADCAST.search("v_pk_mul_f32 v[2:3], v[4:5], v[8:9] op_sel:[0,1] op_sel_hi:[0,0]")


def test_pc_relative_sequences_are_unbroken(tmp_path):
    """The -amdgpu-waitcnt-forcezero fault, found in round 6: a PC-relative address is
    s_getpc_b64 s[n:n+1]; s_add_u32 sn, sn, sym@rel32@lo+4; s_addc_u32 sn+1, sn+1, sym@rel32@hi+12,
    whose relocation addends assume the two adds follow s_getpc_b64 back to back.  That debug flag
    inserted an s_waitcnt after s_getpc_b64 and another before s_addc_u32, so kHeadOut (the heads'
    output widths, constant memory) was read 4 bytes early, a head's width came out wrong and its output
    stores left their buffer: the illegal address of the first deformation forward.  Every shipped code
    object must keep each such sequence contiguous."""
    for lib in LIBS:
        if not os.path.exists(lib):
            continue
        work = tmp_path / ("pc_" + os.path.basename(lib))
        work.mkdir()
        objs = disassemble(lib, work)
        n = 0
        for f, text in objs.items():
            ins = [ln.split("//")[0].strip() for ln in text.splitlines()]
            ins = [x for x in ins if x and not x.endswith(":") and not x.startswith("<") and "file format" not in x
                   and not x.startswith("Disassembly")]
            for i, x in enumerate(ins):
                if x.startswith("s_getpc_b64"):
                    n += 1
                    reg = x.split()[1]                                   # s[a:b]
                    lo, hi = reg[2:-1].split(":")
                    assert ins[i + 1].startswith(f"s_add_u32 s{lo}, s{lo},"), (f, ins[i:i + 3])
                    assert ins[i + 2].startswith(f"s_addc_u32 s{hi}, s{hi},"), (f, ins[i:i + 3])
        assert n > 0   # the check saw the sequences it guards
