"""Round 5's h24 fault: the kept ISA's sign-extended high half
(profiles/r05/h24_sym3_filter_isa.txt) is reproduced, compile-only, from a hash
whose 24-bit product is held in an int (tools/probes/h24_signed_hash.hip), and
not from the same hash in uint32_t — the source's signed intermediate, not the
compiler, produced the out-of-range LDS index.  No GPU: hipcc -S for gfx950."""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "tools", "probes", "h24_signed_hash.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def kernel_asm(asm: str, name: str) -> str:
    m = re.search(r"^_Z\d+%s\w*:[^\n]*\n(.*?)s_endpgm" % name, asm, re.S | re.M)
    assert m, name
    return m.group(1)


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("h24") / "h24.s"
    subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", str(out), SRC],
                   check=True, capture_output=True, timeout=300)
    return out.read_text()


SEXT_HI = re.compile(r"v_lshrrev_b32_sdwa\s+v\d+,\s*v\d+,\s*sext\(v\d+\).*src1_sel:WORD_1")


def test_signed_hash_gives_the_kept_pattern(asm):
    k = kernel_asm(asm, "k_signed")
    assert SEXT_HI.search(k), "sign-extended high half expected"
    assert "0x1ffffffc" in k and "ds_or_rtn_b32" in k


def test_unsigned_hash_has_no_sext(asm):
    k = kernel_asm(asm, "k_unsigned")
    assert "sext(" not in k and "ds_or_rtn_b32" in k
