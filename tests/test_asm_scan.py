"""tools/asm_scc_scan.py's check: an SCC value read after the header capture's
exec-setting asm before anything writes SCC again is flagged; a write first is not. CPU only
(the compile of the real kernels is the tool's own run, recorded under profiles/r06/)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import asm_scc_scan  # noqa: E402

ASM = """\ts_cmp_lg_u32 s4, 0
\t;;#ASMSTART
\ts_and_saveexec_b64 s[6:7], s[8:9]
\tds_write_b128 v1, v[2:5]
\ts_mov_b64 exec, s[6:7]
\t;;#ASMEND
{after}
\ts_endpgm
"""


def test_scc_read_after_capture_is_flagged():
    blocks, f = asm_scc_scan.scan(ASM.format(after="\tv_add_u32_e32 v1, v1, v2\n\ts_cselect_b64 s[0:1], s[2:3], s[4:5]"))
    assert blocks == 1 and len(f) == 1 and f[0]["insn"].startswith("s_cselect_b64")


def test_scc_written_first_is_clean():
    blocks, f = asm_scc_scan.scan(ASM.format(after="\ts_cmp_eq_u32 s1, s2\n\ts_cbranch_scc1 .LBB0_1"))
    assert blocks == 1 and f == []


def test_other_asm_is_ignored():
    blocks, f = asm_scc_scan.scan("\t;;#ASMSTART\n\tv_mov_b32 v0, 0\n\t;;#ASMEND\n\ts_cbranch_scc1 .L")
    assert blocks == 0 and f == []
