#!/usr/bin/env python3
"""Scan the frame kernels' gfx950 ISA for an SCC value live across the header capture's
exec-setting inline asm (HeaderCapture::window in frame_kernels.hip): after each asm block that
holds a ds_write_b128, the first SALU instruction that touches SCC must write it, not read it
(s_cbranch_scc*, s_cselect_*, s_addc / s_subb, s_cmov read it). Compiles the device code
(hipcc --cuda-device-only -S). Prints one JSON line; exit 1 on a finding. Not part of the
product.

    python tools/asm_scc_scan.py [-DFLAG ...]
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READS = re.compile(r"^(s_cbranch_scc[01]|s_cselect_b(32|64)|s_addc_u32|s_subb_u32|s_cmov_b(32|64))\b")
WRITES = re.compile(r"^(s_cmp|s_bitcmp|s_and_|s_or_|s_xor_|s_andn2|s_orn2|s_nand|s_nor|s_xnor|"
                    r"s_add_|s_sub_|s_lshl|s_lshr|s_ashr|s_bfe|s_min|s_max|s_abs|s_not|s_bcnt|"
                    r"s_ff|s_flbit|s_wqm|s_mul_hi|s_absdiff|s_quadmask)")


def scan(asm_text):
    lines = asm_text.split("\n")
    blocks, findings, start = 0, [], None
    for i, l in enumerate(lines):
        if ";;#ASMSTART" in l:
            start = i
        elif ";;#ASMEND" in l and start is not None:
            body = lines[start:i]
            start = None
            if not any("ds_write_b128" in b for b in body):
                continue
            blocks += 1
            for j in range(i + 1, len(lines)):
                t = lines[j].strip()
                if not t or t.startswith((";", ".")) or t.endswith(":"):
                    continue
                if READS.match(t):
                    findings.append({"line": j + 1, "insn": t})
                    break
                if WRITES.match(t) or t.startswith(("s_endpgm", "s_branch", "s_setpc")):
                    break
    return blocks, findings


def main():
    csrc = os.path.join(ROOT, "aipstack_amd", "csrc")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "frame_kernels.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-Wno-unused-parameter", "-I" + os.path.join(ROOT, "include"), "-I" + csrc,
               "--cuda-device-only", "-S", "-o", out, os.path.join(csrc, "frame_kernels.hip")]
        subprocess.run(cmd + sys.argv[1:], check=True, capture_output=True)
        blocks, findings = scan(open(out).read())
    print(json.dumps({"capture_asm_blocks": blocks, "scc_read_after": len(findings),
                      "findings": findings[:10], "flags": sys.argv[1:]}))
    sys.exit(1 if findings or blocks == 0 else 0)


if __name__ == "__main__":
    main()
