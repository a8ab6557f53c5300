#!/bin/bash
# Per-kernel register / spill / LDS usage of one HIP source (kernel-resource-usage remarks):
#   tools/resusage.sh aipstack_amd/csrc/frame_kernels.hip [extra hipcc flags] [| grep NAME]
src=$1; shift
cd "$(dirname "$src")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-parameter \
    -I"$(git rev-parse --show-toplevel)/include" -I. "$@" -c "$(basename "$src")" -o /dev/null \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import re, sys, subprocess
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}; rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, dn in zip(rows, names):
    g = lambda k: r.get(k, "?")
    print("%4s vgpr %2s occ sspill %3s vspill %3s lds %6s  %s" % (g("VGPRs"), g("Occupancy [waves/SIMD]"), g("SGPRs Spill"), g("VGPRs Spill"), g("LDS Size [bytes/block]"), dn[:150]))
'
