"""Debug aid: one gathered-stream strided batch (tunable gather 0) against the oracle, printing
the first mismatching packets. Usage: python3 tools/debug_gathered.py PLEN N OFFSET CHUNK"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import aipstack_amd as A  # noqa: E402
from aipstack_amd import _lib, synth  # noqa: E402
from conftest import Oracle  # noqa: E402

plen, n, off, chunk = (int(x) for x in sys.argv[1:5])
lib = _lib.load()
lib.aipstack_chksum_tune(b"gather", 0)
lib.aipstack_chksum_tune(b"chunk_packets", chunk)
buf = torch.empty(1 << 22, dtype=torch.uint8, device="cuda:0")
synth.fill_device(buf, 31)
hb = buf.cpu().numpy()
got = A.chksum_batch_strided(buf, plen, plen, n, byte_offset=off).cpu().numpy()
want = Oracle().batch_strided(hb[off:], plen, plen, n)
bad = np.nonzero(got != want)[0]
print(f"plen {plen} n {n} off {off} chunk {chunk}: {len(bad)} mismatches; first {bad[:16].tolist()}")
for i in bad[:6]:
    print(f"  packet {i}: got {got[i]:#06x} want {want[i]:#06x}")
