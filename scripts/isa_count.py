#!/usr/bin/env python3
"""Static instruction counts per kernel of a HIP source (device assembly for gfx950).

Usage: isa_count.py [SRC] [-DFLAG=V ...] [KERNEL_SUBSTR ...]   (default SRC: csrc/orb_hip.hip, all kernels;
extra compiler options, e.g. -mllvm ones, in $ISA_EXTRA)
Prints per kernel: VALU / SALU / LDS / VMEM / SMEM / MFMA counts, VGPRs, SGPRs, LDS bytes and
the occupancy the compiler reports.  Static counts (each instruction once, loops not unrolled at
run time): a quick CPU-side check of a kernel edit before it is timed on the GPU."""
import collections
import os
import pathlib
import re
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from __graft_entry__ import hipcc_flags  # noqa: E402

src = pathlib.Path(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].endswith(".hip") else \
    ROOT / "orbslam_jpminipc_amd" / "csrc" / "orb_hip.hip"
keys = [a for a in sys.argv[1:] if not a.endswith(".hip") and not a.startswith("-D")]
flags = [f for f in hipcc_flags() if f not in ("-shared", "-fPIC")] + [
    a for a in sys.argv[1:] if a.startswith("-D")] + os.environ.get("ISA_EXTRA", "").split()
with tempfile.TemporaryDirectory() as d:
    out = pathlib.Path(d) / "k.s"
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-S", "-o", str(out), str(src)], check=True)
    text = out.read_text()

kern = None
cnt = collections.defaultdict(collections.Counter)
meta = collections.defaultdict(dict)
for line in text.splitlines():
    m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
    if m and not m.group(1).startswith((".L", "$")):
        kern = m.group(1)
        continue
    if kern is None:
        continue
    s = line.strip()
    m = re.match(r";\s*(NumVgprs|NumSgprs|Occupancy|ScratchSize|TotalNumVgprs|LDSByteSize):\s*(\d+)", s)
    if m:
        meta[kern][m.group(1)] = int(m.group(2))
        continue
    if not s or s.startswith((";", ".", "//")):
        continue
    op = s.split()[0]
    if op.startswith("v_mfma"):
        cnt[kern]["mfma"] += 1
    elif op.startswith("v_"):
        cnt[kern]["valu"] += 1
    elif op.startswith("s_load") or op.startswith("s_buffer_load"):
        cnt[kern]["smem"] += 1
    elif op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_endpgm", "s_setprio", "s_sleep")):
        cnt[kern]["sync"] += 1
    elif op.startswith("s_"):
        cnt[kern]["salu"] += 1
    elif op.startswith("ds_"):
        cnt[kern]["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cnt[kern]["vmem"] += 1

print(f"{'kernel':60s} {'valu':>5s} {'salu':>5s} {'lds':>4s} {'vmem':>4s} {'smem':>4s} {'mfma':>4s} {'sync':>4s}"
      f" {'vgpr':>4s} {'sgpr':>4s} {'occ':>3s} {'lds_B':>6s} {'scr':>4s}")
for k, c in cnt.items():
    if keys and not any(x in k for x in keys):
        continue
    m = meta[k]
    print(f"{k[:60]:60s} {c['valu']:5d} {c['salu']:5d} {c['lds']:4d} {c['vmem']:4d} {c['smem']:4d} {c['mfma']:4d}"
          f" {c['sync']:4d} {m.get('NumVgprs', -1):4d} {m.get('NumSgprs', -1):4d} {m.get('Occupancy', -1):3d}"
          f" {m.get('LDSByteSize', -1):6d} {m.get('ScratchSize', -1):4d}")
