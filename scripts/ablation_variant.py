#!/usr/bin/env python3
"""Build a timing-ablation variant of liborb_hip.so from a patched copy of the sources (the
product sources are never modified): ablation_variant.py NAME 'old1' 'new1' ['old2' 'new2' ...]
applies exact-string replacements to orb_hip.hip in a scratch copy and builds
build/variants/NAME.so.  Wrong-output ablations live only in these scratch builds."""
import os
import pathlib
import shutil
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parent.parent
name, reps = sys.argv[1], sys.argv[2:]
tmp = pathlib.Path(tempfile.mkdtemp(prefix="orbvar_"))
shutil.copytree(ROOT / "orbslam_jpminipc_amd" / "csrc", tmp / "csrc")
shutil.copytree(ROOT / "include", tmp / "include")
src = tmp / "csrc" / "orb_hip.hip"
s = src.read_text()
for a, b in zip(reps[0::2], reps[1::2]):
    if s.count(a) != 1:
        sys.exit(f"pattern occurs {s.count(a)} times: {a[:80]!r}")
    s = s.replace(a, b)
src.write_text(s.replace('#include "../../include/', '#include "../include/'))
for f in (tmp / "csrc").glob("*.hip"):
    t = f.read_text().replace('"../../include/', '"../include/')
    f.write_text(t)
sys.path.insert(0, str(ROOT))
from __graft_entry__ import HIPCC_FLAGS, build_lib, hipcc_flags  # noqa: E402  (the library's recipe)

out = ROOT / "build" / "variants" / f"{name}.so"
out.parent.mkdir(parents=True, exist_ok=True)
extra = os.environ.get("ORB_VARIANT_EXTRA", "").split()
if os.environ.get("ORB_VARIANT_ASM"):  # device assembly of orb_hip.hip only: build/variants/NAME.s
    flags = [f for f in hipcc_flags() + extra if f not in ("-shared", "-fPIC")] + \
        os.environ.get("ORB_VARIANT_FLAGS", "").split()
    out = out.with_suffix(".s")
    r = subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-S", "-o", str(out),
                        str(tmp / "csrc" / "orb_hip.hip")], capture_output=True, text=True)
    shutil.rmtree(tmp)
    sys.exit(r.stderr[-3000:] if r.returncode else print("asm", out))
if os.environ.get("ORB_VARIANT_NO_OPT"):  # without the probed OPTIONAL_FLAGS (-amdgpu-mfma-vgpr-form=1)
    import __graft_entry__  # noqa: E402

    __graft_entry__.hipcc_flags = lambda hipcc="": list(HIPCC_FLAGS)
try:
    build_lib(out, tmp / "csrc", extra)
finally:
    shutil.rmtree(tmp)
print("built", out)
