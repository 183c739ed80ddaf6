"""Timing builds for A/B runs on the GPU box (diagnostic only, never the
product): ab_variants/libkmc_<tag>.so (repo root, git-ignored) built with extra
-D flags, selected at run time with KMC_DIAG=1 KMC_LIB_PATH=...  The directory
travels to the GPU box only while it exists: delete it after an A/B session
(the default push carries the in-tree build alone).
  python tools/build_variants.py tag=-DFLAG[,-DFLAG2] ...
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kmc-with-a-diffusion-reaction-algorithm_amd"))
import build as B  # noqa: E402

out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ab_variants")
os.makedirs(out, exist_ok=True)
procs = []
for spec in sys.argv[1:]:
    tag, flags = spec.split("=", 1)
    lib = os.path.join(out, "libkmc_%s.so" % tag)
    cmd = [B.HIPCC, *B.FLAGS, *flags.split(","), "-o", lib, *[os.path.join(B.CSRC, s) for s in B.SOURCES]]
    procs.append((tag, subprocess.Popen(cmd)))
rc = 0
for tag, p in procs:
    rc |= p.wait()
    print(tag, "ok" if p.returncode == 0 else "FAILED")
sys.exit(rc)
