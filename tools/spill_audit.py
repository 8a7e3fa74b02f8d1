"""List the kernels of csrc/*.hip that use scratch or spill VGPRs (CPU only: hipcc
--save-temps for gfx950, then the code object metadata of each kernel).  A spill reload
inside a kernel whose loop keeps inline-asm LDS-DMAs in flight (K9t, K2p, the streaming
scans) waits vmcnt(0) and drains the ring every iteration, so the hot kernels must show
nothing here; the k > 16 list variants (KC = 64) spill into AGPRs by design.

  python tools/spill_audit.py [file.hip ...]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mediquery-rag_amd", "csrc")
EXTRA = {"gemm_x6p.hip": ["-fno-slp-vectorize"]}  # as csrc/Makefile


def audit(src, tmp):
    base = os.path.basename(src)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + CSRC,
           "-I" + os.path.join(ROOT, "include"), "--save-temps", "-c", src, "-o",
           os.path.join(tmp, base + ".o")] + EXTRA.get(base, [])
    subprocess.run(cmd, cwd=tmp, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    asm = glob.glob(os.path.join(tmp, os.path.splitext(base)[0] + "-hip-amdgcn-amd-amdhsa-gfx950.s"))[0]
    txt = open(asm).read()
    meta = txt[txt.find("amdhsa.kernels:"):]
    rows = []
    for e in re.split(r"\n  - ", meta):
        name = re.search(r"\.name:\s+(\S+)", e)
        if not name:
            continue
        get = lambda k: int(re.search(r"\.%s:\s+(\d+)" % k, e).group(1)) if re.search(r"\.%s:\s+(\d+)" % k, e) else 0
        priv, spill, vgpr = get("private_segment_fixed_size"), get("vgpr_spill_count"), get("vgpr_count")
        if priv or spill:
            rows.append((base, name.group(1), priv, spill, vgpr))
    return rows


def main():
    srcs = sys.argv[1:] or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with tempfile.TemporaryDirectory() as tmp:
        for src in srcs:
            for base, name, priv, spill, vgpr in audit(os.path.abspath(src), tmp):
                print("%-13s scratch %4d B  spilled %4d  vgpr %3d  %s" % (base, priv, spill, vgpr, name))


if __name__ == "__main__":
    main()
