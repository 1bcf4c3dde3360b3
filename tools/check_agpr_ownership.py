"""Guard for the asm-owned accumulators of the v4 GEMM (csrc/kernels/gemm4.hip).

gemm4_k keeps its 256 fp32 accumulators per lane in AGPRs a[0:255] written and read only by
inline asm (gemm4_acc.inc); hipcc does not know they are live.  If a kernel variant needs more
arch VGPRs than the 256 left to it, the register allocator spills into AGPRs -- silently
overwriting accumulators (a late-round-6 RoPE-epilogue experiment did exactly that at
head_dim 128: garbage outputs).  This compiles gemm4.hip to gfx950 assembly with the build's
flags and fails if any kernel has a compiler-generated AGPR write or a scratch spill.

    python tools/check_agpr_ownership.py [--src csrc/kernels/gemm4.hip]
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast", "-munsafe-fp-atomics",
         "-Wno-unused-result", "--cuda-device-only", "-S"]


def violations(asm: str):
    """(kernel, line) pairs of v_accvgpr_write / scratch instructions outside inline-asm blocks."""
    out, name, inasm = [], None, False
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name = m.group(1)
        if ";;#ASMSTART" in line:
            inasm = True
        elif ";;#ASMEND" in line:
            inasm = False
        elif not inasm and re.search(r"\b(v_accvgpr_write_b32|scratch_store|scratch_load)", line):
            out.append((name, line.strip()))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "csrc", "kernels", "gemm4.hip"))
    a = ap.parse_args()
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    with tempfile.TemporaryDirectory() as d:
        s = os.path.join(d, "k.s")
        r = subprocess.run([hipcc] + FLAGS + ["-I", os.path.dirname(a.src), a.src, "-o", s],
                           capture_output=True, text=True)
        if r.returncode != 0:
            print(r.stderr[-3000:])
            return 2
        bad = violations(open(s).read())
    kernels = sorted({k for k, _ in bad})
    for k in kernels:
        print(f"compiler-owned AGPR write / scratch spill in {k}:")
        for kk, line in bad:
            if kk == k:
                print(f"    {line}")
    print(f"{os.path.basename(a.src)}: {len(kernels)} kernel(s) with compiler AGPR writes or spills")
    return 1 if kernels else 0


if __name__ == "__main__":
    sys.exit(main())
