"""Build the in-tree native extension ``distributed_pytorch_from_scratch_amd/_C*.so``.

Two-stage native build, no hipify, no JIT cache:

1. every ``csrc/{kernels,comm,blas}/*.hip`` -> ``hipcc --offload-arch=gfx950 -O3 -c`` (pure HIP,
   no torch headers, so each file compiles in seconds; parallel; mtime-cached);
2. ``csrc/bindings.cpp`` -> ``g++`` against the PyTorch headers (host code only);
3. link with the ROCm runtime, RCCL and hipBLASLt that PyTorch itself ships (``torch/lib``), so
   the process has exactly one instance of each.

Usage: ``python tools/build_ext.py [--jobs N] [--force] [--kernel-assert]`` (also called by
``__graft_entry__.build()``).  ``--kernel-assert`` builds the debug variant ``_C_kassert*.so``
(``-DDPFS_KERNEL_ASSERT=1``: device-side bounds asserts, ``csrc/kernels/common.h``) next to the
default one, from its own object directory; ``DPFS_KERNEL_ASSERT=1`` at run time loads it.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
PKG = os.path.join(ROOT, "distributed_pytorch_from_scratch_amd")
ARCH = os.environ.get("DPFS_OFFLOAD_ARCH", "gfx950")


# Per-translation-unit flags: the fused attention backward keeps its MFMA accumulators in VGPRs
# (its long-lived ones are asm-owned AGPRs, csrc/kernels/attn_acc.inc), so the compiler must
# not pick the AGPR form for its own MFMAs there; the other kernels keep the default heuristics.
PER_FILE_FLAGS = {"attention_fused.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _hipcc() -> str:
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build the gfx950 kernels)")


def _newer(src_list, dst) -> bool:
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def ext_path(kernel_assert: bool = False) -> str:
    return os.path.join(PKG, ("_C_kassert" if kernel_assert else "_C") + sysconfig.get_config_var("EXT_SUFFIX"))


def build(jobs: int = 8, force: bool = False, verbose: bool = True, kernel_assert: bool = False) -> str:
    import torch
    from torch.utils import cpp_extension as ce

    obj_dir = OBJ + ("_kassert" if kernel_assert else "")
    os.makedirs(obj_dir, exist_ok=True)
    hipcc = _hipcc()
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h")) + glob.glob(os.path.join(CSRC, "comm", "*.h"))
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))) + \
        sorted(glob.glob(os.path.join(CSRC, "comm", "*.hip"))) + \
        sorted(glob.glob(os.path.join(CSRC, "blas", "*.hip")))
    hip_flags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
                 "-munsafe-fp-atomics", "-Wno-unused-result"] + (["-DDPFS_KERNEL_ASSERT=1"] if kernel_assert else [])
    jobs_list = []
    for k in kernels:
        o = os.path.join(obj_dir, os.path.basename(k) + ".o")
        if force or _newer([k] + headers + glob.glob(os.path.join(CSRC, "kernels", "*.inc")), o):
            jobs_list.append([hipcc] + hip_flags + PER_FILE_FLAGS.get(os.path.basename(k), []) + ["-c", k, "-o", o])
    # Host bindings: plain g++ against the torch headers (HIP runtime headers for types).
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    py_inc = sysconfig.get_paths()["include"]
    inc = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames else ce.include_paths(cuda=True)
    b_src = os.path.join(CSRC, "bindings.cpp")
    b_obj = os.path.join(obj_dir, "bindings.o")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cxx_flags = ["-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                 f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=" + ("_C_kassert" if kernel_assert else "_C"), "-DTORCH_API_INCLUDE_EXTENSION_H",
                 "-I" + py_inc, "-I" + os.path.join(rocm, "include"), "-Wno-deprecated-declarations"]
    for i in inc:
        cxx_flags.append("-I" + i)
    if force or _newer([b_src], b_obj):
        jobs_list.append(["g++"] + cxx_flags + ["-c", b_src, "-o", b_obj])

    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_run, c) for c in jobs_list]
            for f, c in zip(futs, jobs_list):
                f.result()
                if verbose:
                    print("[build_ext] compiled", os.path.basename(c[-1]), flush=True)
    objs = [os.path.join(obj_dir, os.path.basename(k) + ".o") for k in kernels] + [b_obj]
    out = ext_path(kernel_assert)
    if force or jobs_list or not os.path.exists(out):
        tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
        # link to a temporary name and rename: a tree snapshot taken during the build (a GPU
        # run's upload) sees either the old or the new library, never a partial one
        tmp_out = out + ".tmp"
        link = ["g++", "-shared", "-o", tmp_out] + objs + [
            "-L" + tlib, "-Wl,-rpath," + tlib, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-lc10_hip", "-ltorch_hip", "-lamdhip64", "-lrccl",   # torch's own librccl.so (same instance)
            "-lhipblaslt"]                                       # and torch's own libhipblaslt.so
        _run(link)
        os.replace(tmp_out, out)
        if verbose:
            print("[build_ext] linked", out, flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--kernel-assert", action="store_true", help="build the bounds-assert variant _C_kassert")
    a = ap.parse_args()
    build(a.jobs, a.force, kernel_assert=a.kernel_assert)


if __name__ == "__main__":
    main()
