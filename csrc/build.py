#!/usr/bin/env python3
"""Build the psx native libraries in-tree (no pip install, no JIT cache).

  libpsx_kernels.so : every HIP kernel in csrc/kernels/*.hip, compiled for gfx950 with hipcc,
                      exported through a plain C ABI (loaded with ctypes after `import torch`, so
                      the kernels run on the same HIP runtime instance as PyTorch-ROCm).
  libpsx_runtime.so : host-only C++ runtime in csrc/runtime/*.cpp (parameter-server core state
                      machine, shared-memory control-plane mailbox, CIFAR binary reader).

Objects are rebuilt only when a source or header is newer than the object. The outputs land
in <package>/_native/ so they travel with `gpurun` snapshots.

Usage:  python csrc/build.py [--clean] [-j N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "distributed-parameter-server-for-ml-training_amd")
OUT = os.path.join(PKG, "_native")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("PSX_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _newer(src_files, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed (%d): %s\n%s" % (r.returncode, " ".join(cmd), r.stdout))
    return r.stdout


# per-source extra flags. wino_fused.hip: no SLP vectorization — packed f32 VALU (v_pk_add /
# v_pk_fma) in the transform that runs beside the other wave's MFMAs measured slower (32x32x64
# forward 52.2 -> 50.7 us without it; MI355X_MICROARCH.md: packed f32 beside MFMAs is an anti-lever)
FILE_FLAGS = {"wino_fused.hip": ["-fno-slp-vectorize"], "wino_wgrad.hip": ["-fno-slp-vectorize", "-ffp-contract=off"]}


def build(jobs: int = 8, debug: bool = False, verbose: bool = False) -> dict:
    os.makedirs(OUT, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    opt = ["-O1", "-g"] if debug else ["-O3"]
    k_hdrs = glob.glob(os.path.join(HERE, "kernels", "*.hpp"))
    k_srcs = sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip")))
    r_hdrs = glob.glob(os.path.join(HERE, "runtime", "*.h")) + glob.glob(os.path.join(HERE, "runtime", "*.hpp"))
    r_srcs = sorted(glob.glob(os.path.join(HERE, "runtime", "*.cpp")))

    hip_flags = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
                 "-Wno-unused-variable", "-munsafe-fp-atomics", "-I", os.path.join(HERE, "kernels")] + opt
    cxx_flags = ["-std=c++17", "-fPIC", "-Wall", "-pthread", "-I", os.path.join(HERE, "runtime")] + opt

    jobs_list = []
    for s in k_srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        if _newer([s] + k_hdrs, o):
            jobs_list.append([HIPCC] + hip_flags + FILE_FLAGS.get(os.path.basename(s), []) + ["-c", s, "-o", o])
    for s in r_srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        if _newer([s] + r_hdrs, o):
            jobs_list.append([CXX] + cxx_flags + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)

    libs = {}
    k_objs = [os.path.join(OBJ, os.path.basename(s) + ".o") for s in k_srcs]
    k_lib = os.path.join(OUT, "libpsx_kernels.so")
    if k_objs and _newer(k_objs, k_lib):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", k_lib] + k_objs)
    libs["kernels"] = k_lib
    r_objs = [os.path.join(OBJ, os.path.basename(s) + ".o") for s in r_srcs]
    r_lib = os.path.join(OUT, "libpsx_runtime.so")
    if r_objs and _newer(r_objs, r_lib):
        _run([CXX, "-shared", "-fPIC", "-pthread", "-o", r_lib] + r_objs + ["-lrt"])
    libs["runtime"] = r_lib

    # libpsx_comm.so: host C++ against the HIP runtime + RCCL headers (RCCL itself is dlopened at
    # run time, see csrc/comm/rccl_comm.cpp); csrc/server/*.cpp is the native server event loop
    c_srcs = sorted(glob.glob(os.path.join(HERE, "comm", "*.cpp")) + glob.glob(os.path.join(HERE, "server", "*.cpp")))
    c_hdrs = (glob.glob(os.path.join(HERE, "comm", "*.h")) + glob.glob(os.path.join(HERE, "server", "*.h")) + r_hdrs)
    c_flags = ["-std=c++17", "-fPIC", "-Wall", "-pthread", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
               "-I", os.path.join(HERE, "runtime"), "-I", os.path.join(HERE, "comm")] + opt
    c_objs = []
    for s in c_srcs:
        o = os.path.join(OBJ, "comm_" + os.path.basename(s) + ".o")
        c_objs.append(o)
        if _newer([s] + c_hdrs, o):
            _run([HIPCC] + c_flags + ["-c", s, "-o", o])
    c_lib = os.path.join(OUT, "libpsx_comm.so")
    if c_objs and _newer(c_objs, c_lib):
        _run([HIPCC, "-shared", "-fPIC", "-pthread", "-o", c_lib] + c_objs + ["-ldl", "-lrt"])
    libs["comm"] = c_lib

    # TEST-ONLY: libpsx_fakecomm.so, an RCCL stand-in for several ranks on one GPU (see
    # csrc/tests/fakecomm.hip); tests load it with PSX_RCCL_LIB + PSX_FAKECOMM_TEST=1
    f_src = os.path.join(HERE, "tests", "fakecomm.hip")
    f_lib = os.path.join(OUT, "testing", "libpsx_fakecomm.so")
    if os.path.exists(f_src) and _newer([f_src], f_lib):
        os.makedirs(os.path.dirname(f_lib), exist_ok=True)
        _run([HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared", "-Wall", "-D__HIP_PLATFORM_AMD__",
              "-I", "/opt/rocm/include"] + opt + [f_src, "-o", f_lib, "-lrt", "-pthread"])
    libs["fakecomm"] = f_lib
    return libs


def build_variant(name: str, defines: list[str], jobs: int = 8) -> str:
    """A/B build of the kernel library with extra -D defines into _native/variants/ (load it
    with PSX_KERNELS_LIB=<path>); e.g. --variant s4 -D PSX_STAT_SLOTS=4."""
    vout = os.path.join(OUT, "variants")
    vobj = os.path.join(OBJ, "variant_" + name)
    os.makedirs(vout, exist_ok=True)
    os.makedirs(vobj, exist_ok=True)
    k_srcs = sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip")))
    flags = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-O3", "-munsafe-fp-atomics", "-I",
             os.path.join(HERE, "kernels")] + [d if d.startswith("-") else f"-D{d}" for d in defines]
    cmds = [[HIPCC] + flags + FILE_FLAGS.get(os.path.basename(s_), []) +
            ["-c", s_, "-o", os.path.join(vobj, os.path.basename(s_) + ".o")] for s_ in k_srcs]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, cmds))
    lib = os.path.join(vout, f"libpsx_kernels_{name}.so")
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] +
         [os.path.join(vobj, os.path.basename(s_) + ".o") for s_ in k_srcs])
    return lib


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--variant", default=None, help="build an A/B kernel library variant (see build_variant)")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args(argv)
    if a.variant:
        print(build_variant(a.variant, a.defines, a.j))
        return 0
    if a.clean:
        shutil.rmtree(OBJ, ignore_errors=True)
        for f in glob.glob(os.path.join(OUT, "*.so")):
            os.remove(f)
    libs = build(a.j, a.debug, a.v)
    for k, v in libs.items():
        print(f"{k}: {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
