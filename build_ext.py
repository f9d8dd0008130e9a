#!/usr/bin/env python3
"""Build the native extension in-tree for gfx950 (no hipify, no JIT cache).

  csrc/kernels/*.hip  --hipcc --offload-arch=gfx950 -O3-->  build/obj/*.o   (device code + host stubs)
  csrc/bindings.cpp   --hipcc (host only, torch headers)-->  build/obj/bindings.o
  link                                                  -->  tensorflowdistributedlearning_amd/_C*.so

Incremental: an object is rebuilt only when its source or any csrc header is newer.  Objects are
compiled in parallel (MAX_JOBS, default min(8, cpus)).  The .so lands next to the package so it
travels with the repository snapshot to the GPU box and is what the GPU tests load.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
PKG = os.path.join(ROOT, "tensorflowdistributedlearning_amd")
ARCH = os.environ.get("TDL_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths()
    libdirs = ce.library_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libdirs, abi


def _newer(src, dst, deps):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return os.path.getmtime(src) > t or any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {cmd[-1]}")
    return cmd[-1]


def so_name():
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def build(verbose=True, force=False):
    os.makedirs(OBJ, exist_ok=True)
    inc, libdirs, abi = _torch_flags()
    headers = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    jobs = []
    common = ["-O3", "-std=c++17", "-fPIC", "-I" + CSRC, "-Wno-unused-result",
              "-Wno-deprecated-declarations"]
    if os.environ.get("TDL_CONV_ABLATION") == "1":  # timing-only TDL_CONV_DBG flags (dev/tools/*_ablate.py)
        common.append("-DTDL_CONV_ABLATION=1")
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        if force or _newer(src, obj, headers):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", *common, "-c", "-o", obj, src])
    for src in sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))):
        obj = os.path.join(OBJ, "rt_" + os.path.basename(src) + ".o")
        if force or _newer(src, obj, headers):
            jobs.append([HIPCC, *common, "-pthread", "-D__HIP_PLATFORM_AMD__=1", "-c", "-o", obj, src])
    bsrc = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(OBJ, "bindings.o")
    if force or _newer(bsrc, bobj, headers):
        py_inc = sysconfig.get_paths()["include"]
        jobs.append([HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                     "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                     f"-D_GLIBCXX_USE_CXX11_ABI={abi}", *["-I" + i for i in inc], "-I" + py_inc,
                     "-c", "-o", bobj, bsrc])
    if jobs:
        n = int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 4)))
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for name in ex.map(_run, jobs):
                if verbose:
                    print(f"[build_ext] compiled {os.path.relpath(name, ROOT)}", flush=True)
    objs = sorted(glob.glob(os.path.join(OBJ, "*.o")))
    out = so_name()
    if jobs or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        torch_lib = libdirs[0]
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs,
                "-L" + torch_lib, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip",
                "-ltorch_hip", "-lamdhip64", "-lz", "-pthread", f"-Wl,-rpath,{torch_lib}",
                # RCCL: torch ships librccl.so (soname librccl.so.1) and loads it first, so the
                # native communicator (csrc/runtime/comm.cpp) shares torch's RCCL instance
                "-L" + torch_lib, "-lrccl"]
        _run(link)
        if verbose:
            print(f"[build_ext] linked {os.path.relpath(out, ROOT)}", flush=True)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
