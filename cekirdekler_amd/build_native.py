"""Build the native runtime (_cek extension) and the AOT gfx950 kernel library.

Everything is built in-tree so the artefacts travel with the repository
snapshot to the GPU box:

* ``cekirdekler_amd/_cek*.so`` — C++17 host runtime (HIP runtime API, hiprtc,
  RCCL, roctx) + pybind11 bindings.
* ``cekirdekler_amd/kernels/*.hsaco`` — hand-written CDNA4 kernels compiled
  ahead of time with ``hipcc --genco --offload-arch=gfx950``.

Usage: ``python -m cekirdekler_amd.build_native [--force] [--jobs N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
KDIR = os.path.join(HERE, "kernels")
BUILD = os.path.join(HERE, "_build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("CEK_ARCH", "gfx950")

SOURCES = ["device.cpp", "jit.cpp", "memory.cpp", "balancer.cpp", "worker.cpp", "dist.cpp",
           "cores.cpp", "pool.cpp", "copy_engine.cpp", "shell_gemm.cpp", "xgmi.cpp", "probe.cpp", "refloops.cpp",
           "bindings.cpp"]


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(HERE, "_cek" + suffix)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout)


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps if os.path.exists(d))


def _headers() -> list[str]:
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]


def build_extension(force: bool = False, jobs: int = 8) -> str:
    import pybind11

    os.makedirs(BUILD, exist_ok=True)
    cxx = os.environ.get("CEK_HOST_CXX", "g++")
    inc = [f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           f"-I{ROCM}/include"]
    flags = ["-O2", "-g", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__=1",
             "-Wall", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    hdrs = _headers()
    objs = []
    todo = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s.replace(".cpp", ".o"))
        objs.append(obj)
        if force or not _newer(obj, [src] + hdrs):
            todo.append([cxx, *flags, *inc, "-c", src, "-o", obj])
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(_run, todo))
    out = ext_path()
    if force or todo or not os.path.exists(out):
        _run([cxx, "-shared", "-o", out + ".tmp", *objs, f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib",
              "-lamdhip64", "-lhiprtc", "-lrccl", "-lrocprofiler-sdk-roctx", "-ldl", "-lpthread", "-lrt"])
        os.replace(out + ".tmp", out)
    return out


def kernel_sources() -> list[str]:
    if not os.path.isdir(KDIR):
        return []
    return sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".hip"))


def _file_flags(src: str) -> list[str]:
    """Per-file compiler flags from a ``// cek-flags: ...`` line in the source."""
    flags: list[str] = []
    with open(src) as f:
        for line in f:
            line = line.strip()
            if line.startswith("// cek-flags:"):
                flags += line.split(":", 1)[1].split()
    return flags


def build_kernels(force: bool = False, jobs: int = 8) -> list[str]:
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(hipcc):
        hipcc = shutil.which("hipcc") or "hipcc"
    todo, outs = [], []
    inc_hdrs = [os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".h")] if os.path.isdir(KDIR) else []
    for src in kernel_sources():
        out = src[:-4] + ".hsaco"
        outs.append(out)
        if force or not _newer(out, [src] + inc_hdrs):
            todo.append([hipcc, "--genco", f"--offload-arch={ARCH}", "-O3", "-std=c++17",
                         "-mcode-object-version=5", f"-I{KDIR}", *_file_flags(src), src, "-o", out])
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(_run, todo))
    return outs


def build_all(force: bool = False, jobs: int = 8) -> None:
    build_extension(force, jobs)
    build_kernels(force, jobs)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args(argv)
    build_all(a.force, a.jobs)
    print("built", ext_path())
    return 0


if __name__ == "__main__":
    sys.exit(main())
