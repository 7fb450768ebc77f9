"""In-tree build of the native components.

* ``libpenny_kernels.so`` -- every ``csrc/kernels/*.hip`` compiled by hipcc for gfx950 only
  (``--offload-arch=gfx950``), linked into one shared library with a plain C ABI.  Python binds
  it with ctypes (``ops/_native.py``); no torch headers are involved, so a full rebuild takes
  seconds and the library loads into the same HIP runtime torch already initialised.
* ``libpenny_kernels_debug.so`` (``--debug``) -- the same kernels with device-side bounds checks
  (``PENNY_DASSERT`` in ``common.h``), loaded instead when ``PENNY_KERNEL_DEBUG=1``.
* ``_penny_runtime*.so`` -- the C++ host runtime (paged-KV block manager with prefix-cache
  hashing, ``csrc/runtime``), built with g++ against pybind11.

Incremental: objects are rebuilt only when a source or header is newer.  Usage::

    python -m financial_chatbot_llm_amd._build          # build everything
    python -m financial_chatbot_llm_amd._build --clean
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

PKG = os.path.dirname(os.path.abspath(__file__))
KDIR = os.path.join(PKG, "csrc", "kernels")
RDIR = os.path.join(PKG, "csrc", "runtime")
BUILD = os.path.join(PKG, "csrc", "build")
LIBDIR = os.path.join(PKG, "_lib")
KERNEL_LIB = os.path.join(LIBDIR, "libpenny_kernels.so")
KERNEL_LIB_DEBUG = os.path.join(LIBDIR, "libpenny_kernels_debug.so")
ARCH = os.environ.get("PENNY_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-DNDEBUG"]
# debug library: device bounds checks (common.h PENNY_DASSERT) on, same code otherwise
HIP_FLAGS_DEBUG = [f for f in HIP_FLAGS if f != "-DNDEBUG"] + ["-DPENNY_KERNEL_DEBUG"]


def kernel_lib(debug: bool = False) -> str:
    return KERNEL_LIB_DEBUG if debug else KERNEL_LIB


def _newer(src_files, target) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build_kernels(jobs: int = 8, verbose: bool = False, debug: bool = False) -> str:
    bdir = BUILD + ("_debug" if debug else "")
    lib = kernel_lib(debug)
    flags = HIP_FLAGS_DEBUG if debug else HIP_FLAGS
    os.makedirs(bdir, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    headers = glob.glob(os.path.join(KDIR, "*.h"))
    srcs = sorted(glob.glob(os.path.join(KDIR, "*.hip")))
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(bdir, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if _newer([s] + headers, o):
            todo.append((s, o))

    def one(so):
        s, o = so
        if verbose:
            print(f"[hipcc{' debug' if debug else ''}] {os.path.basename(s)}", flush=True)
        _run([HIPCC, *flags, "-I", KDIR, "-c", s, "-o", o])
        return o

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(one, todo))
    if todo or _newer(objs, lib):
        tmp = lib + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp, *objs])
        os.replace(tmp, lib)
    return lib


def runtime_lib_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_penny_runtime" + suffix)


def build_runtime(verbose: bool = False) -> str:
    import pybind11
    srcs = sorted(glob.glob(os.path.join(RDIR, "*.cpp")))
    headers = glob.glob(os.path.join(RDIR, "*.h"))
    out = runtime_lib_path()
    if not srcs:
        return ""
    if _newer(srcs + headers, out):
        if verbose:
            print("[g++] runtime", flush=True)
        inc = [pybind11.get_include(), sysconfig.get_paths()["include"]]
        cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall",
               *[f"-I{i}" for i in inc], "-I", RDIR, *srcs, "-o", out + ".tmp"]
        _run(cmd)
        os.replace(out + ".tmp", out)
    return out


def build_all(jobs: int = 8, verbose: bool = False, debug: bool = False) -> None:
    build_kernels(jobs=jobs, verbose=verbose)
    if debug:
        build_kernels(jobs=jobs, verbose=verbose, debug=True)
    build_runtime(verbose=verbose)


def clean() -> None:
    shutil.rmtree(BUILD, ignore_errors=True)
    shutil.rmtree(BUILD + "_debug", ignore_errors=True)
    for p in (KERNEL_LIB, KERNEL_LIB_DEBUG, runtime_lib_path()):
        if os.path.exists(p):
            os.remove(p)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--runtime-only", action="store_true", help="host runtime only (machines without hipcc)")
    ap.add_argument("--debug", action="store_true",
                    help="also build libpenny_kernels_debug.so (device bounds checks; PENNY_KERNEL_DEBUG=1 loads it)")
    args = ap.parse_args(argv)
    if args.clean:
        clean()
    if args.runtime_only:
        print(f"built {build_runtime(verbose=True)}")
        return 0
    # an in-tree debug library is kept in sync with the sources too (a stale one would miss symbols)
    debug = args.debug or os.environ.get("PENNY_KERNEL_DEBUG") == "1" or os.path.exists(KERNEL_LIB_DEBUG)
    build_all(jobs=args.j, verbose=True, debug=debug)
    print(f"built {KERNEL_LIB}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
