#!/usr/bin/env python3
"""Build the in-tree native libraries.

* ``libskrnn_host.so``: ``g++ -O3`` over ``csrc/host/*.cpp``.
* ``libskrnn_hip.so``: ``hipcc --offload-arch=gfx950 -O3`` over
  ``csrc/*.hip``, linked against the HIP runtime by soname with an rpath to
  PyTorch's ``lib/`` so the process uses a single runtime.

Incremental: a target is rebuilt only when a source or header is newer.
Usage: ``python scripts/build_native.py [--force] [--only host|hip] [-j N]``
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "sketch_rnn_amd", "_lib")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("SKR_OFFLOAD_ARCH", "gfx950")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("  $ " + " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def torch_lib_dir():
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        return os.path.join(os.path.dirname(spec.origin), "lib")
    except Exception:
        return None


def build_host(force=False):
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    target = os.path.join(OUT, "libskrnn_host.so")
    if not force and not _newer(target, srcs + hdrs):
        print("host lib up to date")
        return target
    os.makedirs(OUT, exist_ok=True)
    _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-o", target] + srcs + ["-lpthread"])
    return target


def build_hip(force=False, jobs=8):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    target = os.path.join(OUT, "libskrnn_hip.so")
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall", "-Wno-unused-function",
             "-munsafe-fp-atomics", "-I" + CSRC]
    objs, jobs_list = [], []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs_list.append([hipcc] + flags + ["-c", s, "-o", o])
    if jobs_list:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(jobs_list)))) as ex:
            list(ex.map(_run, jobs_list))
    if force or jobs_list or _newer(target, objs):
        link = [hipcc, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", target] + objs
        tl = torch_lib_dir()
        if tl:
            link += ["-Wl,-rpath," + tl]
        _run(link)
    else:
        print("hip lib up to date")
    return target


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["host", "hip"])
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    if a.only in (None, "host"):
        build_host(a.force)
    if a.only in (None, "hip"):
        build_hip(a.force, a.j)


if __name__ == "__main__":
    sys.exit(main())
