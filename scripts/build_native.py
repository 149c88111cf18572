#!/usr/bin/env python3
"""Build the in-tree native libraries.

* ``libskrnn_host.so``: ``g++ -O3`` over ``csrc/host/*.cpp``.
* ``libskrnn_hip.so``: ``hipcc --offload-arch=gfx950 -O3`` over
  ``csrc/*.hip``, linked against the HIP runtime by soname with an rpath to
  PyTorch's ``lib/`` so the process uses a single runtime.

Incremental by CONTENT, not mtime: every object and library carries a
``.sha256`` stamp of its sources, headers, compiler flags and toolchain; a
target is rebuilt whenever the stamp does not match the current tree, so a
library that travelled with a snapshot is never mistaken for a build of
different sources. ``--force`` rebuilds everything.
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


def _digest(files, cmd):
    import hashlib
    h = hashlib.sha256()
    h.update(" ".join(cmd).encode())
    for f in sorted(files):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stale(target, files, cmd):
    """True unless ``target`` exists with a stamp matching ``files`` + ``cmd``."""
    stamp = target + ".sha256"
    if not os.path.exists(target) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(files, cmd)


def _stamp(target, files, cmd):
    with open(target + ".sha256", "w") as f:
        f.write(_digest(files, cmd) + "\n")


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
    cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-o", target] + srcs + ["-lpthread"]
    if not force and not _stale(target, srcs + hdrs, cmd):
        print("host lib up to date")
        return target
    os.makedirs(OUT, exist_ok=True)
    _run(cmd)
    _stamp(target, srcs + hdrs, cmd)
    return target


# Experiment builds (A/B against the default library, loaded with
# SKR_HIP_LIB=<path>): extra defines per variant.
VARIANTS = {"exact_act": ["-DSKR_EXACT_ACT"]}


def build_hip(force=False, jobs=8, variant=None):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    build, out, name = BUILD, OUT, "libskrnn_hip.so"
    if variant:
        build, out, name = BUILD + "_" + variant, os.path.join(OUT, "variants"), "libskrnn_hip_%s.so" % variant
    target = os.path.join(out, name)
    os.makedirs(build, exist_ok=True)
    os.makedirs(out, exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall", "-Wno-unused-function",
             "-munsafe-fp-atomics", "-I" + CSRC] + (VARIANTS[variant] if variant else [])
    tool = [_toolchain_id(hipcc)]
    objs, jobs_list = [], []
    for s in srcs:
        o = os.path.join(build, os.path.basename(s) + ".o")
        objs.append(o)
        cmd = [hipcc] + flags + ["-c", s, "-o", o]
        if force or _stale(o, [s] + hdrs, cmd + tool):
            jobs_list.append((cmd, o, [s] + hdrs))

    def compile_one(job):
        cmd, o, deps = job
        _run(cmd)
        _stamp(o, deps, cmd + tool)

    if jobs_list:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(jobs_list)))) as ex:
            list(ex.map(compile_one, jobs_list))
    link = [hipcc, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", target] + objs
    tl = torch_lib_dir()
    if tl:
        link += ["-Wl,-rpath," + tl]
    if force or jobs_list or _stale(target, objs, link):
        _run(link)
        _stamp(target, objs, link)
    else:
        print("hip lib up to date")
    return target


def _toolchain_id(hipcc):
    try:
        return subprocess.check_output([hipcc, "--version"], stderr=subprocess.STDOUT, text=True).strip()
    except Exception:
        return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["host", "hip"])
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("--variant", choices=sorted(VARIANTS), help="experiment build of the HIP library only")
    a = ap.parse_args()
    if a.variant:
        print(build_hip(a.force, a.j, a.variant))
        return
    if a.only in (None, "host"):
        build_host(a.force)
    if a.only in (None, "hip"):
        build_hip(a.force, a.j)


if __name__ == "__main__":
    sys.exit(main())
