"""Build the two native extensions in-tree.

* ``_psx_host.so``  - C++17 host runtime (g++), no GPU dependency.
* ``_psx_hip.so``   - HIP kernels + C++ solver/graph driver (hipcc, gfx950).

Both are plain pybind11 modules (no torch headers), so a build takes seconds
and the HIP runtime symbols bind to the libamdhip64 that ``import torch``
already loaded (same SONAME).  Rebuilds are skipped when sources and flags are
unchanged (content hash stored next to the .so).

Usage:  python csrc/build.py [--force] [--host-only] [--hip-only] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "parameter-server-architecture-on-apache-kafka_amd")
ARCH = os.environ.get("PSX_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _pybind_includes():
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _hash(files, flags):
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(f.encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _up_to_date(out, digest):
    stamp = out + ".hash"
    return os.path.exists(out) and os.path.exists(stamp) and open(stamp).read().strip() == digest


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise RuntimeError(f"compile failed: {cmd[-1] if cmd else ''}")
    return r.stdout


def _local_includes(src):
    """src + every file it pulls in through #include "..." (recursively)."""
    seen, todo = [], [os.path.abspath(src)]
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.append(f)
        with open(f) as fh:
            for line in fh:
                line = line.strip()
                if line.startswith("#include \""):
                    todo.append(os.path.normpath(os.path.join(os.path.dirname(f), line.split('"')[1])))
    return seen


def _compile_link(compiler, sources, out, cflags, ldflags, jobs, objdir, headers=()):
    """Compile every source whose object is stale (its own content, the shared
    headers' and the flags hashed into <obj>.hash), then link."""
    os.makedirs(objdir, exist_ok=True)
    objs = []
    cmds = []
    for s in sources:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        dig = _hash(_local_includes(s), cflags)
        if _up_to_date(o, dig):
            continue
        cmds.append(([compiler] + cflags + ["-c", s, "-o", o], o, dig))

    def one(job):
        cmd, o, dig = job
        _run(cmd)
        open(o + ".hash", "w").write(dig)

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(one, cmds))
    tmp = out + ".tmp"
    _run([compiler] + objs + ["-shared", "-o", tmp] + ldflags)
    os.replace(tmp, out)


def build_host(force=False, jobs=8):
    sources = sorted(glob.glob(os.path.join(CSRC, "host", "*.cc"))) + [
        os.path.join(CSRC, "bindings", "host_module.cc")
    ]
    headers = sorted(glob.glob(os.path.join(CSRC, "host", "*.h"))) + [os.path.join(CSRC, "kernels", "solver_ctrl.h")]
    out = os.path.join(PKG, "_psx_host" + _ext_suffix())
    cflags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"] + [
        "-I" + i for i in _pybind_includes()
    ]
    ldflags = ["-pthread", "-lrt"]
    digest = _hash(sources + headers, cflags + ldflags)
    if not force and _up_to_date(out, digest):
        return out
    _compile_link("g++", sources, out, cflags, ldflags, jobs, os.path.join(ROOT, "build", "host"), headers)
    open(out + ".hash", "w").write(digest)
    return out


def build_hip(force=False, jobs=8):
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    sources = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))) + sorted(
        glob.glob(os.path.join(CSRC, "solver", "*.hip"))
    ) + sorted(glob.glob(os.path.join(CSRC, "comm", "*.hip"))) + sorted(
        glob.glob(os.path.join(CSRC, "runtime", "*.hip"))) + [os.path.join(CSRC, "bindings", "hip_module.hip")]
    headers = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")) + glob.glob(os.path.join(CSRC, "solver", "*.h")) +
                     glob.glob(os.path.join(CSRC, "comm", "*.h")) + glob.glob(os.path.join(CSRC, "runtime", "*.h")) +
                     [os.path.join(CSRC, "host", "capi.h"), os.path.join(CSRC, "host", "ctrl.h"),
                     os.path.join(CSRC, "host", "sink_record.h")])
    out = os.path.join(PKG, "_psx_hip" + _ext_suffix())
    cflags = [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-fvisibility=hidden",
        "-Wno-unused-result",
        "-munsafe-fp-atomics",
    ] + ["-I" + i for i in _pybind_includes()]
    ldflags = [f"--offload-arch={ARCH}", "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-ldl"]
    digest = _hash(sources + headers, cflags + ldflags)
    if not force and _up_to_date(out, digest):
        return out
    _compile_link(hipcc, sources, out, cflags, ldflags, jobs, os.path.join(ROOT, "build", "hip"), headers)
    open(out + ".hash", "w").write(digest)
    return out


def build_selftest(sanitize: str = "address,undefined", force=False):
    """Host-runtime self-test binary (csrc/tests/host_selftest.cc) under a
    sanitizer: "address,undefined" or "thread" (SURVEY.md §5.2)."""
    sources = [os.path.join(CSRC, "tests", "host_selftest.cc")] + sorted(glob.glob(os.path.join(CSRC, "host", "*.cc")))
    headers = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    tag = sanitize.replace(",", "_")
    out = os.path.join(ROOT, "build", "selftest", f"host_selftest_{tag}")
    flags = ["-O1", "-g", "-std=c++17", f"-fsanitize={sanitize}", "-fno-omit-frame-pointer"]
    if "undefined" in sanitize:
        flags.append("-fno-sanitize-recover=undefined")
    digest = _hash(sources + headers, flags)
    if not force and _up_to_date(out, digest):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    _run(["g++"] + flags + sources + ["-o", out + ".tmp", "-pthread", "-lrt"])
    os.replace(out + ".tmp", out)
    open(out + ".hash", "w").write(digest)
    return out


def build_all(force=False, host=True, hip=True, jobs=8):
    outs = []
    if host:
        outs.append(build_host(force, jobs))
    if hip:
        outs.append(build_hip(force, jobs))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--host-only", action="store_true")
    ap.add_argument("--hip-only", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args(argv)
    outs = build_all(a.force, host=not a.hip_only, hip=not a.host_only, jobs=a.j)
    for o in outs:
        print(o)


if __name__ == "__main__":
    main()
