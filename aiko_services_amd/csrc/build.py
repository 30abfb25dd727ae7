"""In-tree native build for aiko_services_amd (gfx950 only).

Compiles every ``csrc/kernels/*.hip`` (device code, no torch headers: seconds per file),
``csrc/runtime/*.cpp`` and ``csrc/bindings.cpp`` (torch operator registrations) with
``hipcc --offload-arch=gfx950`` and links them into ``aiko_services_amd/_C.so``, which is
loaded with ``torch.ops.load_library``.  Objects are cached under ``csrc/.build`` keyed by a
hash of the source + flags + headers, so rebuilds only touch changed files.

No hipify, no CUDA, no multi-arch: the code objects are built for MI355X (gfx950) alone.

Usage:  python -m aiko_services_amd.csrc.build [--force] [--debug] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

CSRC = Path(__file__).resolve().parent
PKG = CSRC.parent
OUT = PKG / "_C.so"
BUILD = CSRC / ".build"
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (need ROCm at /opt/rocm)")


def _torch_paths():
    import torch  # noqa: F401  (import only to locate headers/libs)
    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    return inc, root / "lib"


def _hash(paths, flags) -> str:
    h = hashlib.sha1()
    for p in paths:
        h.update(Path(p).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def sources():
    kernels = sorted((CSRC / "kernels").glob("*.hip"))
    runtime = sorted((CSRC / "runtime").glob("*.cpp"))
    return kernels, runtime, CSRC / "bindings.cpp"


def _compile(src: Path, flags, headers) -> Path:
    key = _hash([src, *headers], flags)
    obj = BUILD / f"{src.stem}.{key}.o"
    if obj.exists():
        return obj
    tmp = obj.with_suffix(".tmp.o")
    cmd = [_hipcc(), *flags, "-c", str(src), "-o", str(tmp)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    tmp.rename(obj)
    return obj


def build_host_modules(force: bool = False, verbose: bool = True) -> list:
    """CPython extension modules of the control plane (``csrc/host/*.c`` ->
    ``aiko_services_amd/_<name>.so``): plain C against the Python C API, no torch, no HIP, so
    CPU-only processes (brokers, registrars, CPU tests) load them too."""
    BUILD.mkdir(exist_ok=True)
    py_inc = sysconfig.get_paths()["include"]
    cc = os.environ.get("CC") or shutil.which("gcc") or shutil.which("cc") or "cc"
    flags = ["-O2", "-shared", "-fPIC", "-Wall", "-Werror", "-I", py_inc]
    out = []
    for src in sorted((CSRC / "host").glob("*.c")):
        so = PKG / f"_{src.stem}.so"
        key = _hash([src], flags)
        stamp = BUILD / f"host_{src.stem}.stamp"
        if so.exists() and stamp.exists() and stamp.read_text() == key and not force:
            out.append(so)
            continue
        tmp = so.with_suffix(".tmp.so")
        cmd = [cc, *flags, str(src), "-o", str(tmp)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        tmp.replace(so)
        stamp.write_text(key)
        if verbose:
            print(f"[aiko build] built {so}")
        out.append(so)
    return out


def build(force: bool = False, debug: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    # the host modules are optional (utils/sexpr.py falls back to the pure-Python codec): a
    # compile error there must not abort the GPU kernel build
    try:
        build_host_modules(force=force, verbose=verbose)
    except RuntimeError as e:
        print(f"[aiko build] host modules skipped (pure-Python fallbacks in use): {e}", file=sys.stderr)
    BUILD.mkdir(exist_ok=True)
    kernels, runtime, binding = sources()
    tinc, tlib = _torch_paths()
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = ["-fPIC", "-std=c++17", *opt, "-Wno-unused-result", "-Wno-unused-command-line-argument"]
    dev_flags = [*common, f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                 "-I", str(CSRC / "kernels")]
    py_inc = sysconfig.get_paths()["include"]
    host_flags = [*common, "-D_GLIBCXX_USE_CXX11_ABI=1", "-DTORCH_API_INCLUDE_EXTENSION_H",
                  "-DTORCH_EXTENSION_NAME=_C", "-I", str(CSRC), "-I", py_inc,
                  *sum([["-isystem", str(p)] for p in tinc], []), "-Wno-deprecated-declarations"]
    import torch
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    host_flags = [f for f in host_flags if not f.startswith("-D_GLIBCXX_USE_CXX11_ABI")]
    host_flags.append(f"-D_GLIBCXX_USE_CXX11_ABI={abi}")
    headers_dev = sorted((CSRC / "kernels").glob("*.h"))
    headers_host = sorted((CSRC / "runtime").glob("*.h")) + headers_dev
    if force:
        for o in BUILD.glob("*.o"):
            o.unlink()
    jobs = jobs or min(8, os.cpu_count() or 4)
    work = [(k, dev_flags, headers_dev) for k in kernels]
    # runtime .cpp and bindings are host code that uses the HIP runtime API only
    work += [(r, [*host_flags, f"--offload-arch={ARCH}"], headers_host) for r in runtime]
    work.append((binding, [*host_flags, f"--offload-arch={ARCH}"], headers_host))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda a: _compile(*a), work))
    link_key = _hash(objs, ["link"])
    stamp = BUILD / "link.stamp"
    if OUT.exists() and stamp.exists() and stamp.read_text() == link_key and not force:
        if verbose:
            print(f"[aiko build] up to date: {OUT}")
        return OUT
    tmp = OUT.with_suffix(".tmp.so")
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
           "-L", str(tlib), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           f"-Wl,-rpath,{tlib}"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    tmp.replace(OUT)
    stamp.write_text(link_key)
    # prune stale objects
    keep = {o.name for o in objs}
    for o in BUILD.glob("*.o"):
        if o.name not in keep:
            o.unlink()
    if verbose:
        print(f"[aiko build] linked {OUT} from {len(objs)} objects")
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, debug=a.debug, jobs=a.j)


if __name__ == "__main__":
    sys.exit(main())
