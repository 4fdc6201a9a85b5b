"""In-tree build driver for the native extensions.

Two shared objects are produced next to this file:

* ``_kernels<EXT_SUFFIX>`` — every HIP/CDNA4 kernel of the framework, compiled by ``hipcc
  --offload-arch=gfx950`` from ``csrc/kernels/*.hip``.  The binding layer
  (``csrc/kernels/bindings.cpp``) is plain pybind11 taking raw device pointers and a
  ``hipStream_t`` — no torch headers, no hipify step, no CUDA compatibility layer.
* ``_native<EXT_SUFFIX>`` — the host-side C++ runtime (TCP control plane, message
  serialisation, dataset parsers, augmentation, hardware info, env loader, thread affinity),
  compiled by g++ from ``csrc/native/*.cpp``.

Objects are cached under ``build/`` keyed by source mtime + flags, compiled in parallel.
Usage: ``python -m dcnn_amd._build [--force] [--verbose] [--only kernels|native]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
BUILD = ROOT / "build"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("DCNN_OFFLOAD_ARCH", "gfx950")


def _pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _headers(dirpath: Path):
    return sorted(list(dirpath.glob("*.h")) + list(dirpath.glob("*.hpp")))


def _needs_build(obj: Path, src: Path, deps, flags_sig: str) -> bool:
    stamp = obj.with_suffix(obj.suffix + ".sig")
    if not obj.exists() or not stamp.exists():
        return True
    if stamp.read_text() != flags_sig:
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *deps])


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    if verbose and r.stdout.strip():
        print(r.stdout)
    return r.stdout


def _compile_many(jobs, verbose, max_workers):
    todo = [(cmd, obj, sig) for (cmd, obj, sig, need) in jobs if need]
    if not todo:
        return
    with cf.ThreadPoolExecutor(max_workers=max_workers) as ex:
        futs = {ex.submit(_run, cmd, verbose): (obj, sig) for cmd, obj, sig in todo}
        for f in cf.as_completed(futs):
            obj, sig = futs[f]
            f.result()
            obj.with_suffix(obj.suffix + ".sig").write_text(sig)


def build_kernels(force=False, verbose=False, max_workers=None):
    src_dir = PKG / "csrc" / "kernels"
    out_dir = BUILD / "kernels"
    out_dir.mkdir(parents=True, exist_ok=True)
    incs = [f"-I{p}" for p in _pybind_includes()] + [f"-I{src_dir}"]
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              "-Wno-unused-result", "-DNDEBUG"]
    hdrs = _headers(src_dir)
    jobs, objs = [], []
    for src in sorted(src_dir.glob("*.hip")) + sorted(src_dir.glob("*.cpp")):
        obj = out_dir / (src.stem + ".o")
        lang = ["-x", "hip"] if src.suffix == ".hip" else []
        cmd = [HIPCC, *common, *incs, *lang, "-c", str(src), "-o", str(obj)]
        sig = hashlib.sha1(" ".join(cmd).encode()).hexdigest()
        jobs.append((cmd, obj, sig, force or _needs_build(obj, src, hdrs, sig)))
        objs.append(obj)
    _compile_many(jobs, verbose, max_workers or min(8, os.cpu_count() or 4))
    target = PKG / f"_kernels{EXT_SUFFIX}"
    if force or not target.exists() or any(o.stat().st_mtime > target.stat().st_mtime for o in objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(target), "-ldl"],
             verbose)
    return target


def build_native(force=False, verbose=False, max_workers=None):
    src_dir = PKG / "csrc" / "native"
    out_dir = BUILD / "native"
    out_dir.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    incs = [f"-I{p}" for p in _pybind_includes()] + [f"-I{src_dir}"]
    san = os.environ.get("DCNN_NATIVE_SANITIZE", "")  # e.g. "address,undefined" or "thread"
    flags = ["-O2" if san else "-O3", "-fPIC", "-std=c++17", "-pthread", "-Wall", "-Wno-unused-function",
             "-fvisibility=hidden"]
    if san:
        flags += [f"-fsanitize={san}", "-fno-omit-frame-pointer", "-g"]
    hdrs = _headers(src_dir)
    jobs, objs = [], []
    for src in sorted(src_dir.glob("*.cpp")):
        obj = out_dir / (src.stem + (".san" if san else "") + ".o")
        cmd = [cxx, *flags, *incs, "-c", str(src), "-o", str(obj)]
        sig = hashlib.sha1(" ".join(cmd).encode()).hexdigest()
        jobs.append((cmd, obj, sig, force or _needs_build(obj, src, hdrs, sig)))
        objs.append(obj)
    _compile_many(jobs, verbose, max_workers or min(8, os.cpu_count() or 4))
    name = "_native_san" if san else "_native"
    target = PKG / f"{name}{EXT_SUFFIX}"
    if force or not target.exists() or any(o.stat().st_mtime > target.stat().st_mtime for o in objs):
        link_flags = [f"-fsanitize={san}"] if san else []
        _run([cxx, "-shared", "-fPIC", "-pthread", *link_flags, *map(str, objs), "-o", str(target), "-lz", "-ldl"],
             verbose)
    return target


# kernel-library / native objects the C++ host API links (the pybind layers stay out)
_HOST_SKIP_KERNELS = {"bindings", "runtime", "rccl"}
_HOST_NATIVE = ("cpu_ops", "cpu_gemm", "threadpool", "jpeg", "comm")


def build_host(force=False, verbose=False, max_workers=None):
    """C++ host API (csrc/host): ``libdcnn.so`` next to this file (host layers + the HIP kernel
    library + the native CPU kernels, no Python) and the C++ examples (examples/cpp/*.cpp) as
    executables under ``dcnn_amd/bin/``."""
    build_native(force, verbose, max_workers)
    build_kernels(force, verbose, max_workers)
    src_dir = PKG / "csrc" / "host"
    out_dir = BUILD / "host"
    out_dir.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    inc = [f"-I{src_dir}"]
    cflags = ["-O3", "-fPIC", "-std=c++17", "-pthread", "-Wall", "-Wno-unused-function"]
    hflags = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result", "-DNDEBUG"]
    hdrs = _headers(src_dir / "dcnn") + _headers(PKG / "csrc" / "kernels") + _headers(PKG / "csrc" / "native")
    jobs, objs = [], []
    for src in sorted(src_dir.glob("*.cpp")) + sorted(src_dir.glob("*.hip")):
        obj = out_dir / (src.stem + ".o")
        if src.suffix == ".hip":
            cmd = [HIPCC, *hflags, *inc, "-x", "hip", "-c", str(src), "-o", str(obj)]
        else:
            cmd = [cxx, *cflags, *inc, "-c", str(src), "-o", str(obj)]
        sig = hashlib.sha1(" ".join(cmd).encode()).hexdigest()
        jobs.append((cmd, obj, sig, force or _needs_build(obj, src, hdrs, sig)))
        objs.append(obj)
    _compile_many(jobs, verbose, max_workers or min(8, os.cpu_count() or 4))
    kobjs = [o for o in sorted((BUILD / "kernels").glob("*.o")) if o.stem not in _HOST_SKIP_KERNELS]
    nobjs = [BUILD / "native" / f"{n}.o" for n in _HOST_NATIVE]
    lib = PKG / "libdcnn.so"
    deps = objs + kobjs + nobjs
    if force or not lib.exists() or any(o.stat().st_mtime > lib.stat().st_mtime for o in deps):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, deps), "-o", str(lib), "-pthread",
              "-lz", "-ldl"], verbose)
    bins = []
    bin_dir = PKG / "bin"
    bin_dir.mkdir(exist_ok=True)
    for src in sorted((ROOT / "examples" / "cpp").glob("*.cpp")):
        exe = bin_dir / src.stem
        if force or not exe.exists() or exe.stat().st_mtime < max(lib.stat().st_mtime, src.stat().st_mtime,
                                                                  *(h.stat().st_mtime for h in hdrs)):
            _run([cxx, *cflags, *inc, str(src), "-o", str(exe), f"-L{PKG}", "-ldcnn", "-Wl,-rpath,$ORIGIN/..",
                  f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"], verbose)
        bins.append(exe)
    return lib, bins


def build_all(force=False, verbose=False):
    return build_native(force, verbose), build_kernels(force, verbose), build_host(force, verbose)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--only", choices=["kernels", "native", "host"])
    a = ap.parse_args(argv)
    if a.only in (None, "native"):
        print("built", build_native(a.force, a.verbose))
    if a.only in (None, "kernels"):
        print("built", build_kernels(a.force, a.verbose))
    if a.only in (None, "host"):
        lib, bins = build_host(a.force, a.verbose)
        print("built", lib, *bins)


if __name__ == "__main__":
    main()
