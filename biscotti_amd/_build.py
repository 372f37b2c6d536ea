"""In-tree build of the native parts of biscotti_amd.

* ``_biscotti_rt``  -- host runtime (C++17, pybind11): crypto, ledger, protocol FSM.
* ``libbiscotti_hip.so`` -- CDNA4 (gfx950) HIP kernels with a C ABI, loaded through ctypes.

Both land next to this file, so a ``gpurun`` snapshot carries them to the GPU box.  Builds are
incremental (per-object mtime check) and parallel.

Usage: ``python -m biscotti_amd._build [--runtime] [--kernels] [--force]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build"
RT_NAME = "_biscotti_rt" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")
HIP_LIB = "libbiscotti_hip.so"
ARCH = "gfx950"   # MI355X (CDNA4) only
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _jobs() -> int:
    try:
        n = int(os.environ.get("MAX_JOBS", "0"))
    except ValueError:
        n = 0
    return max(1, min(n or (os.cpu_count() or 4), 16))


def _stale(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[0]} {cmd[-1]}")


COMPILED: list = []   # the objects and libraries this process compiled or linked (build_record)


def _compile_many(jobs: list[tuple[list[str], Path, list[Path]]], force: bool) -> list[Path]:
    todo = [(c, o) for c, o, deps in jobs if force or _stale(o, deps)]
    if todo:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            list(ex.map(lambda co: _run(co[0]), todo))
        COMPILED.extend(str(o.relative_to(PKG.parent)) for _, o in todo)
    return [o for _, o, _ in jobs]


def build_record(mode: str, t0: float) -> Path:
    """build/build_record.json: what this build compiled (every object when forced), the toolchain, and the
    sha256 of each source and each built library -- evidence that the libraries in the tree are this tree's."""
    import hashlib
    import json
    import time

    def sha(p: Path) -> str:
        return hashlib.sha256(p.read_bytes()).hexdigest()[:16]

    srcs = sorted(list((CSRC / "runtime").glob("*.[ch]pp")) + list((CSRC / "kernels").glob("*.hip"))
                  + list((CSRC / "kernels").glob("*.h")))
    libs = [PKG / RT_NAME, PKG / HIP_LIB]
    rec = {"mode": mode, "arch": ARCH, "seconds": round(time.time() - t0, 1),
           "finished_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "compiled": sorted(COMPILED), "n_compiled": len(COMPILED),
           "hipcc": subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.splitlines()[:2]
           if Path(HIPCC).exists() else None,
           "sources_sha256_16": {str(p.relative_to(PKG.parent)): sha(p) for p in srcs},
           "libraries_sha256_16": {str(p.relative_to(PKG.parent)): sha(p) for p in libs if p.exists()}}
    BUILD.mkdir(parents=True, exist_ok=True)
    out = BUILD / "build_record.json"
    out.write_text(json.dumps(rec, indent=1) + "\n")
    return out


def build_runtime(force: bool = False) -> Path:
    src_dir = CSRC / "runtime"
    out_dir = BUILD / "runtime"
    out_dir.mkdir(parents=True, exist_ok=True)
    import pybind11

    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{src_dir}"]
    headers = sorted(src_dir.glob("*.hpp"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-sign-compare"]
    extra = os.environ.get("BISCOTTI_RT_CXXFLAGS", "").split()
    jobs = []
    for src in sorted(src_dir.glob("*.cpp")):
        obj = out_dir / (src.stem + ".o")
        jobs.append((["g++", *flags, *extra, *inc, "-c", str(src), "-o", str(obj)], obj, [src, *headers]))
    objs = _compile_many(jobs, force)
    target = PKG / RT_NAME
    if force or _stale(target, objs):
        _run(["g++", "-shared", "-pthread", *extra, "-o", str(target), *map(str, objs)])
    return target


def build_selftest(sanitize: bool | str = True) -> Path:
    """Native self-test of the host runtime (csrc/selftest) on the host code: sanitize True / "asan" -- ASan + UBSan;
    "tsan" -- ThreadSanitizer (the pool / dispatcher stress: `selftest_tsan pool`); False -- none."""
    rt_dir = CSRC / "runtime"
    mode = "asan" if sanitize is True else (sanitize or "")
    out = BUILD / (f"selftest_{mode}" if mode else "selftest")
    out.parent.mkdir(parents=True, exist_ok=True)
    srcs = [s for s in sorted(rt_dir.glob("*.cpp")) if s.name != "bindings.cpp"]
    srcs.append(CSRC / "selftest" / "selftest.cpp")
    flags = ["-O1", "-g", "-std=c++17", "-pthread", f"-I{rt_dir}", "-fno-omit-frame-pointer"]
    if mode == "asan":
        flags += ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    elif mode == "tsan":
        flags += ["-fsanitize=thread"]
    _run(["g++", *flags, *map(str, srcs), "-o", str(out)])
    return out


def build_kernels(force: bool = False) -> Path:
    if not Path(HIPCC).exists() and shutil.which("hipcc") is None:
        raise RuntimeError("hipcc not found; cannot build the gfx950 kernels")
    hipcc = HIPCC if Path(HIPCC).exists() else shutil.which("hipcc")
    src_dir = CSRC / "kernels"
    out_dir = BUILD / "kernels"
    out_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(src_dir.glob("*.h")) + sorted(src_dir.glob("*.hpp"))
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", f"-I{src_dir}"]
    extra = os.environ.get("BISCOTTI_HIP_FLAGS", "").split()
    jobs = []
    for src in sorted(src_dir.glob("*.hip")):
        obj = out_dir / (src.stem + ".o")
        jobs.append(([hipcc, *flags, *extra, "-c", str(src), "-o", str(obj)], obj, [src, *headers]))
    objs = _compile_many(jobs, force)
    target = PKG / HIP_LIB
    if force or _stale(target, objs):
        _run([hipcc, "-shared", f"--offload-arch={ARCH}", "-o", str(target), *map(str, objs)])
    return target


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runtime", action="store_true")
    ap.add_argument("--kernels", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--sanitize", action="store_true",
                    help="build and run the host-runtime self-test under ASan + UBSan")
    ap.add_argument("--tsan", action="store_true",
                    help="build the host-runtime self-test under ThreadSanitizer and run its pool / dispatcher stress")
    a = ap.parse_args(argv)
    if a.tsan:
        exe = build_selftest("tsan")
        print("built", exe)
        r = subprocess.run([str(exe), "pool"], env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1"))
        raise SystemExit(r.returncode)
    if a.sanitize:
        exe = build_selftest(True)
        print("built", exe)
        r = subprocess.run([str(exe)], env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
        raise SystemExit(r.returncode)
    both = not (a.runtime or a.kernels)
    if a.runtime or both:
        print("built", build_runtime(a.force))
    if a.kernels or both:
        print("built", build_kernels(a.force))


if __name__ == "__main__":
    main()
