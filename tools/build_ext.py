#!/usr/bin/env python3
"""Build the HIP kernel library for gfx950 with hipcc directly (no hipify, no torch JIT cache).

Every ``csrc/**/*.hip`` / ``*.cpp`` is compiled to an object under ``build/`` (in parallel, incremental on mtime),
then linked into ``torchmetrics_amd/_C/libtm_amd.so``, which registers the ``torch.ops.tm_amd.*`` operators.
``csrc/bindings/fastcall.cpp`` becomes the CPython extension ``torchmetrics_amd/_C/_fastcall.so`` (dispatcher-free
entry points of the per-batch hot ops), linked against ``libtm_amd.so``.

Usage: ``python tools/build_ext.py [-j N] [--force] [--arch gfx950]``
"""
import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "obj"
OUT = ROOT / "torchmetrics_amd" / "_C" / "libtm_amd.so"
FAST_SRC = CSRC / "bindings" / "fastcall.cpp"
FAST_OUT = ROOT / "torchmetrics_amd" / "_C" / "_fastcall.so"


def _torch_paths():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    lib = tdir / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _sources():
    return sorted(p for p in CSRC.rglob("*") if p.suffix in (".hip", ".cpp") and p.parent.name != "bindings")


def _headers_mtime():
    hs = [p.stat().st_mtime for p in CSRC.rglob("*.h")]
    return max(hs) if hs else 0.0


def compile_one(src: Path, arch: str, force: bool, hdr_mtime: float) -> Path:
    inc, _, abi = _torch_paths()
    obj = BUILD / (src.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime):
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = [
        "hipcc",
        f"--offload-arch={arch}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        "-munsafe-fp-atomics",
        # kernel arguments preloaded into SGPRs at wave launch (the CP fills them once per dispatch) instead of one
        # s_load per wave at kernel start: measured -0.23 us per 16 MB streaming launch (profiles/r05_region_mb_kernarg.jsonl)
        "-mllvm",
        "-amdgpu-kernarg-preload-count=16",
        *[f"-I{p}" for p in inc],
        f"-I{CSRC}",
        "-c",
        str(src),
        "-o",
        str(obj),
    ]
    if src.suffix == ".cpp":
        cmd.insert(1, "-x")
        cmd.insert(2, "hip")
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"hipcc failed on {src}")
    return obj


def link(objs, out: Path) -> None:
    _, lib, _ = _torch_paths()
    out.parent.mkdir(parents=True, exist_ok=True)
    cmd = [
        "hipcc",
        "-shared",
        "-fPIC",
        *map(str, objs),
        "-o",
        str(out),
        f"-L{lib}",
        "-lc10",
        "-lc10_hip",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_hip",
        f"-Wl,-rpath,{lib}",
    ]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError("link failed")


def build_fastcall(force: bool = False, verbose: bool = True) -> Path:
    """Host-only C++ (no device code): Python + torch_python headers, linked to libtm_amd.so via $ORIGIN."""
    import sysconfig

    if not force and FAST_OUT.exists() and FAST_OUT.stat().st_mtime >= max(FAST_SRC.stat().st_mtime, OUT.stat().st_mtime):
        if verbose:
            print(f"[build_ext] {FAST_OUT.relative_to(ROOT)} up to date")
        return FAST_OUT
    inc, lib, abi = _torch_paths()
    cmd = [
        "g++", "-O2", "-fPIC", "-shared", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1", "-Wno-deprecated-declarations",
        f"-I{sysconfig.get_paths()['include']}", *[f"-I{p}" for p in inc], "-I/opt/rocm/include",
        str(FAST_SRC), "-o", str(FAST_OUT),
        f"-L{OUT.parent}", "-ltm_amd", f"-L{lib}", "-ltorch_python", "-ltorch", "-ltorch_cpu", "-lc10",
        "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{lib}", "-ldl",
    ]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError("fastcall build failed")
    if verbose:
        print(f"[build_ext] built {FAST_OUT.relative_to(ROOT)}")
    return FAST_OUT


def build(arch: str = "gfx950", jobs: int = 8, force: bool = False, verbose: bool = True) -> Path:
    srcs = _sources()
    hdr = _headers_mtime()
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: compile_one(s, arch, force, hdr), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if force or not OUT.exists() or OUT.stat().st_mtime < newest:
        link(objs, OUT)
        if verbose:
            print(f"[build_ext] linked {OUT.relative_to(ROOT)} from {len(objs)} objects ({arch})")
    elif verbose:
        print(f"[build_ext] {OUT.relative_to(ROOT)} up to date")
    build_fastcall(force=force, verbose=verbose)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--arch", default=os.environ.get("PYTORCH_ROCM_ARCH", "gfx950"))
    a = ap.parse_args()
    build(a.arch, a.jobs, a.force)
