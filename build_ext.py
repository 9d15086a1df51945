#!/usr/bin/env python3
"""Build the in-tree sftamd extension for gfx950 (MI355X).

Compiles every ``csrc/*.hip`` with ``hipcc --offload-arch=gfx950`` and every ``csrc/*.cpp``
(host-only code) with ``g++``, in parallel, then links ``llm_fine_tune_distributed_amd/_C.so``
against libtorch. No hipify, no JIT cache: the .so lives in the source tree so it travels to
the GPU box with the snapshot. Incremental: objects newer than their sources/headers are reused.

    python build_ext.py [--jobs N] [--force] [--debug]

``--debug`` builds a separate ``_C_debug.so`` (-O1 -g, device asserts ``SFT_DASSERT`` compiled in, objects
under build/obj_debug); the loader picks it when ``SFTAMD_DEBUG=1`` (SURVEY §5.2 triage mode).
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
OBJ_RELEASE = os.path.join(ROOT, "build", "obj")
OBJ_DEBUG = os.path.join(ROOT, "build", "obj_debug")
OUT_RELEASE = os.path.join(ROOT, "llm_fine_tune_distributed_amd", "_C.so")
OUT_DEBUG = os.path.join(ROOT, "llm_fine_tune_distributed_amd", "_C_debug.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, os.path.join(tdir, "lib"), abi


def newer(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return False
    t = os.path.getmtime(obj)
    return all(os.path.getmtime(d) <= t for d in deps)


def main(argv=None) -> str:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true", help="_C_debug.so: -O1 -g, device asserts on")
    ap.add_argument("--save-temps", action="store_true", help="keep .s for inspection (build/obj)")
    args = ap.parse_args(argv)

    inc, libdir, abi = torch_paths()
    OBJ, OUT = (OBJ_DEBUG, OUT_DEBUG) if args.debug else (OBJ_RELEASE, OUT_RELEASE)
    os.makedirs(OBJ, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    common = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-fPIC", "-std=c++17",
              "-DTORCH_EXTENSION_NAME=sftamd", "-Wno-unused-result"] + [f"-I{p}" for p in inc] + [f"-I{CSRC}"]
    opt = ["-O1", "-g", "-DSFTAMD_DEBUG"] if args.debug else ["-O3", "-DNDEBUG"]
    hip_flags = [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-fgpu-flush-denormals-to-zero"] + opt + common
    if args.save_temps:
        hip_flags.append("-save-temps=obj")
    cxx_flags = opt + common + [f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__=1"]

    jobs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp"))):
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        if not args.force and newer(obj, [src, __file__] + headers):
            continue
        if src.endswith(".hip"):
            cmd = [os.path.join(ROCM, "bin", "hipcc"), "-c", src, "-o", obj] + hip_flags
        else:
            cmd = ["g++", "-c", src, "-o", obj] + cxx_flags
        jobs.append((src, cmd))

    def run(job):
        src, cmd = job
        r = subprocess.run(cmd, cwd=OBJ, capture_output=True, text=True)
        return src, r

    failed = False
    with ThreadPoolExecutor(max_workers=max(1, args.jobs)) as ex:
        for src, r in ex.map(run, jobs):
            rel = os.path.relpath(src, ROOT)
            if r.returncode != 0:
                failed = True
                print(f"[build_ext] FAILED {rel}\n{r.stdout}\n{r.stderr}", file=sys.stderr)
            else:
                print(f"[build_ext] compiled {rel}")
    if failed:
        raise SystemExit(1)

    objs = sorted(glob.glob(os.path.join(OBJ, "*.o")))
    srcs = {os.path.basename(p) + ".o" for p in glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp"))}
    objs = [o for o in objs if os.path.basename(o) in srcs]
    if args.force or jobs or not newer(OUT, objs):
        cmd = [os.path.join(ROCM, "bin", "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs + [
            f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{libdir}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            print(f"[build_ext] link failed\n{r.stdout}\n{r.stderr}", file=sys.stderr)
            raise SystemExit(1)
        print(f"[build_ext] linked {os.path.relpath(OUT, ROOT)}")
    return OUT


if __name__ == "__main__":
    main()
