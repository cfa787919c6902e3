"""In-tree native build for torchbooster_amd (gfx950 only).

Builds ``torchbooster_amd/_C.so`` from ``csrc/``:

* ``*.hip``  -> device + launcher translation units, compiled by ``hipcc
  --offload-arch=gfx950`` against ``<hip/hip_runtime.h>`` only (no torch
  headers, so a kernel file rebuilds in seconds);
* ``*.cpp``  -> host runtime + bindings, compiled with the torch headers;
* one ``hipcc -shared`` link against torch's own libraries (``torch/lib``), so the
  extension shares torch's HIP runtime (same ``libamdhip64.so.7`` soname).

No hipify step, no CUDA sources, no multi-arch fat binaries.  Incremental builds
go through a generated ``build.ninja`` in ``build/``.

Usage: ``python -m torchbooster_amd._build [--clean] [-j N]``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
OUT = ROOT / "torchbooster_amd" / "_C.so"
# bounds-checked debug build (TBAMD_BOUNDS=1 loads it)
BUILD_BOUNDS = ROOT / "build_bounds"
OUT_BOUNDS = ROOT / "torchbooster_amd" / "_C_bounds.so"
ARCH = os.environ.get("TBAMD_ARCH", "gfx950")


def _torch_paths():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return tdir, inc


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = Path(rocm) / "bin" / "hipcc"
    return str(cand) if cand.exists() else "hipcc"


def write_ninja(debug: bool = False, bounds: bool = False) -> Path:
    tdir, tinc = _torch_paths()
    import torch

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    py_inc = sysconfig.get_paths()["include"]
    opt = "-O0 -g" if debug else "-O3"
    bdef = " -DTBAMD_BOUNDS" if bounds else ""
    ext = "_C_bounds" if bounds else "_C"
    build_dir = BUILD_BOUNDS if bounds else BUILD
    out = OUT_BOUNDS if bounds else OUT
    hip_flags = (
        f"{opt} -std=c++17 -fPIC --offload-arch={ARCH} -munsafe-fp-atomics "
        f"-I{CSRC} -Wno-unused-result -Wno-unused-command-line-argument{bdef}"
    )
    cpp_flags = (
        f"-O2 -std=c++17 -fPIC -I{CSRC} "
        + " ".join(f"-isystem {p}" for p in tinc)
        + f" -isystem {py_inc} -isystem {os.environ.get('ROCM_PATH', '/opt/rocm')}/include"
        f" -DTORCH_EXTENSION_NAME={ext} -DTORCH_API_INCLUDE_EXTENSION_H{bdef} "
        f"-D_GLIBCXX_USE_CXX11_ABI={abi} -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DHIPBLAS_V2 "
        "-D__HIP_NO_HALF_OPERATORS__=1 -D__HIP_NO_HALF_CONVERSIONS__=1 "
        "-Wno-unused-result -Wno-deprecated-declarations -Wno-unused-command-line-argument"
    )
    tlib = tdir / "lib"
    ldflags = (
        f"-shared -fPIC --offload-arch={ARCH} -L{tlib} -Wl,-rpath,{tlib} "
        "-lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lamdhip64"
    )
    hip_srcs = sorted(CSRC.glob("*.hip"))
    cpp_srcs = sorted(CSRC.glob("*.cpp"))
    headers = sorted(CSRC.glob("*.h"))
    hipcc = _hipcc()
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"hipflags = {hip_flags}",
        f"cppflags = {cpp_flags}",
        f"ldflags = {ldflags}",
        "rule hip",
        "  command = $hipcc $hipflags -x hip -c $in -o $out",
        "  description = HIP $in",
        "rule cpp",
        "  command = $hipcc -x c++ $cppflags -c $in -o $out",
        "  description = CXX $in",
        "rule link",
        "  command = $hipcc $in $ldflags -o $out",
        "  description = LINK $out",
    ]
    objs = []
    hdeps = " ".join(str(h) for h in headers)
    for s in hip_srcs:
        o = build_dir / (s.stem + ".hip.o")
        objs.append(o)
        lines.append(f"build {o}: hip {s} | {hdeps}")
    for s in cpp_srcs:
        o = build_dir / (s.stem + ".cpp.o")
        objs.append(o)
        lines.append(f"build {o}: cpp {s} | {hdeps}")
    lines.append(f"build {out}: link " + " ".join(str(o) for o in objs))
    lines.append(f"default {out}")
    build_dir.mkdir(parents=True, exist_ok=True)
    nf = build_dir / "build.ninja"
    text = "\n".join(lines) + "\n"
    if not nf.exists() or nf.read_text() != text:
        nf.write_text(text)
    return nf


def build(jobs: int | None = None, clean: bool = False, verbose: bool = False, debug: bool = False,
          bounds: bool = False) -> Path:
    bdir = BUILD_BOUNDS if bounds else BUILD
    if clean and bdir.exists():
        shutil.rmtree(bdir)
    nf = write_ninja(debug=debug, bounds=bounds)
    ninja = shutil.which("ninja")
    if ninja is None:
        try:
            import ninja as _nj  # type: ignore

            ninja = str(Path(_nj.BIN_DIR) / "ninja")
        except Exception as e:  # pragma: no cover
            raise RuntimeError("ninja is required to build torchbooster_amd") from e
    if jobs is None:
        jobs = min(16, os.cpu_count() or 4)
    cmd = [ninja, "-f", str(nf), "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True, cwd=str(bdir))
    return OUT_BOUNDS if bounds else OUT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--bounds", action="store_true", help="bounds-checked debug build -> _C_bounds.so")
    a = ap.parse_args(argv)
    out = build(a.j, a.clean, a.v, a.debug, a.bounds)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
