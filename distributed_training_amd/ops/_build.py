"""In-tree native build of the ``_C`` extension (HIP kernels for gfx950 +
RCCL communicator + pybind11 bindings).

No torch.utils.cpp_extension / hipify: every ``.hip`` file is CDNA4 source
compiled directly with ``hipcc --offload-arch=gfx950``; host C++ files are
compiled with ``g++`` against the PyTorch headers; the shared object is
linked with ``hipcc`` into ``distributed_training_amd/_C*.so`` so it travels
with the repository snapshot to the GPU box.

Incremental: an object is rebuilt only when the hash of (its source, every
header in csrc/, the compile command) changes.

Usage::

    python -m distributed_training_amd.ops._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Any, List, Sequence

PKG_DIR = Path(__file__).resolve().parent.parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR.parent / "build" / "dta_native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("DTA_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG_DIR / f"{EXT_NAME}{suffix}"


def _torch_paths() -> Any:
    import torch  # noqa: WPS433 (import inside: build-only dependency)

    tdir = Path(torch.__file__).resolve().parent
    incs = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir, incs, abi


def _py_include() -> str:
    return sysconfig.get_paths()["include"]


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(CSRC.glob("*.h")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


# attention.hip: MFMA accumulators in the VGPR form.  The default heuristic picks the AGPR
# form for the D = 128 backward kernels (one wave per SIMD, 512 registers) and then shuttles
# the dK/dV / dQ accumulators between the two files every loop iteration (868 / 416
# v_accvgpr moves per kernel vs 338 / 154 in the VGPR form).  No SLP vectorisation: it packs
# the softmax's f32 multiplies into v_pk_mul_f32 on misaligned register pairs and re-aligns them
# with v_mov / v_alignbit / v_perm (65-100 extra VALU ops per kernel in MFMA gaps; the guide's
# "packed f32 VALU beside MFMAs is an anti-lever").
_PER_FILE_FLAGS = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"]}


def _compile_cmds() -> List[tuple]:
    tdir, incs, abi = _torch_paths()
    hipcc = str(ROCM / "bin" / "hipcc")
    hip_flags = [
        hipcc, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC",
        "-munsafe-fp-atomics", f"-I{CSRC}",
    ] + os.environ.get("DTA_HIP_EXTRA_FLAGS", "").split()  # e.g. -DDTA_MP_PHASES (diagnostic builds)
    cxx = os.environ.get("CXX", "g++")
    cpp_flags = [
        cxx, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
        "-DTORCH_API_INCLUDE_EXTENSION_H", f"-I{CSRC}", f"-I{ROCM / 'include'}",
        f"-I{_py_include()}", f"-I{_pybind_include()}",
    ] + [f"-I{p}" for p in incs] + ["-w"]
    jobs = []
    for src in sorted(CSRC.glob("*.hip")):
        jobs.append((src, hip_flags + _PER_FILE_FLAGS.get(src.name, []) + ["-c", str(src)]))
    for src in sorted(CSRC.glob("*.cpp")):
        jobs.append((src, cpp_flags + ["-c", str(src)]))
    return jobs


def _obj_for(src: Path) -> Path:
    return BUILD_DIR / (src.name + ".o")


def _run(cmd: Sequence[str]) -> None:
    res = subprocess.run(list(cmd), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"native build failed:\n$ {' '.join(cmd)}\n{res.stdout}")


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> Path:
    """Compile every csrc/ source for gfx950 and link the _C extension."""
    if shutil.which(str(ROCM / "bin" / "hipcc")) is None:
        raise RuntimeError(f"hipcc not found under {ROCM}")
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    hdr = _headers_digest()
    todo = []
    objs = []
    for src, cmd in _compile_cmds():
        obj = _obj_for(src)
        full = cmd + ["-o", str(obj)]
        digest = hashlib.sha256((hdr + " ".join(full)).encode() + src.read_bytes()).hexdigest()
        stamp = obj.with_suffix(".stamp")
        objs.append(obj)
        if force or not obj.exists() or not stamp.exists() or stamp.read_text() != digest:
            todo.append((src, full, stamp, digest))
    if todo:
        n = jobs or min(len(todo), max(1, (os.cpu_count() or 4)))
        n = min(n, 16)
        if verbose:
            print(f"[dta build] compiling {len(todo)} file(s) with {n} job(s)", file=sys.stderr)

        def work(item: str) -> Any:
            src, full, stamp, digest = item
            _run(full)
            stamp.write_text(digest)
            return src.name

        with ThreadPoolExecutor(max_workers=n) as ex:
            for name in ex.map(work, todo):
                if verbose:
                    print(f"[dta build]   ok {name}", file=sys.stderr)
    out = ext_path()
    newest = max(o.stat().st_mtime for o in objs)
    if force or todo or not out.exists() or out.stat().st_mtime < newest:
        tdir, _, _ = _torch_paths()
        link = [
            str(ROCM / "bin" / "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}",
            *map(str, objs), "-o", str(out) + ".tmp",
            f"-L{tdir / 'lib'}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", f"-L{ROCM / 'lib'}", "-lamdhip64", "-ldl",
            f"-Wl,-rpath,{tdir / 'lib'}",
        ]
        _run(link)
        os.replace(str(out) + ".tmp", out)
        if verbose:
            print(f"[dta build] linked {out}", file=sys.stderr)
    return out


def main(argv: Any = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    args = ap.parse_args(argv)
    build(force=args.force, jobs=args.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
