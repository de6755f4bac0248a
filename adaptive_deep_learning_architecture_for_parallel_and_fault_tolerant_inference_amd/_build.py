"""In-tree native build (no setuptools / JIT cache).

* ``_C``        gfx950 HIP kernels + pybind11 bindings, built with hipcc
                (``--offload-arch=gfx950``), linked against the HIP runtime
                that torch already loaded (same SONAME libamdhip64.so.7).
* ``_runtime``  host C++17 runtime (framing transport, LZ4 frame codec,
                zfp-style reversible codec, membership store), built with g++.
* ``_comm``     native RCCL p2p layer (csrc/comm).
* ``_cpu``      OpenMP NHWC fp32 ops of the CPU execution path (csrc/cpu),
                built with g++ -fopenmp; hot loops carry AVX-512 / AVX2 /
                baseline clones picked at load time.

Objects go to ``build/``; the two ``.so`` files are written next to this
file so they travel to the GPU box with the repo snapshot.  Rebuilds are
incremental on source/header mtimes.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import List

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> List[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _newer(target: Path, deps: List[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def kernel_lib_path() -> Path:
    return PKG_DIR / f"_C{EXT}"


def runtime_lib_path() -> Path:
    return PKG_DIR / f"_runtime{EXT}"


# per-file extra compiler flags (none at present: -fno-slp-vectorize plus scalar storage on the F(4x4)
# transform measured 10-20 % slower per K chunk than the compiler's packed v_pk_add / v_pk_fma form,
# gpurun_out/r5k/wino4_exp.json)
FILE_FLAGS: dict = {}


def build_kernels(verbose: bool = False, jobs: int = 8) -> Path:
    src_dir = CSRC / "kernels"
    headers = list(src_dir.glob("*.h"))
    srcs = sorted(src_dir.glob("*.hip")) + sorted(src_dir.glob("*.cpp"))
    out_dir = BUILD / "kernels"
    out_dir.mkdir(parents=True, exist_ok=True)
    inc = _py_includes() + [f"-I{src_dir}"]
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
              "-fno-gpu-rdc", "-munsafe-fp-atomics", "-Wno-unused-result"] + inc

    def compile_one(src: Path) -> Path:
        obj = out_dir / (src.name + ".o")
        if _newer(obj, [src] + headers):
            cmd = common + FILE_FLAGS.get(src.name, []) + ["-c", str(src), "-o", str(obj)]
            if src.suffix == ".cpp":
                cmd = common + ["-x", "hip", "-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), flush=True)
            _run(cmd)
        return obj

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    lib = kernel_lib_path()
    if _newer(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib)] + [str(o) for o in objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
    return lib


def build_runtime(verbose: bool = False, jobs: int = 8) -> Path:
    src_dir = CSRC / "runtime"
    headers = list(src_dir.glob("*.h"))
    srcs = sorted(s for s in src_dir.glob("*.cpp") if s.name != "selftest.cpp")
    out_dir = BUILD / "runtime"
    out_dir.mkdir(parents=True, exist_ok=True)
    flags = ["g++", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-pthread",
             f"-I{src_dir}"] + _py_includes()

    def compile_one(src: Path) -> Path:
        obj = out_dir / (src.name + ".o")
        if _newer(obj, [src] + headers):
            cmd = flags + ["-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), flush=True)
            _run(cmd)
        return obj

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    lib = runtime_lib_path()
    if objs and _newer(lib, objs):
        cmd = ["g++", "-shared", "-fPIC", "-pthread", "-o", str(lib)] + [str(o) for o in objs]
        _run(cmd)
    return lib


def comm_lib_path() -> Path:
    return PKG_DIR / f"_comm{EXT}"


def build_comm(verbose: bool = False) -> Path:
    """``_comm``: native RCCL p2p layer (csrc/comm).  Host code only; the RCCL
    entry points are resolved at run time from the librccl PyTorch mapped, so
    nothing links against a second copy."""
    src_dir = CSRC / "comm"
    srcs = sorted(src_dir.glob("*.cpp"))
    out_dir = BUILD / "comm"
    out_dir.mkdir(parents=True, exist_ok=True)
    lib = comm_lib_path()
    if not _newer(lib, srcs + list(src_dir.glob("*.h"))):
        return lib
    cmd = [HIPCC, "-O2", "-fPIC", "-std=c++17", "-shared", "-Wall", "-pthread", f"-I{ROCM}/include",
           f"-I{src_dir}"] + _py_includes() + [str(s) for s in srcs] + ["-ldl", "-o", str(lib)]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    return lib


def cpu_lib_path() -> Path:
    return PKG_DIR / f"_cpu{EXT}"


def build_cpu(verbose: bool = False) -> Path:
    """``_cpu``: the native CPU execution path (runtime/cpu_executor.py)."""
    src_dir = CSRC / "cpu"
    srcs = sorted(src_dir.glob("*.cpp"))
    lib = cpu_lib_path()
    if not _newer(lib, srcs + list(src_dir.glob("*.h"))):
        return lib
    cmd = ["g++", "-O3", "-fPIC", "-std=c++17", "-shared", "-Wall", "-fopenmp", "-ffp-contract=fast",
           "-fno-math-errno", f"-I{src_dir}"] + _py_includes() + [str(s) for s in srcs] + ["-o", str(lib)]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    return lib


def build_all(verbose: bool = False) -> None:
    build_runtime(verbose)
    build_comm(verbose)
    build_cpu(verbose)
    build_kernels(verbose)


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv)
    print("built", kernel_lib_path(), runtime_lib_path())
