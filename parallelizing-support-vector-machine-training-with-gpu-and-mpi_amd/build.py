"""Native build for svm355: the C++ core, the HIP/gfx950 device library and the CLIs.

Everything is compiled in-tree (``<pkg>/lib`` and ``<pkg>/bin``) so the built objects travel
with the repository snapshot to the GPU box.  Run ``python -m svm355.build`` (or
``__graft_entry__.build()``).  hipcc cross-compiles gfx950 code objects without a GPU.

Targets
  lib/libsvm355_core.so   g++   CPU oracle + data I/O + synthetic data + model files
  lib/libsvm355_hip.so    hipcc CDNA4 kernels (MFMA f64 RBF Gram, fused WSS, SMO step, predict)
                                 and the device-resident SMO driver (hipGraph replay)
  bin/svm_serial          g++   main3.cpp-equivalent CLI
  bin/svm_gpu             hipcc gpu_svm_main3/4-equivalent CLI (--n-limit sweep)
  bin/svm_cascade         hipcc mpi_svm_main2/3-equivalent: one process, a thread per GPU, RCCL
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB = PKG / "lib"
BIN = PKG / "bin"
ARCH = os.environ.get("SVM355_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

CXXFLAGS = ["-std=c++17", "-O3", "-fPIC", "-ffp-contract=off", "-pthread", "-Wall", "-Wextra",
            "-Wno-unused-parameter", f"-I{CSRC / 'include'}", f"-I{CSRC / 'cascade'}"]
HIPFLAGS = ["-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off", f"-I{ROCM / 'include'}",
            f'-DSVM355_RCCL_PATH="{ROCM / "lib" / "librccl.so.1"}"',  # rccl_api.h: the RCCL of these headers
            "-Wall", "-Wno-unused-parameter", "-Wno-unused-result", f"-I{CSRC / 'include'}",
            f"-I{CSRC / 'hip'}", f"-I{CSRC / 'cascade'}"]

# Per-file extra flags.  (Measured and rejected: -fno-honor-nans -mno-amdgpu-ieee on smo.hip was 3%
# faster but changed the f64 division expansion, breaking bit-identity with the CPU oracle.)
HIP_EXTRA: dict = {}

CORE_SRCS = sorted((CSRC / "core").glob("*.cpp")) + sorted((CSRC / "cascade").glob("*.cpp"))
HIP_SRCS = sorted((CSRC / "hip").glob("*.hip"))
HIP_HDRS = (sorted((CSRC / "hip").glob("*.h")) + sorted((CSRC / "include").glob("*.h"))
            + sorted((CSRC / "cascade").glob("*.h")))
CORE_HDRS = (sorted((CSRC / "core").glob("*.h")) + sorted((CSRC / "include").glob("*.h"))
             + sorted((CSRC / "cascade").glob("*.h")))


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(str(c) for c in cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)


def hipcc() -> str:
    exe = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    if not Path(exe).exists():
        raise RuntimeError("hipcc not found (ROCm toolchain required to build the device library)")
    return exe


def build_core(force=False, verbose=False) -> Path:
    LIB.mkdir(exist_ok=True)
    out = LIB / "libsvm355_core.so"
    objdir = LIB / "obj_core"
    objdir.mkdir(exist_ok=True)
    objs, jobs = [], []
    for src in CORE_SRCS:
        obj = objdir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *CORE_HDRS]):
            jobs.append(["g++", *CXXFLAGS, "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _stale(out, objs):
        _run(["g++", "-shared", "-pthread", *objs, "-o", out], verbose)
    return out


def build_hip(force=False, verbose=False) -> Path:
    LIB.mkdir(exist_ok=True)
    out = LIB / "libsvm355_hip.so"
    objdir = LIB / "obj_hip"
    objdir.mkdir(exist_ok=True)
    objs, jobs = [], []
    cc = hipcc()
    for src in HIP_SRCS:
        obj = objdir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *HIP_HDRS, Path(__file__)]):
            jobs.append([cc, *HIPFLAGS, *HIP_EXTRA.get(src.name, []), "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _stale(out, objs):
        _run([cc, "-shared", f"--offload-arch={ARCH}", *objs, f"-L{LIB}", "-lsvm355_core",
              f"-L{ROCM / 'lib'}", "-lrocprofiler-sdk-roctx", "-ldl", "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{ROCM / 'lib'}",
              "-o", out], verbose)
    return out


def build_apps(force=False, verbose=False):
    BIN.mkdir(exist_ok=True)
    rpath = "-Wl,-rpath,$ORIGIN/../lib"
    outs = []
    serial = BIN / "svm_serial"
    src = CSRC / "apps" / "svm_serial.cpp"
    deps = [src, LIB / "libsvm355_core.so", *CORE_HDRS, CSRC / "apps" / "cli_common.h"]
    if force or _stale(serial, deps):
        _run(["g++", *CXXFLAGS, src, f"-L{LIB}", "-lsvm355_core", rpath, "-o", serial], verbose)
    outs.append(serial)
    gpu = BIN / "svm_gpu"
    src = CSRC / "apps" / "svm_gpu.cpp"
    deps = [src, LIB / "libsvm355_core.so", LIB / "libsvm355_hip.so", *HIP_HDRS,
            CSRC / "apps" / "cli_common.h"]
    if force or _stale(gpu, deps):
        _run(["g++", *CXXFLAGS, src, f"-L{LIB}", "-lsvm355_hip", "-lsvm355_core", rpath,
              "-o", gpu], verbose)
    outs.append(gpu)
    # Native cascade (one process, one thread per GPU, RCCL inside libsvm355_hip): C ABI only.
    casc = BIN / "svm_cascade"
    src = CSRC / "apps" / "svm_cascade.cpp"
    deps = [src, LIB / "libsvm355_core.so", LIB / "libsvm355_hip.so", *CORE_HDRS, CSRC / "apps" / "cli_common.h"]
    if force or _stale(casc, deps):
        _run(["g++", *CXXFLAGS, src, f"-L{LIB}", "-lsvm355_hip", "-lsvm355_core", rpath, "-o", casc], verbose)
    outs.append(casc)
    return outs


SANITIZE = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", "-O1", "-g"]


TSANITIZE = ["-fsanitize=thread", "-fno-omit-frame-pointer", "-O1", "-g"]


def host_clang() -> str:
    """The ROCm LLVM's host clang++ (compiler-rt of LLVM 22): its TSan runtime intercepts
    pthread_cond_clockwait, which libstdc++ 11's condition_variable uses and the system gcc 11's libtsan
    does not -- under g++ every wait looks like it returned without the mutex (false 'double lock' and
    data-race reports on everything a condition variable protects)."""
    exe = ROCM / "lib" / "llvm" / "bin" / "clang++"
    if not exe.exists():
        raise RuntimeError(f"{exe} not found (the TSan build needs the ROCm LLVM host compiler)")
    return str(exe)


def _build_host_exe(out_dir: Path, app: str, san, force, verbose, cxx: str = "g++") -> Path:
    out_dir.mkdir(exist_ok=True)
    exe = out_dir / app
    srcs = [*CORE_SRCS, CSRC / "apps" / f"{app}.cpp"]
    if force or _stale(exe, [*srcs, *CORE_HDRS, CSRC / "apps" / "cli_common.h", Path(__file__)]):
        flags = [f for f in CXXFLAGS if f != "-O3"] + san
        tmp = out_dir / f".{app}.{os.getpid()}"  # link aside, then rename: a concurrent run of the
        _run([cxx, *flags, *srcs, "-o", tmp], verbose)  # old file keeps its inode (no ETXTBSY)
        os.replace(tmp, exe)
    return exe


def build_sanitized(force=False, verbose=False) -> Path:
    """Host-only ASan+UBSan build of the CPU core and the serial CLI: one static
    executable ``bin_asan/svm_serial`` (sanitizers on host code only; no GPU code involved)."""
    return _build_host_exe(PKG / "bin_asan", "svm_serial", SANITIZE, force, verbose)


def build_sanitized_threads(force=False, verbose=False):
    """The threaded host code (strict loopback and hostcomm cascades, abort, resume, the decomposition
    oracle's worker team and its distributed thread ranks: apps/svm_threads.cpp) built twice: ASan +
    UBSan (``bin_asan/svm_threads``) and TSan (``bin_tsan/svm_threads``).  Returns both paths."""
    return (_build_host_exe(PKG / "bin_asan", "svm_threads", SANITIZE, force, verbose),
            _build_host_exe(PKG / "bin_tsan", "svm_threads", TSANITIZE, force, verbose, cxx=host_clang()))


def build_all(force=False, verbose=False, hip=True):
    outs = [build_core(force, verbose)]
    if hip:
        outs.append(build_hip(force, verbose))
        outs.extend(build_apps(force, verbose))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-hip", action="store_true", help="build only the CPU core")
    ap.add_argument("--sanitize", action="store_true", help="also build the ASan/UBSan host oracle (bin_asan/)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    for p in build_all(a.force, a.verbose, hip=not a.no_hip):
        print(p)
    if a.sanitize:
        print(build_sanitized(a.force, a.verbose))
        for p in build_sanitized_threads(a.force, a.verbose):
            print(p)


if __name__ == "__main__":
    main()
