"""Native build for tenzing_amd: generates a ninja file and builds, in-tree,

* ``tenzing_amd/_tz<EXT_SUFFIX>``  – the Python extension (C++17 core + HIP runtime + gfx950
  kernels + RCCL transport + pybind11 bindings),
* ``tenzing_amd/bin/tz-search``    – the standalone search CLI (no Python needed),
* ``tenzing_amd/bin/tz-unit``      – native unit tests of the core.

Host C++ is compiled with amdclang++, device code (``*.hip``) with ``hipcc --offload-arch=gfx950``
(cross-compiles without a GPU). Reference build: CMakeLists.txt + src/CMakeLists.txt (object
library + static lib + doctest binaries); here a single ninja graph.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("TZ_OFFLOAD_ARCH", "gfx950")

CORE = ["json", "numeric", "ops", "graph", "state", "serdes", "ctrl", "ctrl_mpi", "benchmark", "solve", "health"]
HIP_HOST = ["hip_runtime", "rccl_comm", "comm_ops", "rocsparse_spmv"]
WORKLOADS = ["halo", "halo_ipc", "halo_relay", "halo_hostsplit", "halo_graph", "halo_stencil", "spmv", "workloads_common", "link_matrix", "fused_ops"]
KERNELS = ["halo_kernels", "spmv_kernels", "stencil_kernels"]


def _git_hash() -> str:
    try:
        return subprocess.check_output(["git", "-C", str(ROOT), "rev-parse", "--short", "HEAD"],
                                       stderr=subprocess.DEVNULL, text=True).strip() or "unknown"
    except Exception:
        return "unknown"


def ext_path() -> Path:
    return PKG / ("_tz" + sysconfig.get_config_var("EXT_SUFFIX"))


def _ninja_file(debug: bool) -> str:
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    opt = "-O0 -g" if debug else "-O3 -g1"
    common = (f"-std=c++17 -fPIC {opt} -Wall -Wextra -Wno-unused-parameter "
              f"-DTZ_GIT_HASH=\\\"{_git_hash()}\\\" -I{CSRC}")
    hipdefs = f"-D__HIP_PLATFORM_AMD__ -I{ROCM}/include"
    cxx = f"{ROCM}/lib/llvm/bin/clang++"
    hipcc = f"{ROCM}/bin/hipcc"
    lines = [
        "ninja_required_version = 1.5",
        f"cxx = {cxx}",
        f"hipcc = {hipcc}",
        f"cflags = {common}",
        f"hipflags = {common} {hipdefs}",
        f"devflags = {common} --offload-arch={ARCH} -munsafe-fp-atomics -ffp-contract=fast",
        f"pyflags = -I{pybind11.get_include()} -I{py_inc}",
        f"ldflags = -L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lamdhip64 -lrccl -lrocsparse -lrocprofiler-sdk-roctx -lpthread -ldl",
        "rule cxx",
        "  command = $cxx $cflags $extra -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $out",
        "rule hipdev",
        "  command = $hipcc $devflags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $out",
        "rule link_so",
        "  command = $hipcc -shared -o $out $in $ldflags",
        "  description = LINK $out",
        "rule link_exe",
        "  command = $hipcc -o $out $in $ldflags",
        "  description = LINK $out",
        "rule ar",
        "  command = rm -f $out && ar rcs $out $in",
        "  description = AR $out",
    ]
    objs_core, objs_rt = [], []
    for n in CORE:
        o = f"{BUILD}/core/{n}.o"
        lines.append(f"build {o}: cxx {CSRC}/core/{n}.cpp")
        objs_core.append(o)
    for n in HIP_HOST:
        o = f"{BUILD}/hip/{n}.o"
        lines.append(f"build {o}: cxx {CSRC}/hip/{n}.cpp")
        lines.append(f"  extra = {hipdefs}")
        objs_rt.append(o)
    for n in WORKLOADS:
        o = f"{BUILD}/workloads/{n}.o"
        lines.append(f"build {o}: cxx {CSRC}/workloads/{n}.cpp")
        lines.append(f"  extra = {hipdefs}")
        objs_rt.append(o)
    for n in KERNELS:
        o = f"{BUILD}/kernels/{n}.o"
        lines.append(f"build {o}: hipdev {CSRC}/kernels/{n}.hip")
        objs_rt.append(o)
    bind = f"{BUILD}/bind/module.o"
    lines.append(f"build {bind}: cxx {CSRC}/bind/module.cpp")
    lines.append(f"  extra = {hipdefs} $pyflags -fvisibility=hidden")
    allobjs = " ".join(objs_core + objs_rt)
    lines.append(f"build {ext_path()}: link_so {allobjs} {bind}")
    for tool in ("tz_search", "tz_unit"):
        o = f"{BUILD}/tools/{tool}.o"
        lines.append(f"build {o}: cxx {CSRC}/tools/{tool}.cpp")
        lines.append(f"  extra = {hipdefs}")
        exe = PKG / "bin" / tool.replace("_", "-")
        lines.append(f"build {exe}: link_exe {allobjs} {o}")
    # the engine as a C++ library (reference: the static `tenzing` library that drivers link),
    # plus a user-side example that defines its own kernel op against it
    lib = BUILD / "libtenzing_amd.a"
    lines.append(f"build {lib}: ar {allobjs}")
    # and a multi-rank program with RCCL comm ops in its graph
    exes = []
    for src, exe_name in (("custom_kernel_op", "tz-example-custom-op"),
                          ("ring_overlap", "tz-example-ring")):
        ex_obj = f"{BUILD}/examples/{src}.o"
        ex_exe = PKG / "bin" / exe_name
        lines.append(f"build {ex_obj}: hipdev {ROOT / 'examples' / 'cpp' / (src + '.hip')}")
        lines.append(f"build {ex_exe}: link_exe {ex_obj} {lib}")
        exes.append(str(ex_exe))
    lines.append(f"default {ext_path()} {PKG / 'bin' / 'tz-search'} {PKG / 'bin' / 'tz-unit'} "
                 f"{lib} {' '.join(exes)}")
    return "\n".join(lines) + "\n"


SANITIZERS = {
    # host-only: the core (graph, synchronizer, solvers, control plane) and its unit suite. GPU
    # code is not instrumented (no GPU sanitizers on this pool)
    "asan": "-fsanitize=address,undefined -fno-sanitize-recover=undefined",
    "tsan": "-fsanitize=thread",
}


def _sanitizer_ninja(kind: str) -> str:
    flags = SANITIZERS[kind]
    out = BUILD / kind
    cxx = f"{ROCM}/lib/llvm/bin/clang++"
    common = (f"-std=c++17 -O1 -g -fno-omit-frame-pointer {flags} -Wall -Wno-unused-parameter "
              f"-DTZ_GIT_HASH=\\\"{_git_hash()}\\\" -I{CSRC}")
    lines = [
        "ninja_required_version = 1.5",
        f"cxx = {cxx}",
        f"cflags = {common}",
        "rule cxx",
        "  command = $cxx $cflags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX[" + kind + "] $out",
        "rule link",
        f"  command = $cxx {flags} -o $out $in -lpthread -ldl",
        "  description = LINK $out",
    ]
    objs = []
    for n in CORE:
        o = f"{out}/core/{n}.o"
        lines.append(f"build {o}: cxx {CSRC}/core/{n}.cpp")
        objs.append(o)
    o = f"{out}/tools/tz_unit.o"
    lines.append(f"build {o}: cxx {CSRC}/tools/tz_unit.cpp")
    objs.append(o)
    lines.append(f"build {out}/tz-unit: link {' '.join(objs)}")
    lines.append(f"default {out}/tz-unit")
    return "\n".join(lines) + "\n"


def build_sanitized(kind: str, jobs: int | None = None) -> Path:
    """Host-only sanitizer build of the native unit suite (``asan``: AddressSanitizer +
    UndefinedBehaviorSanitizer, ``tsan``: ThreadSanitizer). Returns the tz-unit path."""
    if kind not in SANITIZERS:
        raise ValueError(f"sanitizer must be one of {sorted(SANITIZERS)}")
    out = BUILD / kind
    out.mkdir(parents=True, exist_ok=True)
    nf = out / "build.ninja"
    content = _sanitizer_ninja(kind)
    if not nf.exists() or nf.read_text() != content:
        nf.write_text(content)
    ninja = shutil.which("ninja") or "ninja"
    r = subprocess.run([ninja, "-C", str(out), f"-j{jobs or min(16, os.cpu_count() or 4)}"],
                       text=True, capture_output=True)
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError(f"tenzing_amd {kind} build failed")
    return out / "tz-unit"


def build(jobs: int | None = None, debug: bool = False, verbose: bool = False) -> Path:
    """Compile everything (idempotent, incremental). Returns the extension path."""
    BUILD.mkdir(parents=True, exist_ok=True)
    (PKG / "bin").mkdir(exist_ok=True)
    nf = BUILD / "build.ninja"
    content = _ninja_file(debug)
    if not nf.exists() or nf.read_text() != content:
        nf.write_text(content)
    ninja = shutil.which("ninja") or "ninja"
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = [ninja, "-C", str(BUILD), f"-j{jobs}"]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, text=True, capture_output=not verbose)
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError("tenzing_amd native build failed")
    return ext_path()


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--sanitize", choices=sorted(SANITIZERS),
                    help="build the host-only unit suite under a sanitizer instead")
    a = ap.parse_args()
    print(build_sanitized(a.sanitize, a.j) if a.sanitize else build(a.j, a.debug, a.verbose))
