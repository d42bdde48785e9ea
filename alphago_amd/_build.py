"""In-tree native build for alphago_amd.

Shared objects are produced next to the package sources (so they travel to
the GPU box with the repository snapshot):

* ``alphago_amd/_engine*.so`` — C++17 rules engine, featurizer and batched MCTS
  (pybind11, built with g++).
* ``alphago_amd/_hip_kernels.so`` — the production hand-written CDNA4 HIP
  kernels for gfx950 (compiled directly with hipcc; no hipify, no torch JIT
  cache), registered as ``torch.ops.alphago_amd.*`` through TORCH_LIBRARY and
  loaded with ``torch.ops.load_library``.  Only production kernels: the
  kernel-lab tilings are not compiled into it.
* ``alphago_amd/_hip_kernels_debug.so`` — the same library with -DAGK_DEBUG:
  device bounds checks in the conv kernels, every op synchronises and raises
  on a recorded violation (``ALPHAGO_AMD_KERNELS=debug`` selects it).
* ``alphago_amd/_hip_kernels_lab.so`` — the kernel lab (forward-conv tiling
  experiments, wgrad / fp8 variants, cycle stamps) as
  ``torch.ops.alphago_amd_lab.*``, loadable next to the production library.

Usage: ``python -m alphago_amd._build [engine|hip|debug|lab|all] [--force]``.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def engine_path() -> str:
    return os.path.join(PKG, "_engine" + _ext_suffix())


FLAVORS = ("prod", "debug", "lab")


def hip_path(flavor: str = "prod") -> str:
    return os.path.join(PKG, {"prod": "_hip_kernels.so", "debug": "_hip_kernels_debug.so",
                              "lab": "_hip_kernels_lab.so"}[flavor])


def _hip_sources(flavor: str):
    kd = os.path.join(CSRC, "kernels")
    if flavor == "lab":
        return [os.path.join(kd, f) for f in LAB_SOURCES + ("conv.hip", "conv_ws.hip", "conv_fp8.hip", "conv_wgrad_fp8.hip", "ops_lab.cpp")]
    srcs = sorted(glob.glob(os.path.join(kd, "*.hip")) + glob.glob(os.path.join(kd, "*.cpp")))
    return [f for f in srcs if os.path.basename(f) not in LAB_SOURCES + ("ops_lab.cpp",)]


# kernel-lab sources: measured and recorded slower or dead, kept buildable for experiments and out of
# the production library -- forward-tile variants and the compact-halo kernels, wgrad variants 1-4 and
# 6-8, the one-kernel-row wgrad (variant 5, profiles/r3_wgrad_row.md), Winograd (r3_winograd.md), the
# GPU ladder reader (16x slower than the host reader, r2_gpu_ladders.md), hardware probes
LAB_SOURCES = ("conv_fwd_variants.hip", "conv_lab.hip", "conv_wgrad_row.hip", "winograd.hip", "ladder.hip",
               "lab_probes.hip")


def _digest(paths, extra: str = "") -> str:
    h = hashlib.sha1(extra.encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


def _up_to_date(target: str, digest: str) -> bool:
    stamp = target + ".sha1"
    if not (os.path.exists(target) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == digest


def _write_stamp(target: str, digest: str) -> None:
    with open(target + ".sha1", "w") as f:
        f.write(digest)


def _run(cmd, verbose=False):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed (%d):\n%s\n%s" % (r.returncode, " ".join(cmd), r.stdout))
    return r.stdout


def build_engine(force: bool = False, verbose: bool = False) -> str:
    import pybind11

    srcs = sorted(glob.glob(os.path.join(CSRC, "engine", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "engine", "*.h")))
    out = engine_path()
    flags = ["-O3", "-std=c++17", "-fPIC", "-mpopcnt", "-fvisibility=hidden", "-Wall", "-Wno-sign-compare"]
    digest = _digest(srcs + hdrs, " ".join(flags))
    if not force and _up_to_date(out, digest):
        return out
    os.makedirs(BUILD, exist_ok=True)
    incs = ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-I" + os.path.join(CSRC, "engine")]

    def compile_one(src):
        obj = os.path.join(BUILD, "engine_" + os.path.basename(src) + ".o")
        _run(["g++", *flags, *incs, "-c", src, "-o", obj], verbose)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = out + ".tmp"
    _run(["g++", "-shared", "-o", tmp, *objs, "-lpthread"], verbose)
    os.replace(tmp, out)
    _write_stamp(out, digest)
    return out


def build_selftest(sanitize: str = "", force: bool = False, verbose: bool = False) -> str:
    """Standalone engine self-test (csrc/tools/engine_selftest.cpp), optionally
    with host sanitizers: ``address,undefined`` or ``thread``."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "engine", "*.cpp")))
    srcs = [s for s in srcs if not s.endswith(("bindings.cpp", "lzf.cpp", "lockstep.cpp"))]  # pybind11-only files
    hdrs = sorted(glob.glob(os.path.join(CSRC, "engine", "*.h")))
    main = os.path.join(CSRC, "tools", "engine_selftest.cpp")
    tag = sanitize.replace(",", "_") if sanitize else "plain"
    out = os.path.join(BUILD, "engine_selftest_" + tag)
    flags = ["-std=c++17", "-g", "-mpopcnt", "-DAG_NO_PYBIND=1", "-Wall", "-Wno-sign-compare"]
    flags += (["-O1", "-fno-omit-frame-pointer", "-fsanitize=" + sanitize] if sanitize else ["-O2"])
    if sanitize and "undefined" in sanitize:
        flags.append("-fno-sanitize-recover=undefined")
    digest = _digest(srcs + hdrs + [main], " ".join(flags))
    if not force and _up_to_date(out, digest):
        return out
    os.makedirs(BUILD, exist_ok=True)
    _run(["g++", *flags, "-I" + os.path.join(CSRC, "engine"), *srcs, main, "-o", out, "-lpthread"], verbose)
    _write_stamp(out, digest)
    return out


def _torch_paths():
    import torch
    from torch.utils import cpp_extension

    incs = cpp_extension.include_paths(device_type="cuda")
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = "1" if torch._C._GLIBCXX_USE_CXX11_ABI else "0"
    return incs, libdir, abi


def build_hip(force: bool = False, verbose: bool = False, flavor: str = "prod") -> str:
    srcs = _hip_sources(flavor)
    # kernels include engine/ladder_bb.h (shared host/device ladder reader)
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")) + [os.path.join(CSRC, "engine", "ladder_bb.h")])
    out = hip_path(flavor)
    incs, libdir, abi = _torch_paths()
    common = [
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-D_GLIBCXX_USE_CXX11_ABI=" + abi,
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DTORCH_EXTENSION_NAME=_hip_kernels",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
    ] + {"prod": [], "debug": ["-DAGK_DEBUG=1"],
         "lab": ["-DAGK_KERNEL_LAB=1", "-Dagk=agk_lab", "-Dagk_ops=agk_lab_ops"]}[flavor]
    hip_flags = ["--offload-arch=" + ARCH, "-fgpu-rdc" if False else "-fno-gpu-rdc", "-munsafe-fp-atomics"]
    digest = _digest(srcs + hdrs, " ".join(common + hip_flags))
    if not force and _up_to_date(out, digest):
        return out
    os.makedirs(BUILD, exist_ok=True)
    inc_flags = ["-I" + p for p in incs] + ["-I" + os.path.join(CSRC, "kernels"), "-I" + sysconfig.get_paths()["include"]]
    hipcc = os.path.join(ROCM, "bin", "hipcc")

    def compile_one(src):
        obj = os.path.join(BUILD, "hip_%s_%s.o" % (flavor, os.path.basename(src)))
        # every translation unit is compiled for gfx950 only (the op registration
        # file includes the kernel headers)
        cmd = [hipcc, "-x", "hip", *common, *hip_flags, *inc_flags, "-c", src, "-o", obj]
        _run(cmd, verbose)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(srcs)))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = out + ".tmp"
    _run(
        [
            hipcc,
            "-shared",
            "--offload-arch=" + ARCH,
            "-o",
            tmp,
            *objs,
            "-L" + libdir,
            "-Wl,-rpath," + libdir,
            "-lc10",
            "-lc10_hip",
            "-ltorch",
            "-ltorch_cpu",
            "-ltorch_hip",
            "-lamdhip64",
        ],
        verbose,
    )
    os.replace(tmp, out)
    _write_stamp(out, digest)
    return out


def build_all(force: bool = False, verbose: bool = False, flavors=FLAVORS):
    """Engine + every HIP library flavor; returns (engine path, production HIP path)."""
    eng = build_engine(force, verbose)
    paths = [build_hip(force, verbose, f) for f in flavors]
    return eng, paths[0]


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "all"
    force = "--force" in sys.argv
    verbose = "-v" in sys.argv
    if what in ("engine", "all"):
        print("engine:", build_engine(force, verbose))
    if what in ("hip", "all"):
        print("hip:", build_hip(force, verbose))
    if what in ("debug", "all"):
        print("hip debug:", build_hip(force, verbose, "debug"))
    if what in ("lab", "all"):
        print("hip lab:", build_hip(force, verbose, "lab"))
    if what == "selftest":
        san = sys.argv[sys.argv.index("--sanitize") + 1] if "--sanitize" in sys.argv else ""
        print("selftest:", build_selftest(san, force, verbose))
