"""In-tree native build for metisfl_amd (gfx950 only).

Two shared objects are produced next to the Python package:

* ``metisfl_amd/_engine*.so`` -- the federation controller engine
  (scheduler / selector / scalers / aggregators / model store / runtime
  metadata / RNS-CKKS), C++17 + OpenMP + pybind11, plus the device
  aggregation backend (engine/device_agg*, HIP runtime + gfx950 kernels)
  that takes over FedAvg / FedStride / FedRec / PWA when a GPU is visible.  It is the native
  equivalent of the reference's Bazel-built ``controller.so`` and ``fhe.so``
  (reference: setup.py:21-45, metisfl/controller/pybind/controller_pybind.cc,
  metisfl/encryption/pybind/ckks_pybind.cc).
* ``metisfl_amd/_ops*.so`` -- the hand-written HIP/CDNA4 kernels (``*.hip``,
  compiled by hipcc for ``--offload-arch=gfx950``) plus the thin torch binding
  that launches them on the current HIP stream.

The build is driven by a generated ``build.ninja`` (ninja is in the image), so
re-runs only recompile what changed.  ``python -m metisfl_amd.csrc.build``.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
BUILD_DIR = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("METISFL_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> list[str]:
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _py_embed_ldflags() -> str:
    """Link flags for an executable embedding this interpreter (controller_main)."""
    libdir = sysconfig.get_config_var("LIBDIR") or ""
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    extra = sysconfig.get_config_var("LIBS") or ""
    return f"-L{libdir} -Wl,-rpath,{libdir} -lpython{ver} {extra} -lm"


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = [os.path.join(os.path.dirname(torch.__file__), "include"),
           os.path.join(os.path.dirname(torch.__file__), "include", "torch", "csrc", "api", "include")]
    lib = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _rel(p: str) -> str:
    return os.path.relpath(p, BUILD_DIR)


def write_ninja() -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    suffix = _ext_suffix()
    pyinc = " ".join(f"-I{p}" for p in _py_includes())
    tinc, tlib, abi = _torch_paths()
    tincs = " ".join(f"-I{p}" for p in tinc)
    csrc = HERE

    engine_srcs = sorted(glob.glob(os.path.join(csrc, "common", "*.cc"))
                         + glob.glob(os.path.join(csrc, "engine", "*.cc"))
                         + glob.glob(os.path.join(csrc, "he", "*.cc"))
                         + [os.path.join(csrc, "bindings", "engine_pybind.cc")])
    engine_hip = sorted(glob.glob(os.path.join(csrc, "engine", "*.hip")))
    hip_srcs = sorted(glob.glob(os.path.join(csrc, "kernels", "*.hip")))
    ops_bind = sorted(glob.glob(os.path.join(csrc, "bindings", "*.cpp")))

    lines = [
        "ninja_required_version = 1.3",
        f"cxx = g++",
        f"hipcc = {ROCM}/bin/hipcc",
        f"engine_cflags = -O3 -fPIC -std=c++17 -fopenmp -Wall -Wno-sign-compare -Wno-unused-result -fvisibility=hidden "
        f"-D__HIP_PLATFORM_AMD__ -I{csrc} -I{ROCM}/include {pyinc}",
        f"engine_ldflags = -L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lamdhip64",
        f"hip_cflags = --offload-arch={ARCH} -O3 -fPIC -std=c++17 -munsafe-fp-atomics -I{csrc} "
        f"-Wno-unused-result",
        f"bind_cflags = -O2 -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__ -DUSE_ROCM "
        f"-DTORCH_EXTENSION_NAME=_ops -DTORCH_API_INCLUDE_EXTENSION_H -D_GLIBCXX_USE_CXX11_ABI={abi} "
        f"-I{csrc} {tincs} -I{ROCM}/include {pyinc} -Wno-deprecated-declarations",
        f"tool_cflags = {pyinc} -DMETISFL_AMD_DEFAULT_ROOT=\\\"{ROOT}\\\"",
        f"tool_ldflags = {_py_embed_ldflags()}",
        f"ops_ldflags = -shared -fPIC --offload-arch={ARCH} -L{tlib} -Wl,-rpath,{tlib} "
        f"-lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lamdhip64",
        "",
        "rule cxx_engine",
        "  command = $cxx -MMD -MF $out.d $engine_cflags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link_engine",
        "  command = $cxx -shared -fopenmp $in -o $out $engine_ldflags",
        "  description = LINK $out",
        "rule hipcc",
        "  command = $hipcc -MMD -MF $out.d $hip_cflags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule cxx_bind",
        "  command = $cxx -MMD -MF $out.d $bind_cflags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX(torch) $in",
        "rule cxx_tool",
        "  command = $cxx -MMD -MF $out.d -O2 -std=c++17 -fvisibility=hidden $tool_cflags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX(tool) $in",
        "rule link_tool",
        "  command = $cxx $in -o $out $tool_ldflags",
        "  description = LINK $out",
        "rule link_ops",
        "  command = $hipcc $in -o $out $ops_ldflags",
        "  description = LINK $out",
        "",
    ]
    eng_objs = []
    for s in engine_srcs:
        o = os.path.join(BUILD_DIR, "engine", os.path.relpath(s, csrc).replace("/", "__") + ".o")
        eng_objs.append(o)
        lines.append(f"build {_rel(o)}: cxx_engine {_rel(s)}")
    for s in engine_hip:  # the controller's device-aggregation kernels
        o = os.path.join(BUILD_DIR, "engine", os.path.basename(s) + ".o")
        eng_objs.append(o)
        lines.append(f"build {_rel(o)}: hipcc {_rel(s)}")
    eng_so = os.path.join(PKG, "_engine" + suffix)
    lines.append(f"build {_rel(eng_so)}: link_engine " + " ".join(_rel(o) for o in eng_objs))

    ops_objs = []
    for s in hip_srcs:
        # conv32.hip is built once per product variant (exact fp32 / bf16x3;
        # namespaces mfl::c32x / mfl::c32s, kernels/conv32.h)
        variants = [("", "-DMFL_C32_BF16X3=0"), (".bf16x3", "-DMFL_C32_BF16X3=1" + os.environ.get("MFL_C32_EXTRA", ""))] \
            if os.path.basename(s) == "conv32.hip" else [("", None)]
        for tag, flag in variants:
            o = os.path.join(BUILD_DIR, "hip", os.path.basename(s) + tag + ".o")
            ops_objs.append(o)
            lines.append(f"build {_rel(o)}: hipcc {_rel(s)}")
            if flag:
                lines.append(f"  hip_cflags = $hip_cflags {flag}")
    for s in ops_bind:
        o = os.path.join(BUILD_DIR, "bind", os.path.basename(s) + ".o")
        ops_objs.append(o)
        lines.append(f"build {_rel(o)}: cxx_bind {_rel(s)}")
    ops_so = os.path.join(PKG, "_ops" + suffix)
    lines.append(f"build {_rel(ops_so)}: link_ops " + " ".join(_rel(o) for o in ops_objs))
    # standalone controller executable (reference controller_main.cc)
    tool_src = os.path.join(csrc, "tools", "controller_main.cc")
    tool_obj = os.path.join(BUILD_DIR, "tools", "controller_main.o")
    lines.append(f"build {_rel(tool_obj)}: cxx_tool {_rel(tool_src)}")
    lines.append(f"build metisfl_controller: link_tool {_rel(tool_obj)}")
    lines.append("")
    path = os.path.join(BUILD_DIR, "build.ninja")
    with open(path, "w") as f:
        f.write("\n".join(lines))
    return path


def build(targets: list[str] | None = None, jobs: int | None = None, verbose: bool = False) -> None:
    write_ninja()
    jobs = jobs or min(8, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    cmd = ["ninja", "-C", BUILD_DIR, f"-j{jobs}"]
    if verbose:
        cmd.append("-v")
    suffix = _ext_suffix()
    if targets:
        cmd += [_rel(os.path.join(PKG, t + suffix)) for t in targets]
    subprocess.run(cmd, check=True)


if __name__ == "__main__":
    tg = [a for a in sys.argv[1:] if not a.startswith("-")]
    build(tg or None, verbose="-v" in sys.argv)
