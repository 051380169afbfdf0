"""In-tree native build for streamml (no JIT cache, no setuptools magic).

Two shared objects are produced next to this file:

* ``_C.so``  -- the gfx950 HIP kernels + their PyTorch binding.  Each
  ``csrc/kernels/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` into
  its own object (kernels never include torch headers, so they compile in
  seconds); ``csrc/torch_bind.cpp`` is the only torch-dependent translation
  unit and is compiled host-only.
* ``_io.so`` -- host C++17 codecs and runtime pieces (Avro, Confluent framing,
  Kafka wire protocol + in-process broker, HDF5, CSV, synthetic generator),
  pybind11 only, no torch / HIP dependency so they are usable (and testable)
  on CPU-only machines.

Usage: ``python -m streamml._build`` or ``streamml._build.build_all()``.

``python -m streamml._build --checked`` additionally builds ``_C_dbg.so``: the same
kernels compiled with ``-DSML_KERNEL_CHECKS=1`` (device-side ``SML_DCHECK`` bounds
asserts, see ``include/sml_common.h``), loaded instead of ``_C`` when the process
runs with ``SML_KERNEL_CHECKS=1`` (a bounds-checked debug build).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List, Sequence

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "obj")
ARCH = os.environ.get("SML_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
CXX = os.environ.get("CXX", "g++")
JOBS = int(os.environ.get("MAX_JOBS", str(min(8, os.cpu_count() or 4))))


def _newer(src_files: Sequence[str], out: str) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in src_files)


def _headers(*dirs: str) -> List[str]:
    out: List[str] = []
    for d in dirs:
        out += glob.glob(os.path.join(d, "**", "*.h"), recursive=True)
    return out


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _py_include() -> str:
    return sysconfig.get_paths()["include"]


def build_c(verbose: bool = False, force: bool = False, checked: bool = False) -> str:
    """Build ``_C.so`` (HIP kernels + torch binding); ``checked`` builds ``_C_dbg.so``."""
    import torch
    from torch.utils import cpp_extension

    name = "_C_dbg" if checked else "_C"
    obj_dir = os.path.join(BUILD, "checked") if checked else BUILD
    os.makedirs(obj_dir, exist_ok=True)
    inc = os.path.join(CSRC, "include")
    hdrs = _headers(inc)
    kern_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    out = os.path.join(PKG, name + ".so")
    dflags = ["-DSML_KERNEL_CHECKS=1"] if checked else []
    jobs = []
    objs = []
    for src in kern_srcs:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer([src] + hdrs, obj):
            with open(src) as f:
                head = f.read(512)
            # MFMA results straight into VGPRs (no v_accvgpr_read per use), except for
            # kernels that keep large accumulator sets in AGPRs
            vgpr_form = [] if "sml-build: agpr-accumulators" in head else ["-mllvm", "-amdgpu-mfma-vgpr-form"]
            # packed-f32 VALU (v_pk_fma/mul/add_f32) issues slower than the scalar pair it
            # replaces next to MFMAs (MI355X_MICROARCH.md per-instruction costs): kernels that
            # interleave VALU with MFMA opt out of SLP packing
            if "sml-build: no-slp" in head:
                vgpr_form = vgpr_form + ["-fno-slp-vectorize"]
            # SML_HIPCC_EXTRA: extra device-compile flags for A/B builds (e.g. a scheduler strategy)
            extra = os.environ.get("SML_HIPCC_EXTRA", "").split()
            jobs.append([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
                         f"-I{inc}", "-Wno-unused-result", "-munsafe-fp-atomics", *vgpr_form, *dflags, *extra])
    # host runtime pieces that use the HIP runtime API (no device code, no torch)
    for src in sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))):
        obj = os.path.join(BUILD, "rt_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer([src] + hdrs + glob.glob(os.path.join(CSRC, "runtime", "*.h")), obj):
            jobs.append([CXX, "-O2", "-std=c++17", "-fPIC", "-c", src, "-o", obj, f"-I{inc}", f"-I{ROCM}/include",
                         "-D__HIP_PLATFORM_AMD__=1", "-Wall"])
    bind = os.path.join(CSRC, "torch_bind.cpp")
    bind_obj = os.path.join(obj_dir, "torch_bind.o")
    objs.append(bind_obj)
    abi = "1" if torch.compiled_with_cxx11_abi() else "0"
    if force or _newer([bind] + hdrs + glob.glob(os.path.join(CSRC, "runtime", "*.h")), bind_obj):
        cmd = [CXX, "-O2", "-std=c++17", "-fPIC", "-c", bind, "-o", bind_obj, f"-I{inc}", f"-I{_py_include()}",
               f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-DTORCH_EXTENSION_NAME={name}", "-DTORCH_API_INCLUDE_EXTENSION_H",
               "-w"]
        for p in cpp_extension.include_paths():
            cmd.append(f"-I{p}")
        jobs.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=JOBS) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _newer(objs, out):
        libdirs = cpp_extension.library_paths()
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs
        for d in libdirs:
            cmd += [f"-L{d}", f"-Wl,-rpath,{d}"]
        cmd += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
        _run(cmd, verbose)
    return out


def build_io(verbose: bool = False, force: bool = False) -> str:
    """Build ``_io.so`` (host C++ codecs, pybind11 only)."""
    import pybind11

    os.makedirs(BUILD, exist_ok=True)
    inc = os.path.join(CSRC, "include")
    hdrs = _headers(inc, os.path.join(CSRC, "io"))
    srcs = sorted(glob.glob(os.path.join(CSRC, "io", "*.cpp")))
    out = os.path.join(PKG, "_io.so")
    objs, jobs = [], []
    for src in srcs:
        obj = os.path.join(BUILD, "io_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer([src] + hdrs, obj):
            jobs.append([CXX, "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj, f"-I{inc}",
                         f"-I{os.path.join(CSRC, 'io')}", f"-I{pybind11.get_include()}", f"-I{_py_include()}",
                         "-Wall", "-Wno-unused-function"] + _san_flags())
    with cf.ThreadPoolExecutor(max_workers=JOBS) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if not objs:
        return ""
    if force or jobs or _newer(objs, out):
        _run([CXX, "-shared", "-fPIC", "-o", out] + objs + ["-lpthread"] + _san_flags(), verbose)
    return out


def _san_flags() -> List[str]:
    """``SML_SANITIZE=address,undefined`` builds the host codecs instrumented."""
    s = os.environ.get("SML_SANITIZE", "")
    return [f"-fsanitize={s}", "-fno-omit-frame-pointer", "-g"] if s else []


def build_all(verbose: bool = False, force: bool = False, checked: bool = False) -> None:
    build_io(verbose=verbose, force=force)
    build_c(verbose=verbose, force=force)
    if checked:
        build_c(verbose=verbose, force=force, checked=True)


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv, force="-f" in sys.argv, checked="--checked" in sys.argv)
    print("built:", [p for p in (os.path.join(PKG, n) for n in ("_C.so", "_C_dbg.so", "_io.so")) if os.path.exists(p)])
