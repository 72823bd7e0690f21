"""In-tree native build for the MI355X framework.

Two shared objects are produced next to this file:

* ``_C.so``  -- the HIP/CDNA4 kernels (``csrc/kernels/*.hip``) plus the torch op
  registrations (``csrc/bindings.cpp``).  Compiled with ``hipcc --offload-arch=gfx950``;
  no hipify, no CUDA shims.  Loaded with ``torch.ops.load_library`` so every op is a
  ``torch.ops.tsamd.*`` call that can be captured into a hipGraph.  ``_C_debug.so`` is the
  same library with the bounds checks of ``csrc/kernels/dcheck.h`` compiled in
  (TSAMD_KERNEL_DEBUG=1 loads it).
* ``_rt.so`` -- the host-side native runtime (``csrc/runtime/*.cpp``): shared-memory
  SPSC ring buffer (replaces Flink-AI-Extended's JVM<->Python mmap queue),
  TF tensor-bundle checkpoint reader/writer with crc32c, record codec.
  Plain C ABI, loaded with ctypes, no GPU and no torch dependency, so CPU tests use it.

The build is incremental (mtime based) and parallel; ``python -m
textsummarization_on_flink_amd._build`` rebuilds.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _torch_flags():
    import torch
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    libs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [
        f"-I{sysconfig.get_paths()['include']}",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_C",
    ]
    ldflags = [f"-L{p}" for p in libs] + [f"-Wl,-rpath,{p}" for p in libs] + [
        "-lc10", "-ltorch", "-ltorch_cpu", "-lc10_hip", "-ltorch_hip", "-lamdhip64",
    ]
    return cflags, ldflags


def _newer(src_list, dst):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, flush=True)


def _headers(d):
    out = []
    for root, _, files in os.walk(d):
        out += [os.path.join(root, f) for f in files if f.endswith((".h", ".hpp", ".cuh"))]
    return out


def build_kernels(verbose=False, jobs=8, debug=False):
    """Compile csrc/kernels/*.hip + csrc/bindings.cpp into textsummarization_on_flink_amd/_C.so.

    ``debug``: the bounds-checked variant ``_C_debug.so`` (-DTSAMD_DEBUG, csrc/kernels/dcheck.h;
    relocatable device code so every kernel shares the one check record in debug.hip),
    loaded instead of ``_C.so`` when TSAMD_KERNEL_DEBUG=1."""
    bdir = BUILD + ("_debug" if debug else "")
    os.makedirs(bdir, exist_ok=True)
    kdir = os.path.join(CSRC, "kernels")
    hips = sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".hip"))
    hdrs = _headers(kdir)
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast",
              "-Wno-unused-result", "-munsafe-fp-atomics", f"-I{kdir}"]
    if debug:
        common += ["-DTSAMD_DEBUG", "-fgpu-rdc"]
    objs, jobsl = [], []
    for src in hips:
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer([src] + hdrs, obj):
            jobsl.append([HIPCC, *common, "-c", src, "-o", obj])
    tflags, tld = _torch_flags()
    for host in ("bindings.cpp", "blt_gemm.cpp"):  # torch op registrations (blt_gemm: hipBLASLt calls)
        bsrc = os.path.join(CSRC, host)
        bobj = os.path.join(bdir, host.replace(".cpp", ".o"))
        objs.append(bobj)
        if _newer([bsrc] + hdrs, bobj):
            jobsl.append([HIPCC, "-O2", "-std=c++17", "-fPIC", f"-I{kdir}", *tflags, "-c", bsrc, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobsl))
    so = os.path.join(PKG_DIR, "_C_debug.so" if debug else "_C.so")
    if jobsl or not os.path.exists(so):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + (["-fgpu-rdc"] if debug else [])
        # -lhipblaslt resolves to torch's own copy (its lib dir comes first in tld): one instance
        _run([*link, *objs, "-o", so, *tld, "-lhipblaslt"], verbose)
    return so


def build_runtime(verbose=False):
    """Compile csrc/runtime/*.cpp into textsummarization_on_flink_amd/_rt.so (host only)."""
    os.makedirs(BUILD, exist_ok=True)
    rdir = os.path.join(CSRC, "runtime")
    srcs = sorted(os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".cpp"))
    so = os.path.join(PKG_DIR, "_rt.so")
    if not srcs:
        return None
    if _newer(srcs + _headers(rdir), so):
        _run([CXX, "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", f"-I{rdir}", *srcs,
              "-o", so, "-lrt"], verbose)
    return so


def build(verbose=False, debug=True):
    """Host runtime, release kernel library and (``debug``) its bounds-checked variant."""
    rt = build_runtime(verbose)
    c = build_kernels(verbose)
    if debug:
        build_kernels(verbose, debug=True)
    return rt, c


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, debug="--no-debug" not in sys.argv))
