"""Build the gfx950 extension in-tree: ``python -m dgi.build``
(``--sanitize``: the ASan+UBSan and TSan builds of the host ring code instead).

Each ``dgi/csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950``
into an object, ``bindings.cpp`` (torch op registration) is compiled against
the installed PyTorch-ROCm headers, and everything is linked into
``dgi/_C.so``.  No hipify step, no cpp_extension JIT cache: the ``.so`` sits
next to the sources so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "..", "build", "dgi_obj")
OUT = os.path.join(HERE, "_C.so")
ARCH = os.environ.get("DGI_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    kernels = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    jobs = []
    objs = []
    for k in kernels:
        src = os.path.join(CSRC, k)
        obj = os.path.join(BUILD, k + ".o")
        objs.append(obj)
        if force or _newer([src] + hdrs, obj):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics", "-c", src, "-o", obj])
    bsrc = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.o")
    objs.append(bobj)
    py_inc = sysconfig.get_paths()["include"]
    if force or _newer([bsrc], bobj):
        jobs.append([HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
                     *[f"-I{p}" for p in inc], f"-I{py_inc}", "-I/opt/rocm/include", "-x", "c++", "-c", bsrc, "-o", bobj])
    # native runtime pieces (C++ only)
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".cc"):
            src = os.path.join(CSRC, f)
            obj = os.path.join(BUILD, f + ".o")
            objs.append(obj)
            if force or _newer([src] + hdrs, obj):
                jobs.append(["g++", *common, f"-I{py_inc}", *[f"-I{p}" for p in inc], "-c", src, "-o", obj])
    workers = int(os.environ.get("MAX_JOBS", "8"))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(workers, 16))) as ex:
        for r in ex.map(_run, jobs):
            if verbose and r.stderr:
                print(r.stderr, file=sys.stderr)
    if force or jobs or not os.path.exists(OUT):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT, f"-L{lib}",
              "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{lib}"])
    return OUT


SHM_SRC = os.path.join(CSRC, "host", "shm_ring.cc")
SHM_OUT = os.path.join(HERE, "_shm" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_shm(force: bool = False) -> str:
    """``dgi/_shm*.so``: the shared-memory control-plane rings (plain C++ /
    pybind11, no ROCm dependency, so the CPU test-suite uses the same code)."""
    if not force and not _newer([SHM_SRC, os.path.join(CSRC, "host", "shm_ring.h")], SHM_OUT):
        return SHM_OUT
    import pybind11
    py_inc = sysconfig.get_paths()["include"]
    _run(["g++", "-O2", "-fPIC", "-shared", "-std=c++17", "-Wall", f"-I{pybind11.get_include()}", f"-I{py_inc}",
          SHM_SRC, "-o", SHM_OUT, "-lrt"])
    return SHM_OUT


STRESS_SRC = os.path.join(CSRC, "host", "shm_ring_stress.cc")
SANITIZERS = {
    # ASan + UBSan: bounds of every ring copy against the mapping, misaligned cursor access
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
    # TSan: the producer / consumer cursor protocol (release / acquire) on one mapping
    "tsan": ["-fsanitize=thread"],
}


def build_sanitized(kind: str, force: bool = False, defines: tuple = (), tag: str = "") -> str:
    """CPU sanitizer build of the native host code: the shared-memory ring
    core (``csrc/host/shm_ring.h``, the one concurrent native component) linked into the
    stress driver ``shm_ring_stress.cc`` with ``SANITIZERS[kind]``; returns the binary's path
    (``build/sanitize/shm_ring_stress_<kind>``).  Host code only: no GPU code is sanitized."""
    flags = SANITIZERS[kind]
    out_dir = os.path.join(HERE, "..", "build", "sanitize")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"shm_ring_stress_{kind}{tag}")
    hdr = os.path.join(CSRC, "host", "shm_ring.h")
    if force or _newer([STRESS_SRC, hdr], out):
        _run(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-Wextra", *flags, *[f"-D{d}" for d in defines],
              STRESS_SRC, "-o", out, "-lrt", "-pthread"])
    return out


if __name__ == "__main__":
    if "--sanitize" in sys.argv:
        for k in SANITIZERS:
            print(build_sanitized(k, force="--force" in sys.argv))
        sys.exit(0)
    print(build_shm(force="--force" in sys.argv))
    p = build(verbose=True, force="--force" in sys.argv)
    print(p)
