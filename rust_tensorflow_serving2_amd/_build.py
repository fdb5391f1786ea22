"""In-tree build of the two native extensions.

* ``_C``   — CPU data plane (C++17, g++): wire codec, crc32c, TensorBundle
             tables, HTTP/2 gRPC front end, dynamic batcher.  No torch dep.
* ``_hip`` — gfx950 HIP kernels (hipcc --offload-arch=gfx950) + torch op
             bindings (conv/GEMM MFMA kernels, attention, norms, pooling, ...).

Both are compiled straight into the package directory so the ``.so`` files
travel with the repo snapshot to the GPU box (no JIT cache under ~/.cache).
Incremental: an object is rebuilt only when its source, a header it may
include, or the flag set changed.  ``python -m rust_tensorflow_serving2_amd._build``
builds everything.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
KDIR = os.path.join(PKG, "kernels")
BUILD = os.path.join(PKG, "build")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _digest(paths, flags) -> str:
    h = hashlib.sha1(" ".join(flags).encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _local_includes(src, headers):
    """Headers of ``headers`` that ``src`` includes (transitively, via #include "...")."""
    by_name = {os.path.basename(h): h for h in headers}
    seen, todo = set(), [src]
    while todo:
        with open(todo.pop()) as f:
            for line in f:
                line = line.strip()
                if line.startswith("#include \""):
                    h = by_name.get(line.split('"')[1])
                    if h and h not in seen:
                        seen.add(h)
                        todo.append(h)
    return sorted(seen)


def _compile_all(compiler, sources, headers, flags, tag, jobs):
    os.makedirs(BUILD, exist_ok=True)
    objs, todo = [], []
    for src in sources:
        base = os.path.splitext(os.path.basename(src))[0]
        obj = os.path.join(BUILD, f"{tag}_{base}.o")
        stamp = obj + ".sha1"
        d = _digest([src] + _local_includes(src, headers), flags + [compiler])
        if not (os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == d):
            todo.append((src, obj, stamp, d))
        objs.append(obj)

    def work(item):
        src, obj, stamp, d = item
        _run([compiler] + flags + ["-c", src, "-o", obj])
        with open(stamp, "w") as f:
            f.write(d)
        return src

    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for _ in ex.map(work, todo):
                pass
    return objs, bool(todo)


def _py_includes():
    import pybind11
    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _nghttp2_lib() -> str:
    """libnghttp2 runtime (no -dev package in the image: link the .so.N directly)."""
    for d in ("/usr/lib/x86_64-linux-gnu", "/usr/lib64", "/usr/lib", "/lib/x86_64-linux-gnu"):
        for name in ("libnghttp2.so", "libnghttp2.so.14"):
            p = os.path.join(d, name)
            if os.path.exists(p):
                return p
    raise RuntimeError("libnghttp2 not found")


def build_cpu(jobs: int = 8, verbose: bool = False) -> str:
    out = os.path.join(PKG, "_C" + EXT)
    sources = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    flags = ["-O3", "-std=c++17", "-fPIC", "-msse4.2", "-fvisibility=hidden",
             "-Wall", "-Wno-unused-function", "-pthread"] + _py_includes()
    objs, changed = _compile_all(os.environ.get("CXX", "g++"), sources, headers, flags, "cpu", jobs)
    if changed or not os.path.exists(out):
        _run([os.environ.get("CXX", "g++"), "-shared", "-pthread", "-o", out + ".tmp"] + objs +
             [_nghttp2_lib(), "-ldl"])
        os.replace(out + ".tmp", out)
    if verbose:
        print("built", out)
    return out


def _torch_flags():
    import torch
    import torch.utils.cpp_extension as ce
    inc = [f"-I{p}" for p in ce.include_paths(device_type="cuda")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = ["-DTORCH_EXTENSION_NAME=_hip", "-DTORCH_API_INCLUDE_EXTENSION_H",
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
            "-DUSE_ROCM=1", "-DHIPBLAS_V2"]
    libs = [f"-L{p}" for p in ce.library_paths(device_type="cuda")]
    libs += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip", "-lamdhip64"]
    rpath = [f"-Wl,-rpath,{p}" for p in ce.library_paths(device_type="cuda")]
    return inc + defs, libs + rpath


def build_hip(jobs: int = 8, verbose: bool = False) -> str:
    out = os.path.join(PKG, "_hip" + EXT)
    sources = sorted(glob.glob(os.path.join(KDIR, "*.hip")) + glob.glob(os.path.join(KDIR, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(KDIR, "*.h")) + glob.glob(os.path.join(KDIR, "*.cuh")))
    if not sources:
        return ""
    cflags, ldflags = _torch_flags()
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
             "-munsafe-fp-atomics", "-Wno-unused-result", "-Wno-deprecated-declarations",
             "-Wno-unused-command-line-argument"] + cflags + _py_includes()
    objs, changed = _compile_all(HIPCC, sources, headers, flags, "hip", jobs)
    if changed or not os.path.exists(out):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs + ldflags)
        os.replace(out + ".tmp", out)
    if verbose:
        print("built", out)
    return out


def build_all(jobs: int = 8, verbose: bool = True):
    return build_cpu(jobs, verbose), build_hip(jobs, verbose)


if __name__ == "__main__":
    build_all(int(os.environ.get("MAX_JOBS", "8")))
    sys.exit(0)
