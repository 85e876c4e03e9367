"""In-tree build of the native extension ``_C`` (HIP kernels for gfx950 + C++ host runtime).

Kernels (``csrc/kernels/*.hip``) are compiled by ``hipcc --offload-arch=gfx950``; host code
(``csrc/bindings.cpp``, ``csrc/host/*.cpp``) by ``g++`` against libtorch; everything is linked into
``rag_tl_domainllm_optimizer_amd/_C*.so`` next to this file, so the built library travels with the
repository snapshot to the GPU box. Objects are cached by content hash under ``build/``.

No hipify step and no CUDA sources: this is CDNA4 code only.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
ROCM = os.environ.get("ROCM_HOME", "/opt/rocm")
ARCH = os.environ.get("RAGTL_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"


def _ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, EXT_NAME + suffix)


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash_files(paths, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()[:16]


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def kernel_flags(debug: bool = False):
    opt = ["-O1", "-g", "-DRAGTL_DEBUG=1"] if debug else ["-O3"]
    return [
        "-x", "hip", f"--offload-arch={ARCH}", *opt, "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
        "-I", os.path.join(CSRC, "include"), "-Wno-unused-result",
    ]


def host_flags(debug: bool = False, sanitize: bool = False):
    inc, _, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    flags = ["-O1", "-g"] if (debug or sanitize) else ["-O2"]
    if sanitize:
        # host-only AddressSanitizer + UBSan (tokenizer, IVF host code, bindings); the runtime is
        # LD_PRELOADed into python, GPU code is never sanitized
        flags += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
    flags += [
        "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-DTORCH_API_INCLUDE_EXTENSION_H", "-fopenmp",
        "-I", CSRC, "-I", os.path.join(CSRC, "include"), "-I", py_inc, "-I", os.path.join(ROCM, "include"),
        "-Wno-deprecated-declarations", "-Wno-unused-variable",
    ]
    for i in inc:
        flags += ["-isystem", i]
    return flags


def build(verbose: bool = False, force: bool = False, jobs: int | None = None, debug: bool = False,
          sanitize: bool = False) -> str:
    """Compile every HIP kernel for gfx950 and link the extension. Returns the .so path.
    ``sanitize`` builds the host C++ with ASan/UBSan into build/asan/ (load it with
    RAGTL_EXT_PATH=<path> and LD_PRELOAD of libasan / libubsan)."""
    os.makedirs(BUILD, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    headers = glob.glob(os.path.join(CSRC, "include", "*.h")) + glob.glob(os.path.join(CSRC, "host", "*.h"))
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hosts = [os.path.join(CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    kf, hf = kernel_flags(debug), host_flags(debug, sanitize)

    jobs_list = []
    objs = []
    for src in kernels:
        key = _hash_files([src] + headers, " ".join(kf))
        obj = os.path.join(BUILD, f"{os.path.basename(src)}.{key}.o")
        objs.append(obj)
        if force or not os.path.exists(obj):
            jobs_list.append([hipcc, *kf, "-c", src, "-o", obj])
    for src in hosts:
        key = _hash_files([src] + headers, " ".join(hf))
        obj = os.path.join(BUILD, f"{os.path.basename(src)}.{key}.o")
        objs.append(obj)
        if force or not os.path.exists(obj):
            jobs_list.append(["g++", *hf, "-c", src, "-o", obj])

    n = jobs or min(8, os.cpu_count() or 4, int(os.environ.get("MAX_JOBS", "8")))
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for fut in [ex.submit(_run, c, verbose) for c in jobs_list]:
                fut.result()

    out = _ext_path()
    stamp = os.path.join(BUILD, "link.stamp")
    if sanitize:
        adir = os.path.join(REPO, "build", "asan")
        os.makedirs(adir, exist_ok=True)
        out = os.path.join(adir, os.path.basename(out))
        stamp = os.path.join(adir, "link.stamp")
    link_key = hashlib.sha256("|".join(objs).encode()).hexdigest()[:16]
    prev = open(stamp).read().strip() if os.path.exists(stamp) else ""
    if force or jobs_list or prev != link_key or not os.path.exists(out):
        _, tlib, _ = _torch_paths()
        tmp = out + ".tmp"
        _run([hipcc, "-shared", "-fPIC", "-fopenmp", *objs, "-o", tmp, f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch",
              "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", f"-L{os.path.join(ROCM, 'lib')}", "-lamdhip64",
              f"-Wl,-rpath,{tlib}"], verbose)
        os.replace(tmp, out)
        with open(stamp, "w") as f:
            f.write(link_key)
    return out


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build(verbose="-v" in sys.argv, force=force, debug="--debug" in sys.argv, sanitize="--sanitize" in sys.argv))
