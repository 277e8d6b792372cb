"""In-tree build of the native pieces.

* ``_roaring``  – host roaring core (C++17, g++), pybind11 module.
* ``_hipkernels`` – HIP/CDNA4 kernels for gfx950 as a torch extension
  (hipcc --offload-arch=gfx950), see pilosa_amd/kernels/.

Both land next to the package (``pilosa_amd/_roaring*.so``,
``pilosa_amd/_hipkernels*.so``) so they travel with the gpurun snapshot and are
visible to the round-end "native code loaded" check.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
KDIR = os.path.join(PKG, "kernels")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _newer(target: str, sources) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build_roaring(force: bool = False, verbose: bool = False, stats: bool = False) -> str:
    """Host roaring core.  ``stats`` builds the instrumented variant as the
    separate module ``_roaring_stats`` (the reference's ``roaringstats`` build
    tag); ``PILOSA_ROARING_STATS=1`` instruments the default ``_roaring``."""
    import pybind11

    name = "_roaring_stats" if stats else "_roaring"
    out = os.path.join(PKG, name + _ext_suffix())
    srcs = [os.path.join(HERE, f) for f in ("roaring.cpp", "pyroaring.cpp", "arena_io.cpp", "mapped.cpp",
                                          "wire_decode.cpp")]
    deps = srcs + [os.path.join(HERE, f) for f in ("roaring.hpp", "synth.hpp")]
    if not force and not _newer(out, deps):
        return out
    cxx = os.environ.get("CXX", "g++")
    flags = os.environ.get("PILOSA_AMD_CXXFLAGS", "-O3 -mpopcnt -mbmi2 -mavx2").split()
    if stats or os.environ.get("PILOSA_ROARING_STATS", "0") == "1":
        flags.append("-DPILOSA_ROARING_STATS")
    if stats:
        # own module name and C++ namespace: both variants can load in one process
        flags += [f"-DPILOSA_ROARING_MODULE={name}", "-Dpr=pr_stats"]
    cmd = [cxx, "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", *flags,
           "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], *srcs,
           "-o", out + ".tmp", "-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_pql(force: bool = False, verbose: bool = False) -> str:
    import pybind11

    out = os.path.join(PKG, "_pql" + _ext_suffix())
    srcs = [os.path.join(HERE, "pql_parser.cpp"), os.path.join(HERE, "pql_compile.cpp")]
    if not force and not _newer(out, srcs):
        return out
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-std=c++17", "-O2", "-shared", "-fPIC", "-fvisibility=hidden", "-I", pybind11.get_include(),
           "-I", sysconfig.get_paths()["include"], *srcs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_httpd(force: bool = False, verbose: bool = False) -> str:
    """Native HTTP/1.1 front end (httpd.cpp), pybind11 module ``_httpd``."""
    import pybind11

    out = os.path.join(PKG, "_httpd" + _ext_suffix())
    srcs = [os.path.join(HERE, "httpd.cpp")]
    if not force and not _newer(out, srcs):
        return out
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-std=c++17", "-O2", "-shared", "-fPIC", "-fvisibility=hidden", "-I", pybind11.get_include(),
           "-I", sysconfig.get_paths()["include"], *srcs, "-o", out + ".tmp", "-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_shmring(force: bool = False, verbose: bool = False) -> str:
    """The mesh command ring (native/shmring.cpp, POSIX shm + futex)."""
    import pybind11
    src = os.path.join(HERE, "shmring.cpp")
    out = os.path.join(PKG, "_shmring" + _ext_suffix())
    if not force and not _newer(out, [src]):
        return out
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-std=c++17", "-O2", "-shared", "-fPIC", "-fvisibility=hidden", "-I", pybind11.get_include(),
           "-I", sysconfig.get_paths()["include"], src, "-o", out + ".tmp", "-lrt"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_translate(force: bool = False, verbose: bool = False) -> str:
    """Key translation store (translate.cpp), pybind11 module ``_translate``."""
    import pybind11

    out = os.path.join(PKG, "_translate" + _ext_suffix())
    srcs = [os.path.join(HERE, "translate.cpp")]
    if not force and not _newer(out, srcs):
        return out
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-std=c++17", "-O2", "-shared", "-fPIC", "-fvisibility=hidden", "-I", pybind11.get_include(),
           "-I", sysconfig.get_paths()["include"], *srcs, "-o", out + ".tmp", "-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


HOST_MODULES = {
    "_roaring": ("roaring.cpp", "pyroaring.cpp", "arena_io.cpp", "mapped.cpp", "wire_decode.cpp"),
    "_pql": ("pql_parser.cpp", "pql_compile.cpp"),
    "_httpd": ("httpd.cpp",),
    "_translate": ("translate.cpp",),
}


def build_sanitized(name: str, sanitize: str, outdir: str, verbose: bool = False) -> str:
    """A host module built with ``-fsanitize=<sanitize>`` into ``outdir``
    (never in-tree: the sanitizer runtime has to be preloaded into the
    interpreter that imports it).  Used by tests/test_native_sanitizers.py."""
    import pybind11

    os.makedirs(outdir, exist_ok=True)
    out = os.path.join(outdir, name + _ext_suffix())
    srcs = [os.path.join(HERE, f) for f in HOST_MODULES[name]]
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}"]
    if "undefined" in sanitize:
        flags.append("-fno-sanitize-recover=undefined")
    if name == "_roaring":
        flags += ["-mpopcnt", "-mbmi2", "-mavx2"]
    cmd = [cxx, "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", *flags, "-I", pybind11.get_include(),
           "-I", sysconfig.get_paths()["include"], *srcs, "-o", out, "-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return out


def hip_sources():
    return [os.path.join(KDIR, f) for f in sorted(os.listdir(KDIR))
            if f.endswith((".hip", ".cpp", ".h", ".hpp"))]


def build_hip(force: bool = False, verbose: bool = False, kbench: bool = False) -> str:
    """Compile the HIP kernels + torch binding for gfx950 with hipcc.
    ``kbench``: the A/B module ``_hipkernels_kbench`` (-DPK_KBENCH) that also
    holds the measured-and-rejected kernel variants and the cost-isolation
    skeletons (scripts/kbench.py, scripts/topn_kbench.py); the shipped
    ``_hipkernels`` has none of them."""
    import torch
    from torch.utils import cpp_extension

    name = "_hipkernels_kbench" if kbench else "_hipkernels"
    out = os.path.join(PKG, name + _ext_suffix())
    deps = hip_sources()
    if not force and not _newer(out, deps):
        return out
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    tinc = cpp_extension.include_paths()
    tlib = cpp_extension.library_paths()
    arch = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
    srcs = sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith((".hip", ".cpp")))
    objs = []
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              f"-DTORCH_EXTENSION_NAME={name}", "-DTORCH_API_INCLUDE_EXTENSION_H",
              *(["-DPK_KBENCH"] if kbench else []),
              "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              *[f"-I{p}" for p in tinc], "-I", sysconfig.get_paths()["include"]]
    bdir = os.path.join(PKG, "native", "_obj_kbench" if kbench else "_obj")
    os.makedirs(bdir, exist_ok=True)
    procs = []
    for s in srcs:
        o = os.path.join(bdir, os.path.basename(s) + ".o")
        objs.append(o)
        if s.endswith(".hip"):
            cmd = [hipcc, f"--offload-arch={arch}", "-x", "hip", "-c", s, "-o", o, *common,
                   "-munsafe-fp-atomics"]
        else:
            cmd = [hipcc, "-c", s, "-o", o, *common]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    link = [hipcc, "-shared", "-fPIC", *objs, "-o", out + ".tmp",
            *[f"-L{p}" for p in tlib], "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-lc10_hip", "-ltorch_hip", f"--offload-arch={arch}"]
    for p in tlib:
        link.append(f"-Wl,-rpath,{p}")
    if verbose:
        print(" ".join(link))
    subprocess.check_call(link)
    os.replace(out + ".tmp", out)
    return out


def build_all(force: bool = False, verbose: bool = False):
    from pilosa_amd import buildinfo
    buildinfo.write()      # version / build time / release / enterprise of this build
    r = build_roaring(force, verbose)
    build_roaring(force, verbose, stats=True)
    build_pql(force, verbose)
    build_httpd(force, verbose)
    build_translate(force, verbose)
    build_shmring(force, verbose)
    h = build_hip(force, verbose) if os.path.exists(os.path.join(KDIR, "binding.cpp")) else None
    return r, h


if __name__ == "__main__":
    force = "--force" in sys.argv
    if "--kbench" in sys.argv:
        print(build_hip(force=force, verbose=True, kbench=True))
    else:
        print(build_all(force=force, verbose=True))
