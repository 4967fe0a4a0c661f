"""Build the native library in-tree: aclswarm_amd/lib/libaclswarm_amd.so.

hipcc --offload-arch=gfx950, -ffp-contract=off (every f64 op one IEEE
rounding: the assignment must be bit-identical to the CPU restatement).
Usage: python -m aclswarm_amd.build
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lib", "libaclswarm_amd.so")
ROOT = os.path.dirname(HERE)
# C++ facade exerciser (include/aclswarm_amd.hpp), run by tests/test_gpu_facade.py
DRIVER_SRC = os.path.join(ROOT, "tests", "facade_driver.cpp")
DRIVER = os.path.join(HERE, "lib", "libfacade_driver.so")
# the codegen-compatible ADMM entry points driven as aclswarm/src/admm.cpp does
CG_DRIVER_SRC = os.path.join(ROOT, "tests", "codegen_driver.cpp")
CG_DRIVER = os.path.join(HERE, "lib", "libcodegen_driver.so")
SOURCES = ["solve.hip", "auction.hip", "solve_wide.hip", "control.hip", "admm.hip", "hungarian.hip", "cbaa_step.hip", "episode.hip",
           "trial.hip", "formation_gen.hip", "api.cpp"]
# The generated ADMM library's C++ entry points (ADMMGainDesign3D and the
# generic MATLAB-Coder emx utilities) live in their own shim library linked to
# the core, so a process that loads libaclswarm_amd.so next to another
# Coder-generated library does not get these common names interposed.
CODEGEN_SRC = os.path.join(CSRC, "codegen_api.cpp")
CODEGEN_OUT = os.path.join(HERE, "lib", "libaclswarm_amd_codegen.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
         "-fPIC", "-shared", "-Wall", "-Wno-unused-function"]


OBJ = os.path.join(ROOT, "build", "obj")


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(ROOT, "include", "aclswarm_amd.h"))
    return hs


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + _headers()
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile_objects(force, verbose, extra=()):
    """One hipcc per translation unit, in parallel (each TU launches its own
    kernels: no relocatable device code); an object is rebuilt when its
    source or any header is newer."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = max(os.path.getmtime(h) for h in _headers() if os.path.exists(h))
    jobs, objs = [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OBJ, src + ".o")
        objs.append(obj)
        if (force or not os.path.exists(obj) or os.path.getmtime(obj) < max(
                os.path.getmtime(path), hdr_t)):
            flags = [f for f in FLAGS if f != "-shared"] + list(extra)
            jobs.append([HIPCC] + flags + ["-c", path, "-o", obj + ".tmp"])
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(cmd[-1], cmd[-1][:-4])

    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(run, jobs))
    return objs


def _gxx_driver(src, out, incs, deps, force, verbose, libs=("aclswarm_amd",)):
    if not force and os.path.exists(out) and all(
            os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    cmd = (["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fPIC", "-shared"] +
           ["-I" + i for i in incs] + [src, "-L" + os.path.dirname(OUT)] +
           ["-l" + x for x in libs] + ["-Wl,-rpath,$ORIGIN", "-o", out + ".tmp"])
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_driver(force=False, verbose=False):
    """g++ against the library, found next to the binary ($ORIGIN): the C++
    facade exerciser and the codegen-entry-point driver."""
    inc = os.path.join(ROOT, "include")
    build_codegen(force, verbose)
    _gxx_driver(CG_DRIVER_SRC, CG_DRIVER, [os.path.join(inc, "codegen_admm")],
                [CG_DRIVER_SRC, OUT, CODEGEN_OUT, os.path.join(inc, "aclswarm_amd_codegen.h")],
                force, verbose, libs=("aclswarm_amd_codegen", "aclswarm_amd"))
    return _gxx_driver(DRIVER_SRC, DRIVER, [inc],
                       [DRIVER_SRC, OUT, os.path.join(inc, "aclswarm_amd.hpp")], force, verbose)


def build_codegen(force=False, verbose=False):
    """libaclswarm_amd_codegen.so: the codegen entry points over the core's C
    ABI (host code only), found next to the core ($ORIGIN)."""
    deps = [CODEGEN_SRC, OUT, os.path.join(ROOT, "include", "aclswarm_amd.h"),
            os.path.join(ROOT, "include", "aclswarm_amd_codegen.h")]
    if not force and os.path.exists(CODEGEN_OUT) and all(
            os.path.getmtime(d) <= os.path.getmtime(CODEGEN_OUT) for d in deps):
        return CODEGEN_OUT
    cmd = (["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fPIC", "-shared",
            CODEGEN_SRC, "-L" + os.path.dirname(OUT), "-laclswarm_amd", "-Wl,-rpath,$ORIGIN",
            "-o", CODEGEN_OUT + ".tmp"])
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(CODEGEN_OUT + ".tmp", CODEGEN_OUT)
    return CODEGEN_OUT


def build(force=False, verbose=False):
    if not force and not _stale():
        build_driver(force, verbose)
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    objs = _compile_objects(force, verbose)
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared"] + objs + ["-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    build_driver(True, verbose)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
