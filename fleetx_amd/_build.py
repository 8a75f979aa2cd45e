"""AOT build of the native extensions (in-tree, no JIT cache).

* ``fleetx_amd/_C/_kernels*.so``: every ``csrc/kernels/*.hip`` compiled by
  ``hipcc --offload-arch=gfx950`` plus the pybind11 bindings.
* ``fleetx_amd/_C/_native*.so``: host C++ (dataset index builders, bucket
  planner) compiled by ``g++``.

Run ``python -m fleetx_amd._build`` (or ``__graft_entry__.build()``).
Objects are rebuilt only when a source or header is newer.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "fleetx_amd", "_C")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes():
    import pybind11
    return ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n{}\n{}".format(" ".join(cmd), r.stdout))
    return r.stdout


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    return "hipcc"


def build_kernels(verbose=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    kdir = os.path.join(CSRC, "kernels")
    headers = glob.glob(os.path.join(kdir, "*.h")) + glob.glob(os.path.join(kdir, "*.inc"))
    hips = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    common = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-munsafe-fp-atomics",
              "-Wno-unused-result"]
    jobs_list = []
    objs = []
    for src in hips:
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer(obj, [src] + headers):
            jobs_list.append([hipcc()] + common + ["-c", src, "-o", obj])
    bsrc = os.path.join(kdir, "bindings.cpp")
    bobj = os.path.join(OBJ, "bindings.o")
    objs.append(bobj)
    if _newer(bobj, [bsrc]):
        jobs_list.append([hipcc(), "-O2", "-std=c++17", "-fPIC", "-x", "c++", "-D__HIP_PLATFORM_AMD__"]
                         + _py_includes() + ["-I/opt/rocm/include", "-c", bsrc, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 4)) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)
    so = os.path.join(OUT, "_kernels" + EXT)
    if _newer(so, objs):
        _run([hipcc(), "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", so] + objs)
    return so


def build_native(verbose=False):
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(CSRC, "native", "index_helpers.cpp")
    so = os.path.join(OUT, "_native" + EXT)
    if _newer(so, [src]):
        cxx = os.environ.get("CXX", "g++")
        _run([cxx, "-O3", "-std=c++17", "-shared", "-fPIC"] + _py_includes() + [src, "-o", so])
    return so


def build_all(verbose=False):
    paths = [build_native(verbose), build_kernels(verbose)]
    if verbose:
        for p in paths:
            print("built", p)
    return paths


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv)
