"""In-tree build of libpinotgpu.so (gfx950) with hipcc.  No cmake / ninja / torch extension machinery: the
library is a plain shared object with a C ABI (include/pinotgpu.h)."""
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_PATH = os.path.join(HERE, "libpinotgpu.so")
SOURCES = ["kernels.hip", "runtime.cpp"]
HEADERS = ["internal.h"]
ARCH = os.environ.get("PGPU_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build libpinotgpu.so)")


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files.append(os.path.join(ROOT, "include", "pinotgpu.h"))
    return files


def is_stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(f) > t for f in _inputs())


def build(force=False, verbose=False):
    """Compiles the kernels and the host runtime into pinot_amd/libpinotgpu.so (cross-compiles without a GPU)."""
    if not force and not is_stale():
        return LIB_PATH
    cmd = [
        _hipcc(), "--offload-arch=" + ARCH, "-O3", "-fPIC", "-shared", "-std=c++17", "-munsafe-fp-atomics",
        "-Wall", "-Wno-unused-result", "-Wno-unused-value",
        "-o", LIB_PATH + ".tmp",
    ] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    res = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + res.stdout[-8000:])
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force=True, verbose=True))
