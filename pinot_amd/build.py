"""In-tree build of libpinotgpu.so (gfx950) with hipcc.  No cmake / ninja / torch extension machinery: the
library is a plain shared object with a C ABI (include/pinotgpu.h)."""
import hashlib
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_PATH = os.path.join(HERE, "libpinotgpu.so")
# (source, extra flags, object name): the scan kernels are compiled once per accumulator mode so the objects
# build in parallel.
# the host runtime (rt.h): rt_* (core, dictionaries, planning, execution, numGroupsLimit / plan cache) and the C ABI
RUNTIME = ["rt_core", "rt_dict", "rt_plan", "rt_exec", "rt_groups", "abi_table", "abi_plan", "abi_combine",
           "abi_result"]
SOURCES = [("kernels.hip", [], "kernels")] + [(n + ".cpp", [], n) for n in RUNTIME] + [("startree.cpp", [], "startree"),
           ("filter_stats.cpp", [], "filter_stats"), ("range_index.cpp", [], "range_index"), ("comm.cpp", [], "comm"), ("server_response.cpp", [], "server_response"),
           ("k_partition.hip", [], "k_partition"), ("k_hashfinal.hip", [], "k_hashfinal")] + \
    [("k_direct.hip", ["-DPGPU_MODE=%d" % m], "k_direct_%d" % m) for m in range(3)] + \
    [("k_startree.hip", ["-DPGPU_MODE=%d" % m], "k_startree_%d" % m) for m in range(3)]
HEADERS = ["internal.h", "device.h", "scan_direct.h", "host_common.h", "startree_kernels.h",
           "partition.h", "filter_stats.h", "host_result.h", "comm.h", "range_index.h", "rt.h",
           "rt_decls.h"]
ARCH = os.environ.get("PGPU_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build libpinotgpu.so)")


def _inputs():
    files = [os.path.join(CSRC, s[0]) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]
    files.append(os.path.join(ROOT, "include", "pinotgpu.h"))
    return files


def is_stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(f) > t for f in _inputs())


def build(force=False, verbose=False, defines=(), out=None):
    """Compiles the kernels and the host runtime into pinot_amd/libpinotgpu.so (cross-compiles without a GPU).
    Each source is compiled to an object in parallel, then linked.  `defines` / `out`: an A/B variant of the
    library (e.g. ("PGPU_MIN_WAVES=1",)) written to `out` instead, loaded with PGPU_LIB=<out>."""
    lib_path = out or LIB_PATH
    if not force and not defines and not out and not is_stale():
        return LIB_PATH
    hipcc = _hipcc()
    flags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
             "-Wall", "-Wno-unused-result", "-Wno-unused-value"] + ["-D" + d for d in defines]
    objdir = os.path.join(ROOT, "build", "obj" if not out else "obj_" + os.path.basename(out).replace(".", "_"))
    os.makedirs(objdir, exist_ok=True)
    procs = []
    objs = []
    # an object is rebuilt when its command, its source or any header changed (key file beside the object)
    common = hashlib.sha1()
    for h in HEADERS + ["../../include/pinotgpu.h"]:
        with open(os.path.join(CSRC, h), "rb") as f:
            common.update(f.read())
    for src, extra, name in SOURCES:
        obj = os.path.join(objdir, name + ".o")
        objs.append(obj)
        # host sources carry line tables (-g does not change -O3 host code): crash traces resolve with addr2line
        dbg = ["-g"] if src.endswith(".cpp") else []
        cmd = [hipcc] + flags + dbg + extra + ["-c", os.path.join(CSRC, src), "-o", obj]
        key = common.copy()
        key.update(" ".join(cmd).encode())
        with open(os.path.join(CSRC, src), "rb") as f:
            key.update(f.read())
        key = key.hexdigest()
        if not force and os.path.exists(obj) and os.path.exists(obj + ".key"):
            with open(obj + ".key") as f:
                if f.read() == key:
                    continue
        if verbose:
            print(" ".join(cmd))
        procs.append((src, obj, key, subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                                      text=True)))
    errors = []
    for src, obj, key, pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            errors.append("%s:\n%s" % (src, out[-8000:]))
        else:
            with open(obj + ".key", "w") as f:
                f.write(key)
    if errors:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errors))
    cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib_path + ".tmp"] + objs + ["-ldl"]
    res = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + res.stdout[-8000:])
    os.replace(lib_path + ".tmp", lib_path)
    return lib_path


def build_tools():
    """tools/qps_native: concurrent callers of the C ABI without Python (links the in-tree library)."""
    hipcc = _hipcc()
    out = os.path.join(ROOT, "tools", "qps_native")
    cmd = [hipcc, "--offload-arch=" + ARCH, "-O2", "-std=c++17", os.path.join(ROOT, "tools", "qps_native.cpp"), "-I" + os.path.join(ROOT, "include"),
           "-L" + HERE, "-lpinotgpu", "-Wl,-rpath,$ORIGIN/../pinot_amd", "-o", out]
    res = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc (tools) failed:\n" + res.stdout[-4000:])
    return out


SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
             "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer"]
FUZZ_PATH = os.path.join(ROOT, "build", "host_fuzz")


def build_host_fuzz(force=False):
    """build/host_fuzz: tools/host_fuzz.cpp linked with every library source compiled for the host only under
    AddressSanitizer + UndefinedBehaviorSanitizer (host-only flags: the device code is compiled as usual, and the
    harness calls pure host entry points, never a kernel).  Rebuilt when a source is newer than the binary."""
    src = os.path.join(ROOT, "tools", "host_fuzz.cpp")
    if not force and os.path.exists(FUZZ_PATH) and \
            all(os.path.getmtime(f) <= os.path.getmtime(FUZZ_PATH) for f in _inputs() + [src]):
        return FUZZ_PATH
    hipcc = _hipcc()
    flags = ["--offload-arch=" + ARCH, "-O1", "-g", "-std=c++17", "-fPIC",
             "-I" + os.path.join(ROOT, "include")] + SAN_FLAGS
    objdir = os.path.join(ROOT, "build", "obj_san")
    os.makedirs(objdir, exist_ok=True)
    jobs = [(os.path.join(CSRC, s), extra, os.path.join(objdir, name + ".o")) for s, extra, name in SOURCES]
    jobs.append((src, [], os.path.join(objdir, "host_fuzz_main.o")))
    hdr_t = max(os.path.getmtime(f) for f in _inputs() if not f.endswith((".cpp", ".hip")))
    procs = [(s, subprocess.Popen([hipcc] + flags + extra + ["-c", s, "-o", o], cwd=ROOT, stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True)) for s, extra, o in jobs
             if force or not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_t)]
    errors = []
    for s, pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            errors.append("%s:\n%s" % (s, out[-6000:]))
    if errors:
        raise RuntimeError("hipcc (host sanitizers) failed:\n" + "\n".join(errors))
    cmd = [hipcc, "--offload-arch=" + ARCH, "-fsanitize=address", "-fsanitize=undefined", "-o", FUZZ_PATH + ".tmp"] + \
        [o for _, _, o in jobs] + ["-ldl", "-lpthread"]
    res = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc (host sanitizers) link failed:\n" + res.stdout[-6000:])
    os.replace(FUZZ_PATH + ".tmp", FUZZ_PATH)
    return FUZZ_PATH


if __name__ == "__main__":
    print(build(force=True, verbose=True))
