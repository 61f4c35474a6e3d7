"""CPU-side checks of the drop-in boundary: libpinotgpu.so builds for gfx950, loads without a GPU and exports
every entry point include/pinotgpu.h declares (no compute call is made here)."""
import ctypes
import os
import re
import subprocess

from pinot_amd import _lib as L
from pinot_amd.build import LIB_PATH, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "pinotgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pgpu_[a-z0-9_]+)\s*\(", src)))


def test_library_builds_and_loads():
    build()
    assert os.path.exists(LIB_PATH)
    lib = L.load()
    assert lib.pgpu_abi_version() == 3


def test_every_declared_symbol_is_exported_and_bound():
    build()
    declared = _declared()
    assert len(declared) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], stdout=subprocess.PIPE, text=True).stdout
    exported = set(re.findall(r"\bT (pgpu_[a-z0-9_]+)", out))
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert sorted(L.exported_symbols()) == declared


def test_gfx950_code_object_present():
    build()
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          "--input=" + LIB_PATH], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    data = open(LIB_PATH, "rb").read()
    assert b"gfx950" in data, out.stdout


def test_last_error_without_device():
    lib = L.load()
    buf = ctypes.create_string_buffer(64)
    assert lib.pgpu_last_error(buf, len(buf)) >= 0
    # argument validation happens before any device call
    assert lib.pgpu_result_stats(None, None) == L.PGPU_ERR_INVALID_ARGUMENT
    assert "bad arguments" in L.last_error()


def test_config_defaults():
    """pgpu_config_default: the library's executor settings (include/pinotgpu.h), no device needed."""
    lib = L.load()
    c = L.ConfigC()
    assert lib.pgpu_config_default(ctypes.byref(c)) == 0
    assert c.struct_size == ctypes.sizeof(L.ConfigC)
    got = {f: getattr(c, f) for f in L.CONFIG_FIELDS}
    assert got == {"plan_cache": 1, "partitioned_group_by": 1, "hash_partitions": 1, "hash_partition_bits": 14,
                   "hash_partition_lds_kb": 0, "lds_table_kb": 112, "plan_chunk_segments": 4096, "stream_chunks": 1,
                   "compact_results": 1, "star_tree_workgroups": 0, "dense_selectivity": 0.25,
                   "slot_weight_step": 0.11}
    assert lib.pgpu_config_default(None) == L.PGPU_ERR_INVALID_ARGUMENT
    assert lib.pgpu_table_set_config(None, ctypes.byref(c)) == L.PGPU_ERR_INVALID_ARGUMENT


def test_only_diagnostics_read_from_the_environment():
    """Executor settings come from pgpu_config, never the environment: the variables the library reads are the
    diagnostics switch PGPU_TRACE and the diagnostics build's raw workgroup-times file."""
    csrc = os.path.join(ROOT, "pinot_amd", "csrc")
    names = set()
    for f in os.listdir(csrc):
        src = open(os.path.join(csrc, f)).read()
        names |= set(re.findall(r'getenv\("([A-Z0-9_]+)"\)', src))
        assert "getenv_flag" not in src, f
    assert names == {"PGPU_TRACE", "PGPU_WGTIMES_OUT"}, names
