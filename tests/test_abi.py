"""CPU-side checks of the drop-in boundary: libdhtgpu.so loads and exports every
entry point include/dhtgpu.h declares (no compute calls -- no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import opendht_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "dhtgpu.h")).read()
    return sorted(set(re.findall(r"\b(dhtgpu_[a-z0-9_]+)\s*\(", src)))


def test_library_built():
    assert os.path.exists(opendht_amd.LIB_PATH), "run __graft_entry__.build() first"


def test_exports_match_header():
    syms = header_symbols()
    assert len(syms) >= 15
    out = subprocess.check_output(["nm", "-D", "--defined-only", opendht_amd.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    assert sorted(opendht_amd.exported_symbols()) == syms


def test_ctypes_load_and_strerror():
    L = opendht_amd.lib()
    for s in header_symbols():
        assert hasattr(L, s)
    assert L.dhtgpu_strerror(0) == b"ok"
    assert L.dhtgpu_strerror(-5).startswith(b"id set holds duplicate")


def test_cpp_adapter_header_compiles(tmp_path):
    """The C++11 host adapter (include/dhtgpu.hpp) compiles as C++11 against a
    reference-shaped mock table (tests/cpp/adapter_check.cpp)."""
    src = os.path.join(ROOT, "tests", "cpp", "adapter_check.cpp")
    if not os.path.exists(src):
        pytest.skip("adapter check source absent")
    exe = build_adapter_check(str(tmp_path / "adapter_check"))
    assert subprocess.check_output([exe], text=True).strip() == "built"


def test_cpp_adapter_host_walks(tmp_path):
    """The adapter's host walks -- what a single findClosestNodes / getCachedNodes runs below the
    device threshold -- give the oracle's nodes in the oracle's order (no GPU needed)."""
    exe = build_adapter_check(str(tmp_path / "adapter_check"))
    out = subprocess.run([exe, "--host"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "0 mismatches" in out.stdout, out.stdout + out.stderr


def build_adapter_check(exe):
    src = os.path.join(ROOT, "tests", "cpp", "adapter_check.cpp")
    libdir = os.path.dirname(opendht_amd.LIB_PATH)
    odir = os.path.join(ROOT, "oracle")
    subprocess.check_call(["make", "-s", "-C", odir])
    subprocess.check_call(["g++", "-std=c++11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           src, "-o", exe, "-L", libdir, "-ldhtgpu", "-L", odir, "-loracle",
                           "-Wl,-rpath," + libdir, "-Wl,-rpath," + odir])
    return exe


def test_table_depth_vs_oracle():
    """Host-side helper of the C ABI (no device work): RoutingTable::depth."""
    import numpy as np
    import oracle as O
    import opendht_amd
    for seed in (1, 2, 3):
        firsts, _, _ = O.Table(O.gen_ids(seed, 1)[0]).grow(O.gen_ids(seed + 10, 20000)).export()
        for b in range(firsts.shape[0]):
            assert opendht_amd.table_depth(firsts, b) == O.depth(firsts, b)
    assert opendht_amd.table_depth(np.zeros((0, 20), np.uint8), 0) == 0


def test_production_build_has_no_measurement_switches():
    """The shipped library cannot return different nodes (SURVEY §8(b) error contract): the
    sources carry no result-altering measurement macro (#if/#ifdef on a DHT_* name), the Makefile
    takes no extra defines and builds gfx950 only, and DHTGPU_DBG is masked at context creation to
    the diagnostics bits that leave results unchanged (phase stamps; K6 instead of KS for small
    batches -- both exact; tests/test_gpu_parity.py::test_dbg_bits_leave_results_unchanged)."""
    csrc = os.path.join(ROOT, "opendht_amd", "csrc")
    bad = []
    for fn in sorted(os.listdir(csrc)):
        if not fn.endswith((".hip", ".h")):
            continue
        for no, line in enumerate(open(os.path.join(csrc, fn)), 1):
            if re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b.*\bDHT_[A-Z0-9_]+", line):
                bad.append(f"{fn}:{no}: {line.strip()}")
    assert not bad, bad
    mk = open(os.path.join(csrc, "Makefile")).read()
    assert "EXTRA" not in mk and "$(error" in mk and "ifneq ($(ARCH),gfx950)" in mk
    internal = open(os.path.join(csrc, "dhtgpu_internal.h")).read()
    m = re.search(r"constexpr uint32_t kDbgAllowed = ([^;]+);", internal)
    assert m and m.group(1).replace(" ", "") == "256u|(1u<<23)", m
    api = open(os.path.join(csrc, "api.hip")).read()
    assert re.search(r'getenv\("DHTGPU_DBG"\)\)\s*c->dbg = .*& kDbgAllowed;', api)
    batch = open(os.path.join(csrc, "batch.hip")).read()
    assert "c.dbg & 256u" in batch   # K6 honours the stamp bit only
