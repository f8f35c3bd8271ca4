"""The C ABI boundary on CPU: libmarlnav.so loads, exports every entry point
include/marlnav.h declares, its structs match the ctypes mirror byte for
byte, and argument validation fails loudly before anything is launched."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "marlnav.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(marlnav_\w+)\s*\(", src,
                                 re.M)))


def test_library_loads_and_exports_every_declared_symbol(pkg):
    lib = pkg.abi.load_library()
    names = declared_functions()
    assert set(names) == set(pkg.abi.EXPORTS), names
    for n in names:
        assert hasattr(lib, n), n
    assert lib.marlnav_abi_version() == pkg.abi.ABI_VERSION
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.abi.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (marlnav_\w+)", out))
    assert set(names) <= exported


def test_library_holds_gfx950_code(pkg):
    blob = open(pkg.abi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_struct_layout_matches_header(pkg, tmp_path):
    """Compile a probe against include/marlnav.h and compare offsetof/sizeof
    of every field with the ctypes structures."""
    abi = pkg.abi
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"',
             'int main(void) {']
    for cls in (abi.MarlnavDims, abi.MarlnavParams, abi.MarlnavStepBuffers):
        lines.append(f'printf("{cls.__name__} size %zu\\n", sizeof({cls.__name__}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cls.__name__} {fname} %zu\\n", '
                         f'offsetof({cls.__name__}, {fname}));')
    lines.append("return 0; }")
    c = tmp_path / "probe.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", str(c), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True,
                               check=True).stdout.splitlines():
        cls, field, val = line.split()
        got[(cls, field)] = int(val)
    for cls in (abi.MarlnavDims, abi.MarlnavParams, abi.MarlnavStepBuffers):
        assert got[(cls.__name__, "size")] == ctypes.sizeof(cls), cls.__name__
        for fname, _ in cls._fields_:
            assert got[(cls.__name__, fname)] == getattr(cls, fname).offset, (cls, fname)


def test_validation_errors_are_loud(pkg):
    abi = pkg.abi
    lib = abi.load_library()
    d = abi.MarlnavDims(num_parallel=8, num_agents=1, num_obstacles=3, obstacle_stride=3)
    assert lib.marlnav_counter_slots(ctypes.byref(d)) < 0
    assert b"num_agents" in lib.marlnav_last_error()
    d.num_agents = 3
    d.num_obstacles = 4
    rc = lib.marlnav_step(ctypes.byref(d), ctypes.byref(abi.MarlnavParams()),
                          ctypes.byref(abi.MarlnavStepBuffers()), 0, None)
    assert rc == -1 and b"num_obstacles" in lib.marlnav_last_error()
    d.num_obstacles = 3
    rc = lib.marlnav_step(ctypes.byref(d), ctypes.byref(abi.MarlnavParams()),
                          ctypes.byref(abi.MarlnavStepBuffers()), 0, None)
    assert rc == -1 and b"NULL" in lib.marlnav_last_error()
    with pytest.raises(RuntimeError, match="NULL"):
        abi.check(rc, lib)
    # one slot per wave of the grid: 20-env wave tiles at A=3, 4 waves/block
    assert lib.marlnav_counter_slots(ctypes.byref(d)) == 4
    d.num_parallel = 65536
    assert lib.marlnav_counter_slots(ctypes.byref(d)) == 3280
    # the testing hooks check their arguments before any launch
    assert lib.marlnav_debug_acos_range(0, -1, None, None) == -1
    assert b"acos range" in lib.marlnav_last_error()
    assert lib.marlnav_debug_acos_range(0, 0, None, None) == 0
    assert lib.marlnav_debug_fastdiv_check(0, 1, 4, None, None) == -1
    assert b"fastdiv check" in lib.marlnav_last_error()
    assert lib.marlnav_debug_fastdiv_check(0, 1, 0, None, None) == 0


def test_missing_library_is_an_error(pkg, tmp_path):
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pkg.abi.load_library(str(tmp_path / "nope.so"))


def test_env_refuses_cpu_device(pkg):
    from conftest import cli_args
    params = pkg.set_env_params(cli_args(), "cpu")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pkg.Env(params)
