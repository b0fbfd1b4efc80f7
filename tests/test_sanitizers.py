"""ASan + UBSan run of the host code (SURVEY §5 "Race detection / sanitizers").

The library's host sources (scene builders, flattener, SoA validation, C ABI — csrc/*.cpp)
and the CPU oracle are rebuilt with -fsanitize=address,undefined (host side only; the GPU
is not involved) and the CPU test files that drive them run again, in a child pytest with
clang's ASan runtime preloaded (python itself is not instrumented). Any ASan report or
UBSan "runtime error" fails the run (UBSan is built with -fno-sanitize-recover).
"""
import glob
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN_TESTS = ["tests/test_abi.py", "tests/test_oracle.py", "tests/test_numerics.py"]


def _asan_runtime():
    libs = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return libs[-1] if libs else None


@pytest.mark.timeout(900)
def test_host_code_under_asan_and_ubsan():
    runtime = _asan_runtime()
    if runtime is None or os.environ.get("RT_LIB_PATH"):
        pytest.skip("no clang ASan runtime (or already inside the sanitizer run)")
    import __graft_entry__ as ge
    lib, oracle = ge.build_sanitized()
    for path in (lib, oracle):   # really instrumented
        syms = subprocess.run(["nm", "-D", path], capture_output=True, text=True).stdout
        assert "__asan_report_load8" in syms and "__ubsan_handle" in syms, path
    env = dict(os.environ, RT_LIB_PATH=lib, RT_ORACLE_LIB=oracle, LD_PRELOAD=runtime,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        *SAN_TESTS, "tests/test_sanitizers.py::test_sanitized_libraries_are_the_ones_loaded"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=850)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out


def test_sanitized_libraries_are_the_ones_loaded():
    """Inside the sanitizer run: the instrumented builds, not the product ones, are mapped."""
    if not os.environ.get("RT_LIB_PATH"):
        pytest.skip("only meaningful inside test_host_code_under_asan_and_ubsan")
    import __graft_entry__ as ge
    from tests import oracle_binding as ob
    rt = ge.import_binding()
    rt.load_library()
    ob.lib()
    maps = open("/proc/self/maps").read()
    assert "librtiow_amd_asan.so" in maps and "liboracle_asan.so" in maps
    assert "libclang_rt.asan" in maps
