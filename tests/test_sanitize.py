"""ASan + UBSan over the host code, CPU only.

tools/sanitize/Makefile builds the library's host sources (schema.cpp, capi.cpp, hostpath.cpp,
jnicore.cpp) and the oracle's C restatement (oracle/row_oracle.c) with
-fsanitize=address,undefined (device code is not instrumented).  This test checks the builds are
instrumented, then runs the CPU suites that drive that host code -- schema creation and hashing,
argument and descriptor checks, JNI descriptor parsing, the randomised host fuzz, the oracle's
encode / decode of every schema family -- in a child interpreter with the ASan runtime preloaded
and the bindings pointed at the sanitized builds (FURY_ROW_LIB / FURY_ORACLE_LIB).  Any report
(halt_on_error) fails the child and so this test."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MK = os.path.join(ROOT, "tools", "sanitize")
OUT = os.path.join(ROOT, "build", "asan")
SUITES = ["tests/test_oracle.py", "tests/test_abi.py", "tests/test_jni_core.py",
          "tests/test_host_fuzz.py", "tests/test_reference_beans.py", "tests/test_arrow_export.py",
          "tests/test_workloads.py"]


def _build():
    if not shutil.which("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc")
    subprocess.run(["make", "-s", "-j", "4", "-C", MK], check=True, timeout=900)
    rt = subprocess.run(["make", "-s", "-C", MK, "print-rt"], check=True, capture_output=True,
                        text=True).stdout.strip()
    assert os.path.exists(rt), rt
    return rt


def test_host_code_under_asan_ubsan():
    rt = _build()
    for lib in ("libfury_row.so", "liborow_oracle.so"):
        syms = subprocess.run(["nm", "-D", os.path.join(OUT, lib)], check=True,
                              capture_output=True, text=True).stdout
        assert "__asan_report_load8" in syms and "__ubsan_handle" in syms, f"{lib}: not instrumented"
    env = dict(os.environ, LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               FURY_ROW_LIB=os.path.join(OUT, "libfury_row.so"),
               FURY_ORACLE_LIB=os.path.join(OUT, "liborow_oracle.so"),
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    code = ("import sys, ctypes; "
            "assert hasattr(ctypes.CDLL(None), '__asan_init'), 'ASan runtime not loaded'; "
            "import pytest; sys.exit(pytest.main(['-q', '-x', '-m', 'not gpu', '-p', "
            "'no:cacheprovider'] + sys.argv[1:]))")
    p = subprocess.run([sys.executable, "-c", code] + SUITES, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=900)
    tail = (p.stdout[-3000:] + p.stderr[-6000:])
    assert p.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error:" not in p.stderr, tail
    assert " passed" in p.stdout, tail
