"""ASan + UBSan builds of the CPU-side code: the C oracle (tests/native/sancheck.c
compiles oracle/wtprune_oracle.c in) and the product's host-compilable filter-bank core
(tests/native/sancore.cpp over csrc/wt_dwt_core.h), each as a standalone program run to
completion with every sanitizer report fatal."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_build")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def _build_and_run(cc, src, exe, extra):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, exe)
    subprocess.check_call([cc] + SAN + extra + ["-o", path, os.path.join(HERE, "native", src), "-lm"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([path], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    return p.stdout


@pytest.mark.timeout(900)
def test_oracle_asan_ubsan():
    out = _build_and_run("gcc", "sancheck.c", "sancheck", ["-std=c11", "-ffp-contract=off", "-fopenmp"])
    assert "cases clean" in out


@pytest.mark.timeout(600)
def test_filterbank_core_asan_ubsan():
    out = _build_and_run("g++", "sancore.cpp", "sancore", ["-std=c++17", "-ffp-contract=off"])
    assert "cases clean" in out
