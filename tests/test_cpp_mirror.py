"""The C++ host mirror (include/storb_piece.hpp) and its reference-test port.

CPU: the test binary compiles and links against libstorb_rs.so.
GPU: it runs (the Rust-style tests of piece.rs on the MI355X path).
"""
import os
import subprocess

import pytest

from storb_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_piece.cpp")
OUT = os.path.join(ROOT, "tests", "cpp", "_build", "test_piece")


def build_binary():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", OUT, SRC, f"-L{libdir}", "-lstorb_rs",
                    f"-Wl,-rpath,{libdir}", "-lpthread"], check=True)
    return OUT


def test_cpp_mirror_compiles_and_links():
    assert os.path.exists(build_binary())


@pytest.mark.gpu
def test_cpp_mirror_reference_tests_pass():
    exe = build_binary()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_host_pool_copies_and_runs_every_part():
    src = os.path.join(ROOT, "tests", "cpp", "test_host_pool.cpp")
    exe = os.path.join(ROOT, "tests", "cpp", "_build", "test_host_pool")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe, src], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host pool ok" in r.stdout


def test_sequence_numbers_skip_zero_across_the_wrap():
    """the slice words start zeroed, so a sequence number of 0
    would match a never-written word after 2^32 calls (storb_amd/csrc/seq.hpp)."""
    src = os.path.join(ROOT, "tests", "cpp", "test_seq.cpp")
    exe = os.path.join(ROOT, "tests", "cpp", "_build", "test_seq")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, src], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "seq ok" in r.stdout


def test_pattern_memo_matches_get_pattern():
    """The per-call pattern memo in front of the decode-pattern cache
    (decode_stripes.cpp PatternMemo) returns what get_pattern returns --
    pattern, slot positions, error code -- for arrival-ordered share lists
    with duplicates, too few shares, bad indices and n > 64."""
    src = os.path.join(ROOT, "tests", "cpp", "test_pattern_memo.cpp")
    exe = os.path.join(ROOT, "tests", "cpp", "_build", "test_pattern_memo")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I" + os.path.join(ROOT, "include"), "-o", exe, src, f"-L{libdir}",
                    "-lstorb_rs", f"-Wl,-rpath,{libdir}", "-lpthread"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pattern memo ok" in r.stdout
