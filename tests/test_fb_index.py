"""CPU check of the filter-bank kernels' tile decode (csrc/fb_index.h, compiled for the host): the
scalar-unit Granlund-Montgomery divisions against integer division (every divisor up to 65 536,
random ones up to 2^31, dividends near multiples and near 2^31), the XCD-aware tile order as a
permutation, and the frame decode listing each tile outside the interior rectangle exactly once
(empty rectangles, full-width rectangles, c0 = 0).  Only the GPU parity tests reach these on the
device, and over a few shapes."""
import ctypes
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libfbindex.so")
HDR = os.path.join(HERE, "..", "wavelettransforms_amd", "csrc", "fb_index.h")


@pytest.fixture(scope="module")
def fb():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "native", "fbindex.cpp")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(HDR)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO, src])
    return ctypes.CDLL(SO)


def test_fastdiv_exact(fb):
    assert fb.fb_check_fdiv() == 0


def test_xcd_tile_is_a_permutation(fb):
    assert fb.fb_check_xcd() == 0


def test_frame_decode_covers_the_frame_once(fb):
    assert fb.fb_check_frame() == 0
