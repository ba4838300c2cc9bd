"""CPU check of the one-launch small path's tile geometry (csrc/small_geom.h, compiled for the
host): over many line lengths, filter lengths, levels and tile sizes, every sample an analysis
output (wt_ana_point's taps) or a synthesis output (wt_syn_pass's taps) reads lies in the tile's
window of the level below, and the owned ranges partition every level (tests/native/smallgeom.cpp)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "_build", "smallgeom")


def test_small_windows_cover_every_tap():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    src = os.path.join(HERE, "native", "smallgeom.cpp")
    hdr = os.path.join(HERE, "..", "wavelettransforms_amd", "csrc", "small_geom.h")
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", EXE, src])
    out = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-2000:]
    assert out.stdout.strip().endswith("0 failing")
