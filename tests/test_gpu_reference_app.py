"""The reference APPLICATION — RaytracingEngine.cpp's own main(), unmodified — compiled against
this repository's drop-in C++ API (oracle/Makefile target `dropin`) and run on the MI355X.

It renders the reference box scene plus the OBJ model (tests/golden/box.obj: the reference repo
ships no box.obj) at 1000×1000 with the reference default AA=32, tonemaps with the application's
own seven operators and writes seven PPMs.  The reference's AA jitter is unseeded, so the pin is
statistical: 20×20-pixel block means of each PPM against the same application on the reference
CPU renderer (tests/golden/refapp_blocks.npz)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "ref_app_on_rtamd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
NAMES = ["simple", "reinhard_simple", "reinhard_extended", "reinhard_extended_luminance",
         "reinhard_jodie", "uncharted2", "aces"]


def blocks(path, block=20):
    data = open(path, "rb").read()
    header = b"P6\n1000 1000\n255\n"
    assert data.startswith(header)
    img = np.frombuffer(data[len(header):], np.uint8).reshape(1000, 1000, 3).astype(np.float64)
    return img.reshape(1000 // block, block, 1000 // block, block, 3).mean(axis=(1, 3))


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(EXE), reason="built only where /root/reference exists")
def test_reference_main_runs_on_mi355x(tmp_path):
    shutil.copy(os.path.join(GOLDEN, "box.obj"), tmp_path)
    res = subprocess.run([EXE], cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr
    assert res.stdout.count("Image written to") == 7
    # the ffmpeg / del calls never fork: -Wl,--wrap=system (oracle/dropin_nosystem.c)
    assert res.stderr.count("system() not run") == 7, res.stderr
    ref = np.load(os.path.join(GOLDEN, "refapp_blocks.npz"))["blocks"]
    for k, name in enumerate(NAMES):
        got = blocks(tmp_path / f"{name}.ppm")
        d = np.abs(got - ref[k])
        # 32 jittered samples x 400 pixels per block: sampling noise is well under a byte
        assert d.mean() < 0.5 and d.max() < 8.0, (name, d.mean(), d.max())


@pytest.mark.skipif(not os.path.exists(EXE), reason="built only where /root/reference exists")
def test_dropin_app_has_no_system_call():
    """The drop-in application resolves std::system to the non-forking wrapper: no undefined
    `system` symbol is left for the dynamic loader (runs on the CPU too)."""
    res = subprocess.run(["nm", "-D", "--undefined-only", EXE], capture_output=True, text=True,
                         check=True)
    assert not [ln for ln in res.stdout.split() if ln.split("@")[0] == "system"]
