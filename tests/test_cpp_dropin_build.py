"""Source compatibility: the reference application file (RaytracingEngine.cpp, unmodified)
compiles and links against this repository's drop-in C++ API (Math.h, Shape.h, Light.h, Scene.h,
Image.h) instead of the reference renderer.  Runs where /root/reference exists."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/RaytracingEngine"),
                    reason="needs the reference sources")
def test_reference_application_builds_on_dropin_api():
    from raytracingengine_amd import build
    build.build_cpp_api()
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_app_on_rtamd")
    if os.path.exists(exe):
        os.remove(exe)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "dropin"], check=True)
    syms = subprocess.run(["nm", "-C", "-u", exe], capture_output=True, text=True, check=True).stdout
    assert "Scene::RenderImage() const" in syms   # resolved by librtamd_cpp.so, not inlined CPU code
    libs = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
    assert "librtamd_cpp.so" in libs and "librtamd.so" in libs
