"""The C-ABI library loads without a GPU and exports exactly what include/rt_capi.h declares.
No compute call is made here (CPU container)."""
import ctypes
import os
import re
import subprocess

import pytest

from raytracingengine_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt_capi.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from raytracingengine_amd import build
    build.build_library()
    return capi.load_library()


def test_header_and_binding_agree():
    assert declared_functions() == sorted(capi.EXPORTED)


def test_every_declared_symbol_is_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    for f in declared_functions():
        assert getattr(lib, f) is not None


def test_library_is_gfx950_only():
    """The fat binary carries gfx950 code objects and nothing else (no multi-arch dispatch)."""
    blob = open(capi.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[a-z-]*gfx[0-9a-z]+", blob))
    assert targets == {b"amdgcn-amd-amdhsa--gfx950"}, targets
    assert set(re.findall(rb"gfx[0-9]{3,4}[a-z]?", blob)) == {b"gfx950"}


def test_build_record_matches_tree(lib):
    """rt_build_info names the sources the binary was compiled from: a stale librtamd.so (sources
    edited after the build) shows as matches_tree False, here and in every bench line."""
    info = capi.build_info()
    assert info["arch"] == "gfx950"
    assert len(info["source_sha256"]) == 64
    assert info["matches_tree"], info


def test_defaults_match_reference(lib):
    o = capi.default_opts()
    assert o.max_recursion == 10      # Scene.h:24
    assert o.bias == 1e-3             # Scene.h:291
    assert o.tonemap == 6             # tonemap() is ACES, RaytracingEngine.cpp:165-174
    assert o.row_begin == 0 and o.row_end == 0


def test_no_device_fails_loudly_without_fallback(lib):
    if lib.rt_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(capi.RtError) as e:
        capi.Context(0)
    assert e.value.status == capi.RT_ERR_NO_DEVICE


def test_null_arguments_rejected(lib):
    assert lib.rt_context_create(0, None) == capi.RT_ERR_INVALID_ARG
    assert b"NULL" in lib.rt_last_error()
    assert lib.rt_scene_create(None, None, None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_render(None, None, None, None, None, None, None, None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_context_destroy(None) == capi.RT_OK
