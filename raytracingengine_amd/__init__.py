"""MI355X-native (gfx950) renderer with the per-pixel hot path of Sorax5/RaytracingEngine.

The product is ``librtamd.so`` (HIP kernels + the C-ABI of ``include/rt_capi.h``) and the C++20
drop-in headers under ``raytracingengine_amd/api``.  This Python package is plumbing for the
bench and the tests: scene data (:mod:`.scene`), synthetic configs (:mod:`.configs`), the ctypes
binding (:mod:`.capi`) and the multi-GPU row-tile driver (:mod:`.distributed`).
"""
from .scene import (AreaLight, Camera, Material, SceneData)  # noqa: F401
from .configs import make_config  # noqa: F401

__all__ = ["AreaLight", "Camera", "Material", "SceneData", "make_config"]
