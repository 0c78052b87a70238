"""halogen — MI355X-native drop-in for the Halogen path tracer's compute hot path.

The product path is libhalogen_hip.so (HIP megakernel for gfx950 + C-ABI, include/halogen_abi.h); this package
is its host-side mirror of the reference's C# API (HalogenRenderPass / HalogenSettings / RayTracingMesh ...).
"""
from . import abi
from .abi import Context, HalogenError, gpu_available
from .render_pass import Camera, HalogenRenderPass, HalogenSettings, make_params, clamp_settings
from .scene import HalogenMaterial, PackedScene, RayTracingMesh, RayTracingSphere, Scene
from .unity import Transform

__all__ = ["abi", "Context", "HalogenError", "gpu_available", "Camera", "HalogenRenderPass", "HalogenSettings",
           "make_params", "clamp_settings", "HalogenMaterial", "PackedScene", "RayTracingMesh", "RayTracingSphere",
           "Scene", "Transform"]
