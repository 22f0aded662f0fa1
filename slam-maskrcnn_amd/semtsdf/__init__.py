"""semtsdf — MI355X-native semantic TSDF fusion (integrate + association + raycast).

Python host over the C ABI of libsemtsdf.so (include/semtsdf.h).  The compute runs in
hand-written HIP kernels for gfx950; this package only marshals arguments and mirrors the
reference's host interfaces (src/TSDF_Python/tsdf.py, src/SfM_CUDA/tsdf.cuh,
configuration.h, tsdf_cuda.tsdf_update).
"""
from . import _lib
from ._lib import PLACE_PYTHON, PLACE_SFM, RAY_ASSOC, RENDER_COLOR, RENDER_LABEL, SemTSDFError, load
from .config import Configuration, FusionConfig
from .export import export_surface, read_ply, write_ply
from .tsdf import TSDF
from .volume import DeviceBuffer, Volume, default_params, orbit_camera, place_from_frame

__all__ = ["TSDF", "Volume", "DeviceBuffer", "Configuration", "FusionConfig", "SemTSDFError", "load",
           "default_params", "place_from_frame", "orbit_camera", "_lib", "export_surface", "write_ply", "read_ply",
           "RENDER_LABEL", "RENDER_COLOR", "RAY_ASSOC", "PLACE_SFM", "PLACE_PYTHON"]
