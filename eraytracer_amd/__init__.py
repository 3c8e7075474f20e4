"""eraytracer_amd — MI355X-native drop-in for the per-pixel render path of plouj/eraytracer.

The product is ``librtmi355x.so`` (C ABI: include/rt_mi355x.h; HIP kernel:
csrc/rt_render.hip).  This package is the host side: scene records and Erlang term
text (records, terms, scenes), the ctypes binding and scene marshalling (_native), the
reference-shaped strategy functions (raytracer) and the multi-GPU row sharding with an
RCCL gather (dist).
"""
from .records import scene  # noqa: F401
from .raytracer import (  # noqa: F401
    go, raytrace, raytraced_pixel_list_concurrent, raytraced_pixel_list_distributed, raytraced_pixel_list_gpu,
    raytraced_pixel_list_simple, render, standalone, tracing_function, write_pixels_to_ppm,
)

__all__ = [
    "scene", "render", "raytraced_pixel_list_simple", "raytraced_pixel_list_concurrent",
    "raytraced_pixel_list_distributed", "raytraced_pixel_list_gpu", "tracing_function", "raytrace", "go",
    "standalone", "write_pixels_to_ppm",
]
