"""Minimal stand-in for the mmcv API surface DFormer's hot path touches.

Test infrastructure only (oracle harness). Restates the published mmcv 1.x
semantics of ConvModule / build_norm_layer / DropPath so the read-only
reference can be imported on CPU to generate golden vectors.
"""
__version__ = "1.7.0"
