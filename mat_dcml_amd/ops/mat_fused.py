"""Fused HIP MAT kernels (placeholder)."""


def supports(model):
    return False
