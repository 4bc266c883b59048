"""MAT architecture variants (filled in: mat_encoder / mat_decoder / mat_gru)."""


def build_variant(name, *a, **k):
    raise NotImplementedError(f"variant {name}")
