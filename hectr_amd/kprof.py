"""Live timing of the dominant kernel (filled in once profiled)."""


def dominant_kernel(eng, B, L, logn):
    return None
