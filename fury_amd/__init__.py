"""fury_amd — MI355X-native Fury row-format codec (java/fury-format's hot path on gfx950).

Public surface mirrors the reference's Java API (org.apache.fury.format.encoder.Encoders /
RowEncoder, org.apache.fury.format.vectorized.ArrowWriter); the compute runs in hand-written
HIP kernels behind the C ABI in include/fury_row.h (libfury_row.so, built in-tree).
"""
from . import types  # noqa: F401

__all__ = ["types"]
