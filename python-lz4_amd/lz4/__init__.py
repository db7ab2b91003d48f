"""MI355X-native LZ4 (drop-in for python-lz4's ``lz4`` package on its hot path).

``lz4.block`` and ``lz4.frame`` keep the reference API (lz4/__init__.py,
lz4/block/__init__.py, lz4/frame/__init__.py); the block codec and XXH32 run
as HIP kernels on the GPU.
"""
from ._version import version as __version__, library_version_number, library_version_string  # noqa: F401

VERSION = __version__
