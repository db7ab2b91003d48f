"""lz4.frame -- LZ4 frame format on the MI355X codec.

Reference: lz4/frame/__init__.py:1-98 (one-shot functions and constants).
The chunked / context streaming API (compress_begin, LZ4FrameCompressor,
LZ4FrameFile, ...) is outside this codec's scope.
"""
from ._frame import (  # noqa: F401
    compress,
    compress_device,
    decompress_device,
    decompress,
    get_frame_info,
    BLOCKSIZE_DEFAULT,
    BLOCKSIZE_MAX64KB,
    BLOCKSIZE_MAX256KB,
    BLOCKSIZE_MAX1MB,
    BLOCKSIZE_MAX4MB,
)

COMPRESSIONLEVEL_MIN = 0     # lz4/frame/__init__.py:74-98
COMPRESSIONLEVEL_MINHC = 3
COMPRESSIONLEVEL_MAX = 16
