"""lz4.block -- LZ4 block format on the MI355X codec (reference: lz4/block/__init__.py:1)."""
from ._block import compress, decompress, LZ4BlockError  # noqa: F401
from ._block import (  # noqa: F401  batched / device-resident extensions
    compress_many,
    decompress_many,
    compress_batch,
    decompress_batch,
    decompress_host,
    compact,
    xxh32_batch,
    HC_LEVEL_MIN,
    HC_LEVEL_DEFAULT,
    HC_LEVEL_OPT_MIN,
    HC_LEVEL_MAX,
)
