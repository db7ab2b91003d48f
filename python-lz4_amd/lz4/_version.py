"""Version information (reference: lz4/__init__.py:13-17, lz4/_version.c:38-48)."""

version = "4.4.4+mi355x"


def library_version_number() -> int:
    """Version number of the LZ4 format implementation (LZ4_versionNumber):
    the codec is bit-compatible with lz4 v1.9.4."""
    from . import _native
    return int(_native.lib().lz4m_version_number())


def library_version_string() -> str:
    from . import _native
    return _native.lib().lz4m_version_string().decode()
