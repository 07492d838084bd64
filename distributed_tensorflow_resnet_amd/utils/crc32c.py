"""CRC32C (Castagnoli) + TF/LevelDB masking.

Uses the native SSE4.2 implementation in ``_C`` when built, else a pure-Python
table (fine for tests and small records)."""
from __future__ import annotations

_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)

_MASK_DELTA = 0xA282EAD8


def _native():
    try:
        from .. import native

        return native(required=False)
    except Exception:  # pragma: no cover
        return None


def _py_extend(crc: int, data: bytes) -> int:
    c = crc ^ 0xFFFFFFFF
    t = _TABLE
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def extend(crc: int, data) -> int:
    mv = memoryview(data).cast("B")
    nat = _native()
    if nat is not None and hasattr(nat, "crc32c") and len(mv) > 64:
        return nat.crc32c(bytes(mv) if not isinstance(data, (bytes, bytearray)) else data, crc)
    return _py_extend(crc, bytes(mv))


def value(data) -> int:
    return extend(0, data)


def mask(crc: int) -> int:
    """LevelDB/TF masked CRC: rotate right by 15 and add a constant."""
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


def unmask(masked: int) -> int:
    rot = (masked - _MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF
