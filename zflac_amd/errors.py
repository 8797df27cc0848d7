"""zflac's error set as Python exceptions.

Codes are those of include/zflac_hip.h; names are zflac's (src/zflac.zig).
"""
from __future__ import annotations

NAMES = {
    0: "OK", 1: "InvalidSignature", 2: "InvalidMetadataHeader", 3: "MissingStreaminfo", 4: "Unimplemented",
    5: "InvalidChecksum", 6: "InvalidFrameHeader", 7: "InconsistentParameters", 8: "InvalidCodedNumber",
    9: "InvalidSubframeHeader", 10: "InvalidResidualCodingMethod", 11: "EndOfStream", 12: "OutOfMemory",
    13: "DeviceError", 14: "InvalidArgument", 15: "OutOfDomain",
    16: "FrameCrcMismatch",  # only with the opt-in CRC-16 check (zflac ignores the trailer)
}


class ZflacError(Exception):
    """Base class; `code` is the C ABI error code, the class name zflac's error name."""

    code = -1


_BY_CODE: dict[int, type] = {}
for _code, _name in NAMES.items():
    if _code == 0:
        continue
    _cls = type(_name, (ZflacError,), {"code": _code, "__doc__": f"zflac error.{_name}"})
    globals()[_name] = _cls
    _BY_CODE[_code] = _cls


def error_class(code: int) -> type:
    return _BY_CODE.get(code, ZflacError)


def check(code: int, what: str = "") -> None:
    if code:
        cls = error_class(code)
        raise cls(f"{NAMES.get(code, code)}{': ' + what if what else ''}")
