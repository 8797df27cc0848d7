"""Slice the reference's expected-output files into small committed fixtures.

/root/reference/tests/expected_samples/*.raw hold the PCM zflac must produce for the
ietf-wg-cellar subset files (tests/std_subset.zig:16-33: i16 / i32 little-endian in zflac's
left-justified convention, 8-bit as unsigned bytes). The FLAC inputs are absent from the
reference snapshot, so these files pin the OUTPUT convention (left-justify amounts, 8-bit
sign convention) and give real audio content to re-encode: tests/test_raw_convention.py
encodes each slice with the repository's writer and decodes it with the oracle and the HIP
path, which must reproduce the slice byte for byte.

The channel count and bit depth of each file are not stored in the .raw files; they are
inferred from the file names and sizes and from the trailing-zero count of the values
(12-bit -> multiples of 16, 20-bit -> 4096, 24-bit -> 256), and recorded in the manifest.
This is data extraction (a fixture is data), run here where /root/reference exists.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

SRC = "/root/reference/tests/expected_samples"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "raw")

# file stem, channels, bits per sample, container ("s8u" = unsigned bytes, "s16", "s32")
FILES = [
    ("01 - blocksize 4096", 2, 16, "s16"),
    ("14 - wasted bits", 2, 16, "s16"),
    ("16 - partition order 8 containing escaped partitions", 2, 16, "s16"),
    ("22 - 12 bit per sample", 2, 12, "s16"),
    ("23 - 8 bit per sample", 2, 8, "s8u"),
    ("38 - 3 channels (3.0)", 3, 16, "s16"),
    ("60 - mono audio", 1, 16, "s16"),
    ("61 - predictor overflow check, 16-bit", 1, 16, "s16"),
    ("62 - predictor overflow check, 20-bit", 1, 20, "s32"),
    ("63 - predictor overflow check, 24-bit", 1, 24, "s32"),
]
FRAMES_PER_SLICE = 12288  # samples per channel kept from each file


def main():
    os.makedirs(DST, exist_ok=True)
    manifest = []
    for stem, ch, bps, kind in FILES:
        raw = open(os.path.join(SRC, stem + ".raw"), "rb").read()
        dt = {"s8u": np.uint8, "s16": np.dtype("<i2"), "s32": np.dtype("<i4")}[kind]
        v = np.frombuffer(raw, dt)
        assert v.size % ch == 0, stem
        n = v.size // ch
        start = (n // 3) * ch  # a slice from a third of the way in (past any fade-in)
        sl = v[start:start + FRAMES_PER_SLICE * ch]
        name = stem.split(" - ")[0] + ".raw"
        open(os.path.join(DST, name), "wb").write(sl.tobytes())
        nz = sl[sl != 0].astype(np.int64) if kind != "s8u" else None
        tz = None
        if nz is not None and nz.size:
            tz = int(min((int(x) & -int(x)).bit_length() - 1 for x in nz))
        manifest.append({"file": name, "source": stem + ".raw", "channels": ch, "bps": bps, "container": kind,
                         "offset_samples": int(start), "n_values": int(sl.size), "trailing_zeros": tz,
                         "sha256": hashlib.sha256(sl.tobytes()).hexdigest()})
    with open(os.path.join(DST, "manifest.json"), "w") as f:
        json.dump({"generator": "tools/make_raw_fixtures.py", "source": "reference tests/expected_samples",
                   "slices": manifest}, f, indent=1)


if __name__ == "__main__":
    main()
