"""Write the committed golden fixtures under tests/golden/ (run in the dev container).

Each fixture is a small seeded synthetic FLAC stream. Its expected output is pinned two
independent ways before it is written: (1) the writer's source PCM (ground truth) and
(2) the oracle's decode; they must agree bit for bit. The manifest stores the SHA-256
of the expected sample bytes (zflac's output convention: container type, left-justified).
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import synth  # noqa: E402
from tests.util import PARITY_CONFIGS, expected_samples  # noqa: E402

FIXTURES = {
    "c2_mono16_fixed2_k4": dict(PARITY_CONFIGS["c2_mono16_fixed2_k4"], n_samples=4096 * 2 + 100, seed=11),
    "c3_ms16_lpc8": dict(PARITY_CONFIGS["c3_ms16_lpc8"], n_samples=4096 * 2, seed=12),
    "c4_24bit_lpc32_wasted": dict(PARITY_CONFIGS["c4_24bit_lpc32_wasted"], n_samples=4096 * 2, seed=13,
                                  escape_every=3),
    "mono8_lpc3": dict(PARITY_CONFIGS["mono8_lpc3"], n_samples=576 * 3 + 3, seed=14),
    "ch3_16": dict(PARITY_CONFIGS["ch3_16"], n_samples=2048 * 2 + 1, seed=15),
    "variable_blocking": dict(PARITY_CONFIGS["variable_blocking"], n_samples=8000, seed=16),
    "stereo12_ms_rice2": dict(PARITY_CONFIGS["stereo12_ms"], n_samples=1024 * 3, rice2=1, seed=17),
    "ls16_fixed_mix": dict(PARITY_CONFIGS["ls16_fixed_mix"], n_samples=1152 * 3 + 5, seed=18),
}


def main():
    gold = os.path.join(ROOT, "tests", "golden")
    manifest = {"generator": "synth/flacgen.cpp via tools/make_fixtures.py", "fixtures": []}
    for name, cfg in FIXTURES.items():
        st = synth.generate(**cfg)
        exp = expected_samples(st)
        r = oracle.decode(st.flac)
        assert r.error == "OK" and np.array_equal(r.samples, exp), name
        fn = f"{name}.flac"
        with open(os.path.join(gold, fn), "wb") as f:
            f.write(st.flac)
        manifest["fixtures"].append({"file": fn, "error": "OK", "n_samples": int(exp.size),
                                     "channels": cfg["channels"], "bps": cfg["bps"],
                                     "samples_sha256": hashlib.sha256(exp.tobytes()).hexdigest(),
                                     "config": {k: v for k, v in cfg.items()}})
    with open(os.path.join(gold, "fixtures.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(FIXTURES), "fixtures")


if __name__ == "__main__":
    main()
