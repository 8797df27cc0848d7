"""Placement probe: k_decode time of the bench shard vs. a device allocation made before
the batch's buffers (moves every buffer to other addresses). Usage (GPU box):
python tools/pad_probe.py [pad_mb ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import zflac_amd  # noqa: E402


def main():
    pads = [int(x) for x in sys.argv[1:]] or [0, 2, 6, 64]
    streams = bench.make_shard(0, 1, bench.STREAMS_PER_GPU)
    out = []
    for pad in pads:
        keep = torch.empty(max(1, pad) << 20, dtype=torch.uint8, device="cuda") if pad else None
        b = zflac_amd.Batch(streams, device=0, timing=True)
        for _ in range(3):
            b.run()
        d = []
        for _ in range(10):
            b.run()
            d.append(b.timings().decode_ms)
        b.close()
        del keep
        torch.cuda.empty_cache()
        out.append({"pad_mb": pad, "decode_ms": round(float(np.mean(d)), 4), "min": round(min(d), 4)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
