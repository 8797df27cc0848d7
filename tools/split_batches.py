"""Steps over the C5 shard decoded as S sub-batches per step (1250/S streams each), with
inflight*S sub-batches in flight, round robin: ms per step (whole shard) at K steps.
Usage: python tools/split_batches.py K S inflight [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
K, S, INF = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
REPS = int(sys.argv[4]) if len(sys.argv) > 4 else 3
os.environ.setdefault("ZFLAC_RUN_STREAMS", str(min(INF * S, 8)))
import synth  # noqa: E402
import zflac_amd  # noqa: E402

streams = [s.flac for s in synth.generate_many([synth.config_c5(i) for i in range(1250)])]
parts = [streams[i * len(streams) // S:(i + 1) * len(streams) // S] for i in range(S)]
bs = [zflac_amd.Batch(parts[i % S]) for i in range(INF * S)]


def run(k):
    n = k * S
    pend = [False] * len(bs)
    for i in range(n):
        j = i % len(bs)
        if pend[j]:
            bs[j].wait()
        bs[j].submit()
        pend[j] = True
    for j in range(len(bs)):
        if pend[j]:
            bs[j].wait()


run(3)
out = []
for _ in range(REPS):
    t0 = time.perf_counter()
    run(K)
    out.append(1000 * (time.perf_counter() - t0) / K)
print({"K": K, "S": S, "inflight_subbatches": INF * S, "ms_per_step": [round(x, 4) for x in out]})
