"""Is the first timed stretch after a warm-up slower, and why? C5 shard, 4 batches in flight,
round robin: ms per step of consecutive 20-step stretches after W warm-up runs, with an idle
gap (sleep, device synchronized) of G ms before each stretch.
Usage: python tools/warm_test.py W G reps"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
W, G, REPS = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
os.environ.setdefault("ZFLAC_RUN_STREAMS", "4")
import synth  # noqa: E402
import zflac_amd  # noqa: E402

streams = [s.flac for s in synth.generate_many([synth.config_c5(i) for i in range(1250)])]
bs = [zflac_amd.Batch(streams) for _ in range(4)]


def run(k):
    pend = [False] * 4
    for i in range(k):
        j = i % 4
        if pend[j]:
            bs[j].wait()
        bs[j].submit()
        pend[j] = True
    for j in range(4):
        if pend[j]:
            bs[j].wait()


run(W)
out = []
for _ in range(REPS):
    time.sleep(G / 1000)
    t0 = time.perf_counter()
    run(20)
    out.append(round(1000 * (time.perf_counter() - t0) / 20, 4))
print({"warmup": W, "gap_ms": G, "ms_per_step": out})
