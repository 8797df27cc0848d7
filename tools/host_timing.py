"""Host-side cost of the bench's submit / wait calls on the C5 shard (4 batches, round robin):
the time each call spends on the host thread, and the device-side run time, per run."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZFLAC_RUN_STREAMS", "4")
import synth  # noqa: E402
import zflac_amd  # noqa: E402

streams = [s.flac for s in synth.generate_many([synth.config_c5(i) for i in range(1250)])]
bs = [zflac_amd.Batch(streams, timing=True) for _ in range(4)]
for b in bs:
    b.run()
sub, wt, ready_wait = [], [], []
pend = [False] * 4
t_all = time.perf_counter()
for i in range(40):
    j = i % 4
    if pend[j]:
        t0 = time.perf_counter()
        while not bs[j].ready():
            pass
        t1 = time.perf_counter()
        bs[j].wait()
        t2 = time.perf_counter()
        ready_wait.append(t1 - t0)
        wt.append(t2 - t1)
    t0 = time.perf_counter()
    bs[j].submit()
    sub.append(time.perf_counter() - t0)
    pend[j] = True
for j in range(4):
    bs[j].wait()
el = time.perf_counter() - t_all
ms = lambda v: round(1000 * sum(v) / len(v), 4)
print({"runs": 40, "ms_per_run_wall": round(1000 * el / 40, 4), "submit_ms": ms(sub), "wait_after_ready_ms": ms(wt),
       "spin_until_ready_ms": ms(ready_wait)})
