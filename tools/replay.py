"""Device throughput of pipeline parts without the host (diagnostic build with -DZFLAC_REPLAY,
tools/_build/lib_replay.so): after one normal run of each of `inflight` batches of the C5
shard, re-enqueue walk / decode / walk + decode / whole runs back to back on the batches' run
streams and report ms per run for each. Usage:
ZFLAC_HIP_LIB=tools/_build/lib_replay.so python tools/replay.py [inflight] [reps]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
os.environ.setdefault("ZFLAC_RUN_STREAMS", str(nb))
import synth  # noqa: E402
import zflac_amd  # noqa: E402
from zflac_amd import _lib  # noqa: E402

streams = [s.flac for s in synth.generate_many([synth.config_c5(i) for i in range(1250)])]
bs = [zflac_amd.Batch(streams) for _ in range(nb)]
if not os.environ.get("REPLAY_NORUN"):  # (scan-ablation variants: front parts only, no real run)
    for b in bs:
        b.run()
L = _lib.load()
fn = L.zflac_hip_replay
fn.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
               ctypes.POINTER(ctypes.c_double)]
arr = (ctypes.c_void_p * nb)(*[b._h.value if hasattr(b._h, "value") else b._h for b in bs])
out = {"inflight": nb, "reps": reps}
parts = ((1, "walk"), (2, "decode"), (3, "walk+decode"), (4, "run"), (8, "scan"), (16, "front"))
only = os.environ.get("REPLAY_PARTS")  # e.g. "scan,front3"
for what, name in parts:
    if only and name not in only.split(","):
        continue
    ms = ctypes.c_double()
    fn(arr, nb, 2, what, ctypes.byref(ms))  # warm
    rc = fn(arr, nb, reps, what, ctypes.byref(ms))
    out[name] = {"rc": rc, "ms_per_run": round(ms.value / (reps * nb), 4)}
    # one batch alone (serial)
    rc = fn(arr, 1, reps, what, ctypes.byref(ms))
    out[name + "_serial"] = round(ms.value / reps, 4)
print(json.dumps(out))
