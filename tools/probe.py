"""Timing-probe run (experimental build with -DZFLAC_PROBE, tools/_build/lib_probe.so):
cycles per chunk phase of k_walk and k_decode, summed over waves, for the C5 shard or one
tiled stream of a BASELINE config (c2 / c3 / c4, 65,536 frames).
Usage: ZFLAC_HIP_LIB=tools/_build/lib_probe.so python tools/probe.py [streams | c2 | c3 | c4]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import synth  # noqa: E402
import zflac_amd  # noqa: E402
from zflac_amd import _lib  # noqa: E402

arg = sys.argv[1] if len(sys.argv) > 1 else "1250"
if arg.isdigit():
    n = int(arg)
    streams = [s.flac for s in synth.generate_many([synth.config_c5(i) for i in range(n)])]
elif arg.startswith("row:"):  # a row of tools/bench_configs.py (substring of its name)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs  # noqa: E402

    name = next(k for k in bench_configs.ROWS if arg[4:] in k)
    cfg, seg, frames, _ = bench_configs.ROWS[name]
    st = synth.generate(**dict(cfg, n_samples=4096 * seg, seed=cfg.get("seed", 7)))
    streams = [synth.tile_flac(st, max(1, frames // seg))]
    n = name
else:
    cfg = {"c2": synth.config_c2, "c3": synth.config_c3, "c4": synth.config_c4}[arg]()
    seg = 512
    st = synth.generate(**dict(cfg, n_samples=4096 * seg, seed=cfg.get("seed", 7)))
    streams = [synth.tile_flac(st, 65536 // seg)]
    n = arg
b = zflac_amd.Batch(streams, timing=True)
L = _lib.load()
fn = L.zflac_hip_probe
fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
b.run()
fn(b._h, buf, 16)  # discard the warm-up run
b.run()
fn(b._h, buf, 16)
t = b.timings()
names = ["topup", "fast", "slow", "chunks", "fast_chunks", "redos", "pair_chunks", "pair_redos"]
out = {"streams": n, "walk_ms": t.walk_ms, "decode_ms": t.decode_ms}
for k, base in (("walk", 0), ("decode", 8)):
    v = [buf[base + i] for i in range(8)]
    ch = max(1, v[3])
    out[k] = {names[i]: v[i] for i in range(8)}
    out[k]["cycles_per_chunk"] = {names[i]: round(v[i] / ch, 1) for i in range(3)}
print(json.dumps(out, indent=1))
