"""Build libzflac_hip.so in-tree (hipcc, gfx950). Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libzflac_hip.so")
SOURCES = [os.path.join(CSRC, f"decode_k{k}_{lay}{mix}.hip") for k in (1, 2, 0) for lay in ("stereo", "mono", "multi")
           for mix in ("", "_mix")]
SOURCES += [os.path.join(CSRC, n) for n in ("scan.hip", "md5.hip", "crc16.hip", "walk_wave.hip", "host.cpp")]
HEADERS = [os.path.join(CSRC, n) for n in ("common.h", "md5.hpp", "device_common.h", "decode.inc")]
DEPS = SOURCES + HEADERS + [os.path.join(ROOT, "include", "zflac_hip.h")]
ARCH = os.environ.get("ZFLAC_OFFLOAD_ARCH", "gfx950")
CFLAGS = ["-O3", "-std=c++20", "-fPIC", "-Wall", "-Wno-unused-function"]


def source_fingerprint(defines=()) -> str:
    """sha256 over the library's sources, headers, target, compile flags and -D defines. hipcc
    output is not bit-reproducible (each compile draws a new CUID), so this, not the .so's own
    hash, is what says that two builds hold the same kernels. Every build embeds it
    (zflac_hip_build_id() returns "src=<fingerprint>"), so a measurement names the kernels of
    the library it actually loaded."""
    import hashlib

    h = hashlib.sha256(f"{ARCH}|{' '.join(CFLAGS)}|{' '.join(sorted(defines))}".encode())
    for d in sorted(DEPS):
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def sources_present() -> bool:
    return all(os.path.exists(d) for d in DEPS)


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


def lib_build_id(path: str | None = None) -> str | None:
    """The build id ("src=<fingerprint>") embedded in a built library, read from the .so file
    without loading it (so it works without a GPU and for any ZFLAC_HIP_LIB variant)."""
    import re

    try:
        with open(path or LIB, "rb") as f:
            m = re.search(rb"src=([0-9a-f]{64})", f.read())
    except OSError:
        return None
    return m.group(0).decode() if m else None


def _obj_deps(src: str):
    """Headers a translation unit includes (decode.inc only for the decode units). host.cpp
    embeds the fingerprint of every source, so it depends on all of them."""
    if src.endswith("host.cpp"):
        return list(DEPS)
    hdrs = [h for h in HEADERS if not h.endswith("decode.inc") or "decode_k" in src]
    return [src] + hdrs + [os.path.join(ROOT, "include", "zflac_hip.h")]


def build(force: bool = False, verbose: bool = False, defines=(), out: str | None = None, units=None) -> str:
    """Build libzflac_hip.so (or, with `out`, a variant with extra -D `defines` for timing
    experiments: separate object directory, never the product library). `units`: basenames
    of the translation units the defines affect; the variant takes every other unit's object
    from the product build (built first), so a one-kernel experiment compiles one unit."""
    lib = out or LIB
    if not force and not defines and not out and not needs_build():
        return LIB
    if units:
        build()  # the product objects the variant shares
        units = set(units) | {"host.cpp"}  # host.cpp embeds the variant's fingerprint
    objs = []
    tag = "_".join(d.replace("=", "-") for d in defines)
    build_dir = os.path.join(HERE, "_build" + ("_" + tag if tag else ""))
    os.makedirs(build_dir, exist_ok=True)
    procs = []
    fp = source_fingerprint(defines)
    jobs = max(1, min(int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 1, 16))
    for src in SOURCES:  # translation units compile in parallel; up-to-date objects are kept
        if units and os.path.basename(src) not in units:
            objs.append(os.path.join(HERE, "_build", os.path.basename(src) + ".o"))
            continue
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d)
                                                                               for d in _obj_deps(src)):
            objs.append(obj)
            continue
        cmd = ["hipcc", f"--offload-arch={ARCH}"] + CFLAGS + ["-I", os.path.join(ROOT, "include"), "-c", src, "-o", obj]
        cmd[1:1] = [f"-D{d}" for d in defines]
        if src.endswith(".hip"):
            cmd[1:1] = ["-x", "hip"]
        if src.endswith("host.cpp"):
            cmd[1:1] = [f'-DZFLAC_BUILD_ID="src={fp}"']
        if verbose:
            print(" ".join(cmd))
        while sum(p.poll() is None for _, p in procs) >= jobs:  # bounded: each decode unit is GBs of RAM
            time.sleep(0.2)
        procs.append((src, subprocess.Popen(cmd)))
        objs.append(obj)
    failed = [src for src, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError(f"hipcc failed for {failed}")
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs
    subprocess.check_call(cmd)
    return lib


if __name__ == "__main__":
    # python -m zflac_amd.build [--force] [-DNAME ...] [-o out.so] [--units a.hip,b.hip]
    a = sys.argv[1:]
    out = a[a.index("-o") + 1] if "-o" in a else None
    units = a[a.index("--units") + 1].split(",") if "--units" in a else None
    build(force="--force" in a, verbose=True, defines=[x[2:] for x in a if x.startswith("-D")], out=out, units=units)
