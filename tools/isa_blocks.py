"""Basic blocks of one kernel in a device assembly listing (hipcc --cuda-device-only -S):
per block the instruction mix (VALU / SALU / LDS / VMEM / branches) and its successors, so
the blocks a chunk runs through can be read off and their VALU summed. ISA study only.

usage: python tools/isa_blocks.py <file.s> <kernel-substring> [--min-valu N] [--show BLOCK]"""
import re
import sys


def kernel_lines(path, sub):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and sub in l.split(":")[0]:
            start = i
        elif start is not None and (l.startswith(".Lfunc_end") or re.match(r"^_Z\S*:", l)):
            return lines[start:i]
    return lines[start:] if start is not None else []


def classify(op):
    if op.startswith(("v_readlane", "v_readfirstlane")):
        return "valu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc")):
        return "br"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_sched") or op.startswith("s_barrier"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def blocks(lines):
    out = []
    cur = {"name": "entry", "ins": [], "succ": [], "loop": None}
    for l in lines:
        s = l.split(";")[0].rstrip()
        m = re.match(r"^(\.LBB\S+):", s)
        mb = re.match(r"^; %bb\.(\d+):", l.strip())
        if mb:
            m = re.match(r"(.*)", "bb." + mb.group(1))
        elif m:
            m = re.match(r"(.*)", "bb." + m.group(1).split("_")[-1])
        if m:
            if cur["ins"] and not cur["ins"][-1].startswith(("s_branch", "s_setpc", "s_endpgm")):
                cur["succ"].append(m.group(1))
            out.append(cur)
            cur = {"name": m.group(1), "ins": [], "succ": [], "loop": None}
            lm = re.search(r"(?:Header=|Loop: Header=)BB\d+_(\d+) Depth=(\d+)", l)
            hm = re.search(r"This Loop Header: Depth=(\d+)", l)
            if lm:
                cur["loop"] = (int(lm.group(1)), int(lm.group(2)))
            pending_header = hm is not None
            continue
        if l.strip().startswith("; =>  This Loop Header: Depth=") and cur["loop"] is None:
            cur["loop"] = (int(cur["name"].split(".")[-1]), int(l.strip().split("=")[-1]))
        s = s.strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        cur["ins"].append(s)
        t = re.match(r"^(s_cbranch_\w+|s_branch)\s+(\.LBB\S+)", s)
        if t:
            cur["succ"].append("bb." + t.group(2).split("_")[-1])
    out.append(cur)
    return out


def main():
    a = sys.argv[1:]
    path, sub = a[0], a[1]
    minv = int(a[a.index("--min-valu") + 1]) if "--min-valu" in a else 0
    show = a[a.index("--show") + 1] if "--show" in a else None
    bl = blocks(kernel_lines(path, sub))
    tot = {}
    for b in bl:
        c = {}
        for i in b["ins"]:
            k = classify(i.split()[0])
            c[k] = c.get(k, 0) + 1
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        b["c"] = c
        if show and b["name"] == show:
            print("\n".join(b["ins"]))
        rl = sum(1 for i in b["ins"] if i.startswith("v_readlane"))
        if not show and c.get("valu", 0) >= minv:
            lp = f"L{b['loop'][0]}/{b['loop'][1]}" if b.get("loop") else "-"
            print(f"{b['name']:>14} {lp:>9} n={len(b['ins']):5d} valu={c.get('valu', 0):4d} rl={rl:2d} salu={c.get('salu', 0):3d} "
                  f"lds={c.get('lds', 0):3d} vmem={c.get('vmem', 0):3d} wait={c.get('wait', 0):3d} -> {' '.join(b['succ'])}")
    if not show:
        print("total", tot, "blocks", len(bl))


if __name__ == "__main__":
    main()
