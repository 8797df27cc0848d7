"""Extract the three known-answer streams of the reference's tests/basic.zig:4-95
(RFC 9639 Appendix D examples) into tests/golden/basic_kat.json.

Only DATA is extracted: the FLAC byte arrays and the expected PCM values. Run in the
development container (where /root/reference exists); the JSON it writes is committed.
"""
import json
import re
import sys

SRC = "/root/reference/tests/basic.zig"


def parse_int(tok):
    tok = tok.strip()
    m = re.match(r"@bitCast\(@as\(u16,\s*(0x[0-9a-fA-F]+|0b[01]+)\)\)", tok)
    if m:
        v = int(m.group(1), 0)
        return v - 0x10000 if v >= 0x8000 else v
    return int(tok, 0)


def main(out_path):
    text = open(SRC).read()
    tests = re.split(r'test "', text)[1:]
    kats = []
    for t in tests:
        name = t.split('"', 1)[0]
        arr = re.search(r"const Example = \[_\]u8\{(.*?)\};", t, re.S).group(1)
        data = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]{2}", arr)]
        ch = int(re.search(r"expectEqual\((\d+), r\.channels\)", t).group(1))
        kind = re.search(r"r\.samples\.(s8|s16|s32)", t).group(1)
        m = re.search(r"expectEqualSlices\(i(?:8|16|32), &\[_\]i(?:8|16|32)\{(.*?)\}, r\.samples", t, re.S)
        if m:
            body = re.sub(r"//[^\n]*", "", m.group(1))
            toks = []
            depth = 0
            cur = ""
            for chn in body:
                if chn == "(":
                    depth += 1
                elif chn == ")":
                    depth -= 1
                if chn == "," and depth == 0:
                    toks.append(cur)
                    cur = ""
                else:
                    cur += chn
            if cur.strip():
                toks.append(cur)
            expected = [parse_int(x) for x in toks if x.strip()]
        else:
            expected = [int(v) for v in re.findall(r"expectEqual\((-?\d+), r\.samples\.s\d+\[\d+\]\)", t)]
        kats.append({"name": name, "source": "tests/basic.zig", "flac_hex": bytes(data).hex(),
                     "channels": ch, "sample_kind": kind, "expected": expected})
    with open(out_path, "w") as f:
        json.dump({"origin": "Senryoku/zflac tests/basic.zig:4-95 (RFC 9639 Appendix D examples)",
                   "kats": kats}, f, indent=1)
    print(f"wrote {len(kats)} KATs to {out_path}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "tests/golden/basic_kat.json")
