"""Exposed memory round trips in a kernel's prologue, from the device assembly (hipcc -S --cuda-device-only):
for every kernel, the vector-memory wait instructions that drain the whole queue (s_waitcnt vmcnt(0)) before the
first workgroup barrier, and how many global loads are issued AFTER the first of them (each such drain makes the
loads behind it a second dependent round trip). Usage: python tools/isa_waits.py file.s [name-filter ...]"""
import re
import sys


def main():
    src = open(sys.argv[1]).read()
    filt = sys.argv[2:]
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):\s*;", src, re.M)]
    for k, (pos, name) in enumerate(starts):
        if filt and not any(f in name for f in filt):
            continue
        body = src[pos:starts[k + 1][0] if k + 1 < len(starts) else len(src)]
        body = body[:body.find("s_endpgm")] if "s_endpgm" in body else body
        lines = body.split("\n")
        fb = next((i for i, l in enumerate(lines) if "s_barrier" in l), len(lines))
        pre = lines[:fb]
        loads = [i for i, l in enumerate(pre) if re.search(r"\b(global|buffer)_load", l)]
        w0 = [i for i, l in enumerate(pre) if "s_waitcnt vmcnt(0)" in l]
        after = sum(1 for i in loads if w0 and i > w0[0])
        print(f"{name[:78]:78s} loads {len(loads):3d}  drains {len(w0):2d}  loads behind first drain {after:3d}")


if __name__ == "__main__":
    main()
