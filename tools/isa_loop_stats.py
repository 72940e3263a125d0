#!/usr/bin/env python3
"""tools/isa_loop_stats.py -- instruction mix of a kernel's outermost loop in a
device assembly file (hipcc --cuda-device-only -S): which blocks belong to the
loop is read from the compiler's "in Loop: Header=" block comments.

  python tools/isa_loop_stats.py k.s <kernel-symbol-substring> [--top N]
"""
import argparse
import collections
import re


def kernel_lines(path, sym):
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S*:", ln) and sym in ln.split(":")[0]:
            start = i
            break
    if start is None:
        raise SystemExit(f"no kernel matching {sym}")
    end = next((j for j in range(start + 1, len(lines)) if lines[j].startswith(".Lfunc_end")), len(lines))
    return lines[start:end], lines[end:end + 400]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("sym")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    body, tail = kernel_lines(a.asm, a.sym)
    # the outermost loop with the most instructions
    loops = collections.defaultdict(list)
    cur = None
    for ln in body:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", ln)
        if m:
            lab, c = m.groups()
            h = re.search(r"Header=BB(\d+_\d+) Depth=1", c)
            if "=>This Loop Header: Depth=1" in c:
                cur = lab[4:]
            elif h:
                cur = h.group(1)
            else:
                cur = None
            continue
        t = ln.strip()
        if cur and ln.startswith("\t") and t and not t.startswith((";", ".")):
            loops[cur].append(t.split()[0])
    hdr, ins = max(loops.items(), key=lambda kv: len(kv[1]))
    cat = collections.Counter()
    for i in ins:
        if i.startswith("s_waitcnt") or i.startswith("s_nop"):
            cat[i.split("_")[0] + "_" + i.split("_")[1]] += 1
        elif i.startswith("s_cbranch") or i.startswith("s_branch"):
            cat["branch"] += 1
        elif i.startswith(("s_load", "s_buffer")):
            cat["smem"] += 1
        elif i.startswith("s_"):
            cat["salu"] += 1
        elif i.startswith("ds_"):
            cat["lds"] += 1
        elif i.startswith(("buffer_", "global_", "flat_")):
            cat["vmem"] += 1
        elif i.startswith("v_"):
            cat["valu"] += 1
        else:
            cat["other"] += 1
    meta = {k: v for k, v in (re.findall(r"; (NumVgprs|NumSGPRsForWavesPerEU|ScratchSize|Occupancy): (\d+)",
                                         "\n".join(tail)))}
    print(f"loop BB{hdr}: {len(ins)} instrs; " + ", ".join(f"{k} {v}" for k, v in sorted(cat.items())) + f"; {meta}")
    for k, v in collections.Counter(ins).most_common(a.top):
        print(f"  {v:5d} {k}")


if __name__ == "__main__":
    main()
