#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing, by basic block: the blocks with MFMAs
first. usage: asm_stats.py FILE.s SUBSTRING [--top N]"""
import collections
import re
import sys


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(sub), l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = [], collections.Counter(), "entry"
    ops_of = collections.defaultdict(collections.Counter)
    for l in lines[start + 1:end]:
        t = l.strip()
        if re.match(r"^\.LBB\S+:", t):
            blocks.append((name, cur))
            name, cur = t.split(":")[0], collections.Counter()
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        cur[classify(op)] += 1
        ops_of[name][op] += 1
    blocks.append((name, cur))
    tot = collections.Counter()
    for _, c in blocks:
        tot.update(c)
    print(lines[start].split(":")[0][:90])
    print("total", dict(tot))
    for name, c in sorted(blocks, key=lambda b: -b[1]["mfma"])[:top]:
        if not c["mfma"]:
            break
        v = c["valu"] / max(1, c["mfma"])
        print(f"{name:14s} mfma {c['mfma']:4d} valu {c['valu']:4d} ({v:.2f}/mfma) lds {c['lds']:3d} "
              f"salu {c['salu']:3d} wait {c['wait']:3d} vmem {c['vmem']:3d} barrier {c['barrier']}")
        if "-v" in sys.argv:
            print("   ", ", ".join(f"{k} {n}" for k, n in ops_of[name].most_common(14) if k.startswith("v_")))


if __name__ == "__main__":
    main()
