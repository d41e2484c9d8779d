#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing (total, and inside the hottest loop).

    python scripts/isa_mix.py file.s <kernel-substring> [top]"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    key = sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    m = re.search(r"^(\S*" + re.escape(key) + r"\S*):", s, re.M)
    if not m:
        sys.exit("kernel not found")
    i = m.start()
    j = s.find(".Lfunc_end", i)
    body = s[i:j].split("\n")
    c = collections.Counter()
    blocks, cur = {}, None
    for line in body:
        t = line.strip()
        if re.match(r"^\.LBB\S+:", t):
            cur = t[:-1]
            blocks[cur] = collections.Counter()
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c[op] += 1
        if cur:
            blocks[cur][op] += 1
    print(f"total {sum(c.values())} instructions")
    for k, v in c.most_common(top):
        print(f"{v:6d} {k}")
    big = sorted(blocks.items(), key=lambda kv: -sum(kv[1].values()))[:3]
    for name, bc in big:
        print(f"block {name}: {sum(bc.values())} instr, mfma {sum(v for k, v in bc.items() if 'mfma' in k)}, "
              f"valu {sum(v for k, v in bc.items() if k.startswith('v_') and 'mfma' not in k)}, "
              f"ds {sum(v for k, v in bc.items() if k.startswith('ds_'))}, "
              f"global {sum(v for k, v in bc.items() if k.startswith(('global_', 'buffer_')))}")


if __name__ == "__main__":
    main()
