"""Static instruction count of one kernel per source line (hipcc -g -save-temps
ISA with .loc directives).  Usage: python tools/isa_lines.py file.s kernel_symbol"""
import collections
import re
import sys


def main(path, sym):
    t = open(path).read().split("\n")
    files = {}
    for ln in t:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    s = [i for i, ln in enumerate(t) if ln.startswith(sym + ":")][0]
    cur = ("?", 0)
    cnt = collections.defaultdict(lambda: collections.Counter())
    for ln in t[s + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
        if m:
            cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        x = ln.strip()
        if not ln.startswith("\t") or not x or x.startswith((".", ";")):
            continue
        op = x.split()[0]
        kind = "v" if op.startswith("v_") else "s" if op.startswith("s_") else "m"
        cnt[cur][kind] += 1
    for (f, l), c in sorted(cnt.items()):
        print(f"{f}:{l} v={c['v']} s={c['s']} m={c['m']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
