"""List the s_waitcnt vmcnt waits of a kernel's loops, with the loads they follow.

usage: python tools/isa_waits.py FILE.s KERNEL_SUBSTRING [-v]

FILE.s from `hipcc --cuda-device-only -S`.  For every basic block inside a loop, prints the
vmcnt waits and the count of VMEM loads issued since the loop header, so a vmcnt(0) that
also waits for loads meant to stay in flight across iterations (the refill of the next x
block) shows up directly.
"""

import re
import sys


def kernel_body(text: str, sub: str):
    names = [n for n in re.findall(r"^(\S+):\s*(?:;.*)?$", text, re.M) if sub in n and not n.startswith(".")]
    if not names:
        raise SystemExit(f"no kernel matching {sub!r}")
    name = names[0]
    i = text.index(name + ":")
    j = text.index(".Lfunc_end", i)
    return name, text[i:j].split("\n")


def main(argv):
    path, sub = argv[1], argv[2]
    verbose = "-v" in argv
    name, body = kernel_body(open(path).read(), sub)
    print(name)
    in_loop = False
    loads = 0
    for k, line in enumerate(body):
        s = line.strip()
        if s.startswith(".LBB") and "Loop Header" in s:
            in_loop, loads = True, 0
            print(f"{k:5d} {s}")
            continue
        if s.startswith(".LBB") and "in Loop" not in s and "Loop Header" not in s:
            in_loop = False
        if not in_loop:
            continue
        if re.match(r"(buffer|global)_load", s):
            loads += 1
            if verbose:
                print(f"{k:5d}   {s[:90]}")
        elif "vmcnt" in s:
            print(f"{k:5d}   {s:28s} after {loads} loads in this iteration")


if __name__ == "__main__":
    main(sys.argv)
