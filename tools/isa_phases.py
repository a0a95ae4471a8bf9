"""Static VALU breakdown of a kernel's main loop by phase (opcode family).

usage: python tools/isa_phases.py FILE.s KERNEL_SUBSTRING

Counts the VALU instructions of the innermost loop that holds the kernel's MFMAs (the
filter's per-block step), grouped by what they do.  Conditional blocks (pair / full-item
appends, exec-masked stores) are counted once, as if every step took them, so the total is
an upper bound per step; `SQ_INSTS_VALU / (blocks x subspaces)` is the measured mean.
"""

import re
import sys
from collections import Counter, OrderedDict

PHASES = OrderedDict([
    ("stage: scale + cvt to f16", re.compile(r"^v_(pk_mul_f32|mul_f32|cvt_pk_f16_f32|cvt_f16_f32)")),
    ("row norm (dot2)", re.compile(r"^v_dot2")),
    ("rank: pack index", re.compile(r"^v_(and_or_b32|bfi_b32|or3_b32)")),
    ("rank: top-2 / merge (max, min, med3)", re.compile(r"^v_(max_f32|min_f32|med3_f32|max3_f32|min3_f32)")),
    ("lane-pair exchange", re.compile(r"^v_(permlane|mov_b32_dpp|readlane|writelane)")),
    ("window / classify (cmp, cndmask, fma, sqrt)", re.compile(r"^v_(cmp|cndmask|fma|fmac|fmamk|fmaak|sqrt|mul_f32|add_f32|sub_f32|addc|sub_co|add_co)")),
    ("accumulator init / moves", re.compile(r"^v_(mov_b32|mov_b64|accvgpr)")),
    ("addresses / integer", re.compile(r"^v_(lshl|lshr|ashr|add_u32|sub_u32|mad_u32|mad_u64|and_b32|or_b32|xor_b32|bcnt|mbcnt|xad|add3|lshl_add|lshl_or|bfe|alignbit)")),
])


def main(argv):
    path, sub = argv[1], argv[2]
    text = open(path).read()
    names = [n for n in re.findall(r"^(\S+):\s*(?:;.*)?$", text, re.M) if sub in n and not n.startswith(".")]
    name = names[0]
    i = text.index(name + ":")
    body = text[i:text.index(".Lfunc_end", i)].split("\n")
    # loops: from a header to the last line that says "in Loop: Header=<it>"
    headers = [(k, re.search(r"(\.LBB\d+_\d+)", l).group(1)) for k, l in enumerate(body) if "Loop Header" in l]
    best = None
    for k, lab in headers:
        tag = "Header=" + lab[1:].replace("LBB", "BB")
        ends = [j for j, l in enumerate(body) if tag in l]
        end = max(ends) if ends else k
        # the loop body runs to the next block label after its last member
        j = end + 1
        while j < len(body) and not body[j].startswith(".LBB"):
            j += 1
        seg = body[k:j]
        nm = sum(1 for l in seg if "v_mfma" in l)
        if best is None or nm > best[0]:
            best = (nm, k, j, seg)
    nm, k0, k1, seg = best
    ops = [l.strip().split()[0] for l in seg if l.strip().startswith("v_") and "v_mfma" not in l]
    c = Counter()
    other = Counter()
    for op in ops:
        for ph, rx in PHASES.items():
            if rx.match(op):
                c[ph] += 1
                break
        else:
            other[op] += 1
    print(f"{name}\nloop lines {k0}..{k1}: {nm} MFMAs, {len(ops)} VALU (static, every branch once)")
    for ph in PHASES:
        print(f"  {c[ph]:5d}  {ph}")
    print(f"  {sum(other.values()):5d}  other: {', '.join(f'{o} x{n}' for o, n in other.most_common(8))}")


if __name__ == "__main__":
    main(sys.argv)
