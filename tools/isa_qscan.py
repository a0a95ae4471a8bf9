"""Static VALU count of adc_qscan_kernel's main loop (one wave-step: 64 rows x 16 queries) in the
built libmivq.so, split by encoding size (32-bit VOP1/VOP2/VOPC vs 64-bit VOP3/VOP3P/literal forms:
the VALU-rate probe, tools/probes/valu_rate.hip, measured them at different issue rates).

bench.py's ADC roofline quotes the scan's VALU issue rate from these counts
(QSCAN_VALU_PER_STEP); tests/test_abi.py checks that they match the built library.

usage: python tools/isa_qscan.py [path/to/libmivq.so]
"""
from __future__ import annotations

import json
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import isa_audit  # noqa: E402

LINE = re.compile(r"^\s+([a-z_0-9]+)(.*?)//\s*([0-9A-F]+):((?:\s[0-9A-F]{8})+)\s*(?:<[^>]*>)?\s*$")


def kernel_lines(txt: str, needle: str):
    """(mnemonic, operands, address, encoding dwords) of the first kernel whose symbol holds needle."""
    out, on = [], False
    for line in txt.splitlines():
        if line.endswith(">:") and "<" in line:
            if on:
                break
            on = needle in line
            continue
        if on:
            m = LINE.match(line)
            if m:
                out.append((m.group(1), m.group(2).strip(), int(m.group(3), 16), len(m.group(4).split())))
    return out


def main_loop(ins):
    """The backward branch whose body holds the most ds_read_b128 (the scan's row loop)."""
    best = None
    for i, (mn, ops, addr, nw) in enumerate(ins):
        if not mn.startswith("s_cbranch"):
            continue
        off = int(ops.split()[0])
        off = off - 65536 if off >= 32768 else off
        tgt = addr + 4 + 4 * off
        if tgt >= addr:
            continue
        body = [x for x in ins if tgt <= x[2] <= addr]
        nds = sum(1 for x in body if x[0] == "ds_read_b128")
        if best is None or nds > best[0]:
            best = (nds, body)
    return best[1] if best else []


def count(lib: Path) -> dict:
    txt = isa_audit.disassemble(lib)
    res = {}
    # the variants the product runs: M = 16 unpinned (the pinned one has the same count), M = 32
    # pinned (launch_qscan always takes it at M = 32, with the buffer-loaded code rows)
    for mc, m, pin in ((1, 16, 0), (2, 32, 1)):
        body = main_loop(kernel_lines(txt, f"adc_qscan_kernelILi{mc}ELb{pin}E"))
        valu = [x for x in body if x[0].startswith("v_")]
        res[str(m)] = {"valu": len(valu), "valu_32bit": sum(1 for x in valu if x[3] == 1),
                       "valu_64bit": sum(1 for x in valu if x[3] >= 2),
                       "ds_read_b128": sum(1 for x in body if x[0] == "ds_read_b128")}
    return res


if __name__ == "__main__":
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else isa_audit.ROOT / "vector-quantization_amd" / "lib" / "libmivq.so"
    print(json.dumps(count(lib)))
