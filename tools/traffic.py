"""Write profiles/traffic.json: HBM bytes per launch of each benched kernel group, from a
tools/pmc_traffic.sh run, stamped with the kernel-source hash of the tree that was profiled
(bench.py refuses an entry whose hash differs from the running tree's).

usage: python tools/traffic.py gpurun_out/pmc_traffic [last_n]
Per dispatch: FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half the bytes of a wide coalesced
read, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, both in KiB; the mean over the last_n
dispatches of each kernel, summed over the kernels of a workload.
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT / "tools"))
from pmc_select import select  # noqa: E402

# workload -> kernel-name substrings (template arguments select the shape)
WORKLOADS = {
    "pq16_encode_1000000x1536_gaussian": ["pq_encode_cs_kernelILi6ELi3ELi96", "pq_resolve_merged_kernelILi6ELi96",
                                          "pq_transpose_codes16_kernel<16>"],
    # the sweep's PQ8 shape (dsub 192): filter + resolve (its transpose kernel, <0>, is shared
    # with the OPQ32 encode that runs after it, so its last dispatches are not this leg's)
    "pq8_encode_1000000x1536": ["pq_encode_cs_kernelILi12ELi3ELi192", "pq_resolve_merged_kernelILi12ELi192"],
    "opq32_rotate_1000000x1536": ["opq_row_scale_kernel", "opq_split_gemm_kernel"],
    "sq8_encode_1000000x3072": ["sq_encode_f32_vec_kernel"],
    "rabitq1_encode_1000000x3072": ["rabitq_encode_wide_kernel"],  # d % 512 == 0 (rabitq.hip)
}


def per_launch(root, sub, last_n):
    """Mean HBM bytes of the selected dispatches (tools/pmc_select.py: the kernel's largest grid,
    last_n of each pass; refuses a selection that mixes grid sizes) and that grid size."""
    vals, _, grid = select(root, sub, last_n)
    if not vals.get("FETCH_SIZE"):
        return None, None
    fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write = sum(vals["WRITE_SIZE"]) / max(1, len(vals["WRITE_SIZE"]))
    return fetch * 1024 * 2 + write * 1024, grid


def main():
    from haag_vq import _native

    root = sys.argv[1]
    last_n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    out_path = ROOT / "profiles" / "traffic.json"
    data = {}
    for w, kernels in WORKLOADS.items():
        sel = {k: per_launch(root, k, last_n) for k in kernels}
        parts = {k: v[0] for k, v in sel.items()}
        if all(v is None for v in parts.values()):
            continue
        data[w] = {"bytes_per_launch": sum(v for v in parts.values() if v), "per_kernel": parts,
                   "grid_sizes": {k: v[1] for k, v in sel.items()},
                   "kernel_source_hash": _native.kernel_source_hash(),
                   "source": f"{root}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH x2 "
                             f"(gfx950 correction), mean of the last {last_n} dispatches per kernel "
                             f"among those with its largest grid (tools/pmc_select.py)"}
    out_path.write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(data, indent=1))


if __name__ == "__main__":
    main()
