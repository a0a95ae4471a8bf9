"""`vq-benchmark` command line — /root/reference/src/haag_vq/cli.py:1-21.

Registers the commands on the hot path: ``sweep``, ``streaming-sweep``, ``precompute-gt``
(exact ground truth on the GPU) and ``ivf-bench`` (the flat PQ / OPQ / SQ, IVF-PQ and
RaBitQ method runners).  Upstream's ``run`` / ``plot`` commands (report drivers and plots) are
out of scope of the MI355X build.  Entry points: the ``vq-benchmark``
console script of vector-quantization_amd/pyproject.toml, or ``python -m haag_vq``.
"""

import typer

from .benchmarks.ivf_benchmark import ivf_benchmark
from .benchmarks.precompute_ground_truth import precompute_ground_truth
from .benchmarks.streaming_sweep import streaming_sweep
from .benchmarks.sweep import sweep

app = typer.Typer(add_completion=False)
app.command(name="sweep")(sweep)
app.command(name="streaming-sweep")(streaming_sweep)
app.command(name="precompute-gt")(precompute_ground_truth)
app.command(name="ivf-bench")(ivf_benchmark)


def main():
    app()


if __name__ == "__main__":
    main()
