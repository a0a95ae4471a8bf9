"""Search-index benchmark driver on the GPU (reference run_benchmarks.py:273-415): compare mode
over every method of the build on the synthetic set, the CSV, and sweep mode for pq_flat."""
import pandas as pd
import pytest

from haag_vq.benchmarks import run_benchmarks as rb


@pytest.mark.gpu
def test_run_benchmarks_compare_and_sweep(dev, tmp_path):
    df = rb.main(["--dataset", "synthetic", "--methods", "pq_flat,opq_flat,sq_flat,faiss_ivfpq,rabitq,pq_ivf",
                  "--bpd", "4", "--K", "32", "--nprobe", "8", "--output", str(tmp_path / "r.csv")])
    assert list(df["method"]) == ["pq_flat", "opq_flat", "sq_flat", "faiss_ivfpq", "rabitq"]
    assert ((df["recall_at_k"] >= 0) & (df["recall_at_k"] <= 1) & (df["qps"] > 0)).all()
    assert (df["N"] == 2000).all() and (df["D"] == 64).all()
    by = df.set_index("method")
    assert by.loc["sq_flat", "recall_at_k"] > 0.5 and by.loc["pq_flat", "recall_at_k"] > 0.3
    saved = list(tmp_path.glob("r_*.csv"))
    assert len(saved) == 1 and list(pd.read_csv(saved[0])["method"]) == list(df["method"])
    sw = rb.main(["--dataset", "synthetic", "--methods", "pq_flat", "--sweep-bpd", "2,4"])
    assert list(sw["bpd"]) == [2.0, 4.0]
    assert sw["recall_at_k"].iloc[1] >= sw["recall_at_k"].iloc[0] - 0.05
    assert sw["compression_ratio"].iloc[0] > sw["compression_ratio"].iloc[1]
