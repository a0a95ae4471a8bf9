"""SQLite run log with the reference's schema.

Same table and columns as /root/reference/src/haag_vq/utils/run_logger.py:10-125
(``runs(id, timestamp, git_branch, git_commit, package_version, method, dataset,
cli_command, metrics_json, config_json, sweep_id)``), so the reference's ``vq-benchmark
plot`` can read rows written here.  Device facts (arch, GPU count) go into
``config_json``.
"""

from __future__ import annotations

import json
import os
import shlex
import sqlite3
import subprocess
import sys
from datetime import datetime, timezone

import numpy as np


def _native(obj):
    if isinstance(obj, dict):
        return {k: _native(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_native(v) for v in obj]
    if isinstance(obj, (np.integer, np.floating)):
        return obj.item()
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    return obj


def log_run(method, dataset, metrics: dict, config: dict = None, sweep_id: str = None, db_path: str = None):
    """Append one row to the ``runs`` table (db_path > $DB_PATH > logs/benchmark_runs.db)."""
    if db_path is None:
        db_path = os.getenv("DB_PATH", "logs/benchmark_runs.db")
    db_dir = os.path.dirname(db_path)
    if db_dir:
        os.makedirs(db_dir, exist_ok=True)
    try:
        branch = subprocess.check_output(["git", "rev-parse", "--abbrev-ref", "HEAD"],
                                         stderr=subprocess.DEVNULL).decode().strip()
        commit = subprocess.check_output(["git", "rev-parse", "HEAD"], stderr=subprocess.DEVNULL).decode().strip()
    except Exception:
        branch = commit = "unknown"
    try:
        from importlib.metadata import version
        pkg_version = version("haag-vq")
    except Exception:
        pkg_version = "mivq-dev"
    cli = " ".join(shlex.quote(a) for a in sys.argv)
    con = sqlite3.connect(db_path, timeout=120)  # ranks of `--gpus N` share the file
    cur = con.cursor()
    cur.execute(
        "CREATE TABLE IF NOT EXISTS runs (id INTEGER PRIMARY KEY AUTOINCREMENT, timestamp TEXT, "
        "git_branch TEXT, git_commit TEXT, package_version TEXT, method TEXT, dataset TEXT, "
        "cli_command TEXT, metrics_json TEXT)"
    )
    for col in ("config_json", "sweep_id"):
        try:
            cur.execute(f"ALTER TABLE runs ADD COLUMN {col} TEXT")
            con.commit()
        except sqlite3.OperationalError:
            pass
    cur.execute(
        "INSERT INTO runs (timestamp, git_branch, git_commit, package_version, method, dataset, "
        "cli_command, metrics_json, config_json, sweep_id) VALUES (?, ?, ?, ?, ?, ?, ?, ?, ?, ?)",
        (
            datetime.now(timezone.utc).replace(tzinfo=None).isoformat(),
            branch,
            commit,
            pkg_version,
            method,
            dataset,
            cli,
            json.dumps(_native(metrics)),
            json.dumps(_native(config)) if config else "{}",
            sweep_id,
        ),
    )
    con.commit()
    con.close()
