"""bench.py contract (driver-facing): one JSON line from rank 0 with the required keys, for N=1 and for
N=2 ranks under torch.distributed.run (gloo + the CPU oracle engine, so it runs without a GPU)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
SMALL = ["--engine", "cpu", "--msgs", "1500", "--devices", "1500", "--steps", "2", "--warmup", "1", "--store", "65536",
         "--batches", "2"]


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_bench_single_rank_json():
    r = subprocess.run([sys.executable, "bench.py", *SMALL], cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert KEYS <= set(d) and d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["metric"] == "device_events_per_sec" and d["value"] > 0 and d["higher_is_better"] is True
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])
    # the timed region ends with every block of the run durable on disk
    dd = d["detail"]["durable"]
    assert d["config"]["durable"] and dd["all_durable"] and dd["rows"] == d["detail"]["persisted"]
    assert dd["bytes_per_event"] > 0 and dd["durable_bytes_per_s"] > 0 and dd["fdatasyncs"] >= 1
    assert d["detail"]["conservation"]["ok"]


@pytest.mark.slow
def test_bench_two_ranks_torchrun(tmp_path):
    """Two ranks on gloo, each with its own segment directory (one per disk: ``--durable-dir a,b``):
    conservation holds over both ranks and each rank's blocks are in its own directory."""
    d1, d2 = str(tmp_path / "disk1"), str(tmp_path / "disk2")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", *SMALL,
                        "--durable-dir", f"{d1},{d2}", "--disk-probe-mb", "8"],
                       cwd=REPO, capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 3000 and d["config"]["parallelism"].startswith("dp2")
    assert d["detail"]["payloads"] == 2 * 2 * 1500
    # self-checking multi-rank record: the backend and world the process group really had, per-rank time
    det = d["detail"]
    assert det["backend"] == "gloo" and det["world"] == 2 and len(det["rank_elapsed_s"]) == 2
    assert det["exchange_bytes_per_rank_step"] > 0 and det["shuffle_overflow"] == 0
    assert det["conservation"]["ok"] and det["conservation"]["checked"] >= 4
    assert det["durable"]["disk_probe"]["dirs"] == 2 and det["durable"]["disk_probe"]["node_gbps"] > 0
    # local rank r writes to dirs[r % 2]
    for d, r in ((d1, 0), (d2, 1)):
        files = os.listdir(os.path.join(d, f"rank{r}"))
        assert any(f.endswith(".sweg") for f in files), (d, files)
