"""``bench.py`` at N=8 on the CPU: eight processes over gloo run the native CPU
engine through the bench's own multi-rank path -- device-sharded all-to-all re-key of every step,
durable blocks per rank, reject routing -- and the bench's conservation checks hold on every rank
(each decoded event is persisted once by its owner or rejected where its payload is)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_gloo_world8_conserves(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "3", "--warmup", "1", "--engine", "cpu", "--msgs", "4096",
           "--devices", "4096", "--store", str(1 << 20), "--dedup-filter-ids", str(1 << 20),
           "--disk-probe-mb", "0", "--durable-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=str(tmp_path), env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 8 and d["detail"]["world"] == 8 and d["detail"]["backend"] == "gloo"
    assert d["detail"]["conservation"]["ok"], d["detail"]["conservation"]
    assert d["detail"]["exchange_bytes_per_rank_step"] > 0
    assert d["detail"]["durable"]["all_durable"]
