"""Sustained O_DIRECT write bandwidth of the segment directory's disk by writer parallelism: GB
written in 4 MiB pwrite()s at consecutive offsets of one file by 1, 2, 4, 8 threads (each thread the
next free chunk), fdatasync every 64 MiB group (the segment store's group commit) -- does the disk
take more than one in-flight write?  One JSON line."""
from __future__ import annotations

import json
import mmap
import os
import sys
import threading
import time


def run(path, total_mb, threads, chunk=4 << 20, group=64 << 20):
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | getattr(os, "O_DIRECT", 0), 0o600)
    bufs = []
    for _ in range(threads):
        b = mmap.mmap(-1, chunk)
        b.write(os.urandom(4096) * (chunk // 4096))
        bufs.append(b)
    n = total_mb * (1 << 20) // chunk
    per_group = group // chunk
    t0 = time.perf_counter()
    for g0 in range(0, n, per_group):
        idx = list(range(g0, min(n, g0 + per_group)))
        lock = threading.Lock()

        def work(k):
            while True:
                with lock:
                    if not idx:
                        return
                    i = idx.pop(0)
                os.pwrite(fd, bufs[k], i * chunk)
        th = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        os.fdatasync(fd)
    dt = time.perf_counter() - t0
    os.close(fd)
    os.remove(path)
    return round(n * chunk / dt / 1e9, 2)


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    out = {}
    for t in (1, 2, 4, 8):
        out[f"threads_{t}_gbps"] = run(os.path.join(d, f".par-probe-{os.getpid()}"), mb, t)
        print(json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
