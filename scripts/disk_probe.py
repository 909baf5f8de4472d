"""O_DIRECT write bandwidth of a directory (the bench's segment store disk) by writer layout: one
writer issuing W-MiB writes, or T threads each writing its own file or its own slice of one file
(pwrite at disjoint offsets), each ending with fdatasync.  Prints one JSON line per layout.

    python scripts/disk_probe.py [--dir DIR] [--mb 2048]"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import tempfile
import threading
import time


def _write(fd, buf, offset, n, use_pwrite):
    for k in range(n):
        if use_pwrite:
            os.pwrite(fd, buf, offset + k * len(buf))
        else:
            os.write(fd, buf)


def run(directory, total_mb, chunk_mb, threads, one_file):
    chunk = chunk_mb << 20
    per = max(1, total_mb // chunk_mb // threads)
    bufs = []
    for _ in range(threads):
        b = mmap.mmap(-1, chunk)
        b.write(os.urandom(4096) * (chunk // 4096))
        bufs.append(b)
    flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC | getattr(os, "O_DIRECT", 0)
    paths = [os.path.join(directory, f".probe-{os.getpid()}-{t}") for t in range(1 if one_file else threads)]
    fds = [os.open(p, flags, 0o600) for p in paths]
    t0 = time.perf_counter()
    ths = [threading.Thread(target=_write, args=(fds[0 if one_file else t], bufs[t], t * per * chunk, per, True))
           for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for fd in fds:
        os.fdatasync(fd)
    dt = time.perf_counter() - t0
    for fd, p in zip(fds, paths):
        os.close(fd)
        os.remove(p)
    for b in bufs:
        b.close()
    return threads * per * chunk / dt / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=None)
    ap.add_argument("--mb", type=int, default=2048)
    a = ap.parse_args()
    d = a.dir or tempfile.mkdtemp(prefix="sw-disk-probe-")
    import shutil
    print(json.dumps({"dir": d, "fs_free_gb": round(shutil.disk_usage(d).free / 1e9, 1)}), flush=True)
    for chunk_mb, threads, one_file in ((4, 1, True), (16, 1, True), (64, 1, True), (16, 2, True), (16, 4, True),
                                        (16, 8, True), (16, 4, False), (64, 4, True)):
        gbps = run(d, a.mb, chunk_mb, threads, one_file)
        print(json.dumps({"chunk_mb": chunk_mb, "threads": threads, "one_file": one_file, "gbps": round(gbps, 2)}),
              flush=True)
    if not a.dir:
        os.rmdir(d)


if __name__ == "__main__":
    main()
