"""Sequential write bandwidth of a file system, the way a segment store writes: large appends,
fdatasync per commit group, optionally O_DIRECT.  Usage: probe_disk.py PATH [GiB]"""
import mmap
import os
import sys
import time


def run(path, total, chunk, sync_every, direct):
    flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC | (os.O_DIRECT if direct else 0)
    fd = os.open(path, flags, 0o644)
    buf = mmap.mmap(-1, chunk)            # page-aligned (O_DIRECT needs it)
    buf.write(os.urandom(1 << 20) * (chunk >> 20))
    t0 = time.perf_counter()
    done, since, syncs = 0, 0, 0
    while done < total:
        n = os.write(fd, buf)
        done += n
        since += n
        if since >= sync_every:
            os.fdatasync(fd)
            since = 0
            syncs += 1
    os.fdatasync(fd)
    dt = time.perf_counter() - t0
    os.close(fd)
    os.unlink(path)
    return done / dt / 1e9, syncs


def main():
    path = sys.argv[1]
    gib = float(sys.argv[2]) if len(sys.argv) > 2 else 4
    total = int(gib * (1 << 30))
    for direct in (False, True):
        for chunk, sync_every in ((4 << 20, 64 << 20), (16 << 20, 256 << 20), (64 << 20, 1 << 30)):
            try:
                gbs, syncs = run(path, total, chunk, sync_every, direct)
                print(f"direct={int(direct)} chunk={chunk >> 20}MiB sync_every={sync_every >> 20}MiB: "
                      f"{gbs:.2f} GB/s ({syncs} syncs)", flush=True)
            except OSError as e:
                print(f"direct={int(direct)} chunk={chunk >> 20}MiB: {e}", flush=True)


if __name__ == "__main__":
    main()
