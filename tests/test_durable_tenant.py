"""Durable persistence of the MI355X-pipeline tenant (``gpu-columnar``) across a kill.

Reference: ``DeviceEventBuffer.java:99-135`` buffers Mongo bulk writes and loses them on a crash
(SURVEY §5.4).  Here every engine step's block is on disk, with a commit record of the raw-topic
offset it completes, before that offset is committed.  The test kills an instance mid-stream
(``os._exit``: nothing flushed or closed) and checks, from the files alone, that

* the events on disk are exactly those of the raw batches before the durable offset the store's
  commit records name (the child loses the bus commits past batch 9, so the disk runs ahead of the
  bus, as after a crash between a block's fdatasync and its offset commit);
* a new instance over the same directories resumes behind that offset and, once it has consumed
  the rest, every event of every batch is on disk exactly once (no loss, no duplicate).

CPU engines drive the same tenant code as the MI355X engine (``device: auto`` picks the native
CPU engine in this container)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
N_BATCHES, PER, KILL_AFTER = 24, 40, 9


def _child(phase: str, bus_dir: str, data_dir: str, timeout=240):
    env = dict(os.environ, SITEWHERE_DATA_DIR=data_dir)
    p = subprocess.run([sys.executable, os.path.join(HERE, "durable_child.py"), phase, bus_dir, str(N_BATCHES),
                        str(PER), str(KILL_AFTER)], capture_output=True, text=True, timeout=timeout, env=env)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def _values_on_disk(path: str):
    from sitewhere_amd.persistence.segments import DurableEventStore, decode_block
    st = DurableEventStore(path)
    try:
        vals = [decode_block(st.seg.read_block(e))["v0"] for e in st.seg.index()
                if int(e["boot"]) != st.api_boot]                 # engine blocks (not API-added events)
        return np.sort(np.concatenate(vals)) if vals else np.zeros(0), st
    except Exception:
        st.close()
        raise


def _expected(batches):
    return np.sort(np.array([float(1000 * b + i) for b in batches for i in range(PER)]))


def test_durable_tenant_survives_kill_exactly_once(tmp_path):
    from sitewhere_amd.bus.log import EventBus
    bus_dir, data_dir = str(tmp_path / "bus"), str(tmp_path / "data")
    rc, out, err = _child("run", bus_dir, data_dir)
    assert rc == 9, err[-3000:]
    info = out[0]
    store_dir = os.path.join(data_dir, "dur", "events")

    # ---- after the kill: what is on disk is exactly what the commit records name
    vals, st = _values_on_disk(store_dir)
    try:
        durable = st.source_offset(info["src_topic"], 0)
    finally:
        st.close()
    bus = EventBus(bus_dir, default_partitions=1)
    committed = bus.committed(info["group"], info["topic"], 0)
    bus.close()
    print(f"killed: durable offset {durable}, committed {committed}")
    assert durable is not None and committed == KILL_AFTER    # later bus commits were lost (see child)
    assert KILL_AFTER + 3 <= durable <= N_BATCHES     # the disk ran ahead of the bus commit
    np.testing.assert_array_equal(vals, _expected(range(durable)))

    # ---- restart: resume behind the durable offset, consume the rest, every event exactly once
    rc, out2, err = _child("resume", bus_dir, data_dir)
    assert rc == 0, err[-3000:]
    assert out2[0]["boot"] != info["boot"]              # a new engine incarnation
    assert out2[-1]["committed"] == N_BATCHES
    assert out2[-1]["persisted"] == (N_BATCHES - durable) * PER   # nothing before the offset re-stepped
    vals, st = _values_on_disk(store_dir)
    try:
        assert st.source_offset(info["src_topic"], 0) == N_BATCHES
        boots = {int(e["boot"]) for e in st.seg.index()} - {st.api_boot}     # engine incarnations
    finally:
        st.close()
    np.testing.assert_array_equal(vals, _expected(range(N_BATCHES)))
    assert len(boots) == (2 if durable < N_BATCHES else 1)


def test_commit_records_survive_reopen_and_torn_tail(tmp_path):
    """Blocks with commit records: offsets come back on reopen; a flagged block whose record was
    torn off is dropped with it (the block and its offsets are durable together or not at all)."""
    from sitewhere_amd.models.columnar import OUT_REC
    from sitewhere_amd.persistence.segments import (SegmentStore, encode_block, seal, set_commit_flag,
                                                    source_key)

    def block(k):
        rows = np.zeros(50, OUT_REC)
        rows["event_date"] = 1_700_000_000_000 + np.arange(50) + 100 * k
        rows["v0"] = np.arange(50) + 1000.0 * k
        b = encode_block(rows)
        seal(b, 50 * k, 1, 7, 0, 1)
        set_commit_flag(b)
        return b

    d = str(tmp_path / "s")
    st = SegmentStore(d, direct=False)
    for k in range(3):
        b = block(k)
        st.append(b.ctypes.data, len(b), b, src=[("raw", 0, k + 1), ("raw", 1, 10 * (k + 1))])
    st.flush()
    assert st.sources() == {source_key("raw", 0): 3, source_key("raw", 1): 30}
    st.close()
    st = SegmentStore(d, direct=False)
    assert st.source_offset("raw", 0) == 3 and len(st.index()) == 3
    path = st.file_path(int(st.index()[-1]["file"]))
    st.close()
    size = os.path.getsize(path)
    with open(path, "r+b") as f:
        f.truncate(size - 4096 + 100)       # tear the last commit record
    st = SegmentStore(d, direct=False)
    assert len(st.index()) == 2 and st.source_offset("raw", 0) == 2
    assert st.source_offset("raw", 1) == 20
    st.close()
