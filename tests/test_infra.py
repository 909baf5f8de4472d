"""Network infra (bus + coordination over gRPC) and a multi-process instance.

Mirrors the reference's deployment shape: separate service processes sharing Kafka + ZooKeeper and
calling each other over gRPC (SURVEY §1 process boundaries, §5.3 failure detection).
"""
from __future__ import annotations

import os
import subprocess
import sys
import time

import pytest

from sitewhere_amd.bus.log import EventBus
from sitewhere_amd.coord.store import NODE_ADDED, NODE_REMOVED, Coordination, InterProcessMutex, NoNodeError
from sitewhere_amd.services.dataset_runner import params as dataset_params
from sitewhere_amd.rpc.infra import InfraServer, RemoteCoordination, RemoteEventBus

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def infra():
    srv = InfraServer(EventBus(None, default_partitions=4), Coordination(), session_timeout_s=2.0).start()
    yield srv
    srv.stop()


def test_remote_bus_produce_consume_groups(infra):
    a, b = RemoteEventBus(infra.address), RemoteEventBus(infra.address)
    prod = a.producer()
    for i in range(100):
        prod.send("t1", f"dev-{i % 10}", f"v{i}".encode())
    c1 = b.consumer("g", ["t1"])
    c2 = a.consumer("g", ["t1"])
    got = []
    end = time.time() + 10
    while len(got) < 100 and time.time() < end:
        for c in (c1, c2):
            for recs in c.poll(100).values():
                got += recs
            c.commit()
    assert sorted(r.value for r in got) == sorted(f"v{i}".encode() for i in range(100))
    # per-key ordering within a partition
    by_key: dict = {}
    for r in got:
        by_key.setdefault(r.key, []).append(int(r.value[1:]))
    assert all(v == sorted(v) for v in by_key.values())
    assert {tp[1] for tp in c1.assignment()}.isdisjoint({tp[1] for tp in c2.assignment()})
    # committed offsets: a new member of the group starts where the group left off
    c1.close()
    c2.close()
    c3 = b.consumer("g", ["t1"])
    assert sum(len(x) for x in c3.poll(200).values()) == 0
    # a fresh group replays everything (fan-out)
    c4 = b.consumer("other", ["t1"])
    n = 0
    end = time.time() + 5
    while n < 100 and time.time() < end:
        n += sum(len(x) for x in c4.poll(100).values())
    assert n == 100


def test_remote_coordination_crud_watch_lock(infra):
    c1, c2 = RemoteCoordination(infra.address), RemoteCoordination(infra.address)
    events = []
    cancel = c2.watch_tree("/sw", lambda k, p, d: events.append((k, p)), initial=False)
    c1.create("/sw/conf/a.json", b"{}")
    assert c2.get_data("/sw/conf/a.json") == b"{}"
    st = c1.set("/sw/conf/a.json", b'{"x":1}')
    assert st.version == 1
    assert c2.children("/sw/conf") == ["a.json"]
    with pytest.raises(NoNodeError):
        c2.get("/sw/missing")
    end = time.time() + 5
    while time.time() < end and (NODE_ADDED, "/sw/conf/a.json") not in events:
        time.sleep(0.05)
    assert (NODE_ADDED, "/sw/conf/a.json") in events
    cancel()
    # ephemeral node vanishes when its session is closed (process death -> expiry)
    s = c1.open_session()
    c1.create("/sw/live/me", b"", ephemeral=True, session=s)
    assert c2.exists("/sw/live/me")
    c1.close_session(s)
    assert not c2.exists("/sw/live/me")
    # inter-process mutex across clients
    m1 = InterProcessMutex(c1, "/sw/locks/boot")
    m2 = InterProcessMutex(c2, "/sw/locks/boot")
    assert m1.acquire(2)
    assert not m2.acquire(0.5)
    m1.release()
    assert m2.acquire(2)
    m2.release()
    assert c2.wait_for("/sw/conf/a.json", 1.0)
    assert not c2.wait_for("/sw/nothing", 0.3)


def test_session_expiry_removes_ephemerals(infra):
    c = RemoteCoordination(infra.address, keepalive_s=100.0)   # no keepalive: session will expire
    s = c.open_session()
    c.create("/sw/eph", b"", ephemeral=True, session=s)
    removed = []
    RemoteCoordination(infra.address).watch_tree("/sw", lambda k, p, d: removed.append((k, p)), initial=False)
    end = time.time() + 8
    while time.time() < end and (NODE_REMOVED, "/sw/eph") not in removed:
        time.sleep(0.1)
    assert (NODE_REMOVED, "/sw/eph") in removed


def _spawn(args, log):
    env = dict(os.environ, PYTHONPATH=REPO)
    return subprocess.Popen([sys.executable, "-m", "sitewhere_amd.serve", "--heartbeat", "0.5", "--log-level", "WARNING",
                             *args], cwd=REPO, env=env, stdout=log, stderr=subprocess.STDOUT)


@pytest.mark.slow
def test_multiprocess_instance(infra, tmp_path):
    """Global services in one process, device+event management in another, client in a third."""
    from sitewhere_amd.runtime.config import InstanceSettings
    from sitewhere_amd.runtime.microservice import Instance
    from sitewhere_amd.runtime.topology import TopologyStateAggregator
    logs = [open(tmp_path / f"p{i}.log", "w") for i in range(2)]
    procs = [_spawn(["service", "instance-management", "user-management", "tenant-management", "--infra",
                     infra.address], logs[0]),
             _spawn(["service", "device-management", "event-management", "asset-management", "--infra",
                     infra.address], logs[1])]
    try:
        inst = Instance(InstanceSettings(heartbeat_s=0.5), bus=RemoteEventBus(infra.address),
                        coord=RemoteCoordination(infra.address),
                        network_rpc=True)
        topo = TopologyStateAggregator(inst.bus, inst.naming.microservice_state_updates(), "test-client", 30.0)
        from sitewhere_amd.core.lifecycle import LifecycleProgressMonitor
        topo.lifecycle_start(LifecycleProgressMonitor())
        inst.router.topology = topo
        assert topo.wait_for("device-management", 60, tenant="default"), "device-management never came up"
        dm = inst.router.proxy("DeviceManagement", "default")
        n = 0
        end = time.time() + 60
        while time.time() < end:
            try:
                n = inst.system_user.run(lambda: dm.list_devices({"pageSize": 0}).num_results, "default")
                if n == 20 + dataset_params()["devices_per_site"]:          # demo fleet + scripted
                    break
            except Exception:
                pass
            time.sleep(0.2)
        assert n == 20 + dataset_params()["devices_per_site"]
        um = inst.router.proxy("UserManagement")
        assert inst.system_user.run(lambda: um.get_user_by_username("admin")).username == "admin"
        em = inst.router.proxy("DeviceEventManagement", "default")
        dev = inst.system_user.run(lambda: dm.get_device_by_token("meitrack-000"), "default")
        ev = inst.system_user.run(lambda: em.add_measurements(dev.device_assignment_id, {"name": "x", "value": 1.0}),
                                  "default")
        assert ev[0].device_id == dev.id
        topo.lifecycle_stop(LifecycleProgressMonitor())
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        for f in logs:
            f.close()
