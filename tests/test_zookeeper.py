"""ZooKeeper wire protocol: the coordination surface on a ZooKeeper session (chroot namespace,
versions, ephemeral/sequential nodes, TreeCache-style watches, the mutex recipe) against the
in-process ZooKeeper stand-in, and a whole instance coordinated through it.  Parity unpinned against a
real ZooKeeper ensemble (none here)."""
import threading
import time

import pytest

from sitewhere_amd.coord.store import (INITIALIZED, NODE_ADDED, NODE_REMOVED, NODE_UPDATED, BadVersionError,
                                       InterProcessMutex, NodeExistsError, NoNodeError, NotEmptyError)
from sitewhere_amd.coord.zk import ZooKeeperCoordination
from sitewhere_amd.coord.zk_server import MiniZooKeeperServer


@pytest.fixture
def zk():
    srv = MiniZooKeeperServer(port=0).start()
    yield srv
    srv.stop()


def test_crud_versions_sequential_ephemeral(zk):
    c = ZooKeeperCoordination(f"{zk.address}/sitewhere")
    assert "/sitewhere" in zk.nodes                       # namespace created as a chroot
    c.create("/a/b/c", b"x")                              # parents created on demand
    assert c.get_data("/a/b/c") == b"x" and c.children("/a") == ["b"]
    st = c.set("/a/b/c", b"y")
    assert st.version == 1 and c.exists("/a/b/c").version == 1
    with pytest.raises(BadVersionError):
        c.set("/a/b/c", b"z", version=0)
    with pytest.raises(NodeExistsError):
        c.create("/a/b/c")
    with pytest.raises(NotEmptyError):
        c.delete("/a")
    s1 = c.create("/q/item-", b"1", sequential=True)
    s2 = c.create("/q/item-", b"2", sequential=True)
    assert s1 == "/q/item-0000000000" and s2 == "/q/item-0000000001"
    sess = c.open_session()
    c.create("/eph", b"", ephemeral=True, session=sess)
    assert zk.nodes["/sitewhere/eph"].owner != 0
    c.close_session(sess)                                  # session end removes its ephemerals
    end = time.time() + 5
    while c.exists("/eph") is not None and time.time() < end:
        time.sleep(0.02)
    assert c.exists("/eph") is None
    c.delete("/a", recursive=True)
    assert c.walk("/") == ["/", "/q", "/q/item-0000000000", "/q/item-0000000001"]
    with pytest.raises(NoNodeError):
        c.get("/a")
    c.close()


def test_tree_watch_and_wait_for(zk):
    c = ZooKeeperCoordination(f"{zk.address}/sw")
    c.create("/conf/tenants/t1/svc.json", b"v1")
    got, ready = [], threading.Event()

    def cb(kind, path, data):
        got.append((kind, path, data))
        if kind == INITIALIZED:
            ready.set()
    cancel = c.watch_tree("/conf", cb)
    assert ready.wait(5)
    assert (NODE_ADDED, "/conf/tenants/t1/svc.json", b"v1") in got
    got.clear()
    other = ZooKeeperCoordination(f"{zk.address}/sw")          # another process's client
    other.put("/conf/tenants/t1/svc.json", b"v2")
    other.create("/conf/tenants/t2/svc.json", b"n")
    other.delete("/conf/tenants/t1", recursive=True)

    def seen(kind, path):
        end = time.time() + 5
        while time.time() < end:
            if any(k == kind and p == path for k, p, _ in got):
                return True
            time.sleep(0.02)
        return False
    assert seen(NODE_UPDATED, "/conf/tenants/t1/svc.json")
    assert seen(NODE_ADDED, "/conf/tenants/t2/svc.json")
    assert seen(NODE_REMOVED, "/conf/tenants/t1/svc.json") and seen(NODE_REMOVED, "/conf/tenants/t1")
    threading.Timer(0.3, lambda: other.create("/state/bootstrapped")).start()
    assert c.wait_for("/state/bootstrapped", 5) and not c.wait_for("/state/never", 0.3)
    cancel()
    c.close()
    other.close()


def test_mutex_recipe_over_zookeeper(zk):
    a, b = ZooKeeperCoordination(f"{zk.address}/sw"), ZooKeeperCoordination(f"{zk.address}/sw")
    m1, m2 = InterProcessMutex(a, "/locks/boot"), InterProcessMutex(b, "/locks/boot")
    assert m1.acquire(2)
    assert not m2.acquire(0.3)                             # held by the other session
    threading.Timer(0.2, m1.release).start()
    assert m2.acquire(5)
    m2.release()
    a.close()
    b.close()


def test_whole_instance_coordinated_by_zookeeper(zk):
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire
    from sitewhere_amd.runtime.config import InstanceSettings
    from sitewhere_amd.runtime.microservice import Instance
    inst = Instance(InstanceSettings(heartbeat_s=1.0), coord=ZooKeeperCoordination(f"{zk.address}/sitewhere"))
    sw = SiteWhereInstance(instance=inst).start()
    try:
        sw.wait_for_tenant("default", 120)
        assert any(p.endswith("/bootstrapped") for p in zk.nodes)      # markers live in ZooKeeper
        run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "default"), sw.api("DeviceEventManagement", "default")
        aid = run(lambda: dm.get_device_by_token("meitrack-002")).device_assignment_id
        sw.tenant_engine("event-sources").inject("default-protobuf", wire.measurements("meitrack-002", {"zk.t": 3.0}))
        end, res = time.time() + 30, []
        while not res and time.time() < end:
            res = run(lambda: em.list_measurements_for_index("Assignment", [aid])).results
            time.sleep(0.1)
        assert res and res[0].value == 3.0
    finally:
        sw.stop()
