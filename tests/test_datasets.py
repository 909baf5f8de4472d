"""Dataset templates run as initializer scripts on tenant bootstrap (``services/dataset_runner.py``,
``services/builders.py``, ``sitewhere_amd/datasets/*``).

Reference: ``service-tenant-management/dockerimage/datasets/construction`` and ``airtraffic``
(``dataset-template.json`` + ``deviceModel.groovy`` / ``assetModel.groovy`` / ``scheduleModel.groovy``):
a tenant created from the construction template gets the reference device types (including the
composite gateway and its nested element schema), commands, groups, assigned devices with
measurements / alerts / locations and alarms for critical alerts, the asset catalogue and the
schedules; a tenant-scoped ``initializer-<name>`` script replaces the packaged initializer."""
from __future__ import annotations

import pytest

from sitewhere_amd.assembly import SiteWhereInstance
from sitewhere_amd.services.dataset_runner import dataset_templates, params


@pytest.fixture(scope="module")
def sw():
    inst = SiteWhereInstance().start()
    inst.wait_for_tenant("default", 60)
    yield inst
    inst.stop()


def test_templates_listed():
    t = dataset_templates()
    assert {"empty", "construction", "airtraffic"} <= set(t)
    assert t["construction"]["initializers"]["deviceManagement"] == ["device_model.py"]
    assert params()["devices_per_site"] == 3          # conftest sizing via SITEWHERE_DATASET_*


def test_construction_dataset(sw):
    run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
    dm, am = sw.api("DeviceManagement", "default"), sw.api("AssetManagement", "default")
    em, sm = sw.api("DeviceEventManagement", "default"), sw.api("ScheduleManagement", "default")
    types = {t.token: t for t in run(lambda: dm.list_device_types({"pageSize": 0})).results}
    assert {"galaxytab3", "uno", "mega2560", "raspberrypi", "mt90", "gateway", "openhab", "nodered", "laipac-S911",
            "iphone6s", "ipad"} <= set(types)
    gw = types["gateway"]
    assert getattr(gw.container_policy, "value", gw.container_policy) == "Composite"
    schema = gw.device_element_schema
    units = schema["deviceUnits"] if isinstance(schema, dict) else schema.device_units
    paths = {(u["path"] if isinstance(u, dict) else u.path) for u in units}
    assert paths == {"default", "hv1"}
    cmds = {c.token for c in run(lambda: dm.list_device_commands({"deviceTypeToken": "raspberrypi",
                                                                  "pageSize": 0})).results}
    assert {"raspberrypi-helloWorld", "raspberrypi-ping", "raspberrypi-testEvents"} <= cmds
    groups = {g.token for g in run(lambda: dm.list_device_groups({"pageSize": 0})).results}
    assert {"heavy-equipment", "personnel", "sensors", "supervisors"} <= groups
    devices = run(lambda: dm.list_devices({"pageSize": 0})).results
    assert len(devices) == 3 + 20                          # scripted devices + fixed demo fleet
    scripted = [d for d in devices if "-" in d.token and d.token.split("-")[0].isdigit()]
    assert len(scripted) == 3 and all(d.device_assignment_id for d in scripted)
    total_mx = 0
    for d in scripted:
        mx = run(lambda d=d: em.list_measurements_for_index("Assignment", [d.device_assignment_id],
                                                              {"pageSize": 0}))
        total_mx += mx.num_results
        locs = run(lambda d=d: em.list_locations_for_index("Assignment", [d.device_assignment_id], {"pageSize": 0}))
        assert locs.num_results == params()["locations_per_assignment"]
    assert total_mx == 3 * 2 * params()["measurements_per_assignment"]
    assets = {a.token for a in run(lambda: am.list_assets()).results}
    assert {"derek.adams@sitewhere.com", "923483933-SERIAL-NUMBER-416F", "asset-0", "asset-5"} <= assets
    assert run(lambda: sm.get_schedule_by_token("every-hour")) is not None
    assert run(lambda: sm.get_schedule_by_token("on-the-half-hour")) is not None


def test_airtraffic_dataset_and_script_override(sw):
    tm = sw.api("TenantManagement")
    scripts = sw.instance.scripts
    scripts.create_script("ovr", "asset-management", "initializer-asset_model", "custom assets",
                          "asset_builder.persist(asset_builder.new_asset_type('drone', 'Drone', 'Hardware'))\n"
                          "asset_builder.persist(asset_builder.new_asset('drone', 'drone-1', 'Drone 1'))\n")
    for tok in ("air", "ovr"):
        sw.instance.system_user.run(lambda tok=tok: tm.create_tenant({"token": tok, "name": tok,
                                                                      "datasetTemplateId": "airtraffic"}))
    for tok in ("air", "ovr"):
        sw.wait_for_tenant(tok, 120)
    run = lambda f, t="air": sw.instance.system_user.run(f, t)  # noqa: E731
    dm, am = sw.api("DeviceManagement", "air"), sw.api("AssetManagement", "air")
    devs = [d.token for d in run(lambda: dm.list_devices({"pageSize": 0})).results]
    assert sorted(devs) == [f"flight-{i:03d}" for i in range(params()["flights"])]
    assert run(lambda: dm.get_zone_by_token("atl-restricted")) is not None
    assert {a.token for a in run(lambda: am.list_assets()).results} >= {"aircraft-000", "derek.adams@sitewhere.com"}
    am2 = sw.api("AssetManagement", "ovr")
    assert [a.token for a in run(lambda: am2.list_assets(), "ovr").results] == ["drone-1"]
