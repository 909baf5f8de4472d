"""The reference's gRPC plane: ``/com.sitewhere.grpc.service.<Service>/<Rpc>`` with the ``G*``
protobuf messages (``rpc/protoplane.py``).

The wire-compatibility test builds its client from the reference's own ``.proto`` files
(``sitewhere-grpc-*/src/main/proto``, parsed with the protobuf runtime's descriptor pool; the copies
under ``sitewhere_amd/rpc/schema`` when the reference tree is absent) -- raw request messages
serialized by that pool, responses parsed by it, nothing of this framework's converter on the
client side -- and drives a device-type / device / assignment / measurements round trip over a
real gRPC socket against an instance serving its network RPC plane."""
from __future__ import annotations

import glob
import os

import grpc
import pytest

from sitewhere_amd.assembly import SiteWhereInstance
from sitewhere_amd.rpc import protoplane as pp

REF = "/root/reference"
SVC = "com.sitewhere.grpc.service"
MODEL = "com.sitewhere.grpc.model"


def _reference_pool():
    from google.protobuf import message_factory
    from sitewhere_amd.models.protoschema import load_proto_files
    paths = [p for p in glob.glob(os.path.join(REF, "sitewhere-grpc-*/src/main/proto/*.proto"))
             if not p.endswith("sitewhere-kafka.proto")]
    if not paths:                                   # no reference tree: the repo's schema copies
        paths = glob.glob(os.path.join(pp.SCHEMA_DIR, "*.proto"))
    files = {}
    for p in paths:
        with open(p) as f:
            files[os.path.basename(p)] = f.read()
    pool = load_proto_files(files)

    def get(name):
        try:
            return message_factory.GetMessageClass(pool.FindMessageTypeByName(name))
        except KeyError:
            return pool.FindEnumTypeByName(name)            # an enum descriptor
    return get


@pytest.fixture(scope="module")
def inst():
    sw = SiteWhereInstance(network_rpc=True).start()
    sw.wait_for_tenant("default", 60)
    yield sw
    sw.stop()


def _raw_call(channel, jwt, service, rpc, req, resp_cls, tenant="default"):
    stub = channel.unary_unary(f"/{SVC}.{service}/{rpc}", request_serializer=lambda m: m.SerializeToString(),
                               response_deserializer=resp_cls.FromString)
    return stub(req, metadata=[("authorization", f"Bearer {jwt}"), ("tenant", tenant)], timeout=30)


def test_reference_schema_client_round_trip(inst):
    G = _reference_pool()
    jwt = inst.instance.system_jwt()
    dm = grpc.insecure_channel(inst["device-management"].rpc_server.address)
    em = grpc.insecure_channel(inst["event-management"].rpc_server.address)

    # CreateDeviceType
    req = G(f"{SVC}.GCreateDeviceTypeRequest")()
    req.request.token.value = "wire-type"
    req.request.name.value = "Wire Type"
    req.request.description.value = "from a reference-schema client"
    req.request.metadata["rev"] = "3"
    dt = _raw_call(dm, jwt, "DeviceManagement", "CreateDeviceType", req, G(f"{SVC}.GCreateDeviceTypeResponse")).deviceType
    assert dt.name == "Wire Type" and dt.entityInformation.token == "wire-type"
    assert dt.entityInformation.metadata["rev"] == "3" and (dt.entityInformation.id.msb or dt.entityInformation.id.lsb)

    # CreateDevice (device type by token), CreateDeviceAssignment (device by token)
    req = G(f"{SVC}.GCreateDeviceRequest")()
    req.request.token.value = "wire-dev-1"
    req.request.deviceTypeToken.value = "wire-type"
    req.request.comments.value = "wired"
    dev = _raw_call(dm, jwt, "DeviceManagement", "CreateDevice", req, G(f"{SVC}.GCreateDeviceResponse")).device
    assert dev.entityInformation.token == "wire-dev-1" and dev.comments.value == "wired"
    assert (dev.deviceTypeId.msb, dev.deviceTypeId.lsb) == (dt.entityInformation.id.msb, dt.entityInformation.id.lsb)
    req = G(f"{SVC}.GCreateDeviceAssignmentRequest")()
    req.request.deviceToken.value = "wire-dev-1"
    asg = _raw_call(dm, jwt, "DeviceManagement", "CreateDeviceAssignment", req,
                    G(f"{SVC}.GCreateDeviceAssignmentResponse")).assignment
    assert (asg.deviceId.msb, asg.deviceId.lsb) == (dev.entityInformation.id.msb, dev.entityInformation.id.lsb)
    assert G(f"{MODEL}.GDeviceAssignmentStatus").values_by_number[asg.status].name.endswith("ACTIVE")

    # ListDevices filtered by device type, paged
    req = G(f"{SVC}.GListDevicesRequest")()
    req.criteria.deviceType.token = "wire-type"
    req.criteria.paging.pageNumber, req.criteria.paging.pageSize = 1, 10
    res = _raw_call(dm, jwt, "DeviceManagement", "ListDevices", req, G(f"{SVC}.GListDevicesResponse")).results
    assert res.count == 1 and [d.entityInformation.token for d in res.devices] == ["wire-dev-1"]

    # AddMeasurements, then ListMeasurementsForIndex (assignment index), newest first
    req = G(f"{SVC}.GAddMeasurementsRequest")()
    req.deviceAssignmentId.CopyFrom(asg.entityInformation.id)
    for i, v in enumerate((20.5, 21.5, 22.5)):
        m = req.requests.add()
        m.name, m.value = "temp", v
        m.event.eventDate = 1_700_000_000_000 + 1000 * i
        m.event.alternateId.value = f"wire-{i}"
    added = _raw_call(em, jwt, "DeviceEventManagement", "AddMeasurements", req,
                      G(f"{SVC}.GAddMeasurementsResponse")).measurements
    assert [m.value for m in added] == [20.5, 21.5, 22.5]
    assert all(m.event.alternateId.value == f"wire-{i}" for i, m in enumerate(added))
    req = G(f"{SVC}.GListMeasurementsForIndexRequest")()
    req.index = G(f"{MODEL}.GDeviceEventIndex").values_by_name["EVENT_INDEX_ASSIGNMENT"].number
    req.entityIds.add().CopyFrom(asg.entityInformation.id)
    req.criteria.pageNumber, req.criteria.pageSize = 1, 2
    res = _raw_call(em, jwt, "DeviceEventManagement", "ListMeasurementsForIndex", req,
                    G(f"{SVC}.GListMeasurementsForIndexResponse")).results
    assert res.count == 3 and [m.value for m in res.measurements] == [22.5, 21.5]
    assert res.measurements[0].event.eventDate == 1_700_000_002_000
    assert (res.measurements[0].event.deviceAssignmentId.msb, res.measurements[0].event.deviceAssignmentId.lsb) == \
        (asg.entityInformation.id.msb, asg.entityInformation.id.lsb)
    dm.close()
    em.close()


def test_reference_client_api_objects(inst):
    """The converter client (:class:`ReferenceClient`): API objects in, domain models out."""
    c = pp.ReferenceClient(inst["device-management"].rpc_server.address, jwt=inst.instance.system_jwt(),
                           tenant="default")
    dm = c.api("DeviceManagement")
    t = dm.create_device_type({"token": "api-type", "name": "API Type", "metadata": {"k": "v"}})
    assert t.token == "api-type" and t.metadata == {"k": "v"}
    assert dm.get_device_type_by_token("api-type").id == t.id
    d = dm.create_device({"token": "api-dev", "deviceTypeToken": "api-type"})
    assert d.device_type_id == t.id
    page = dm.list_device_types({"pageNumber": 1, "pageSize": 100})
    assert page.num_results >= 1 and "api-type" in {x.token for x in page.results}
    with pytest.raises(grpc.RpcError) as e:
        dm.delete_device_type(t.id)                     # in use by a device
    assert e.value.code() != grpc.StatusCode.INTERNAL
    c.close()


def test_engine_event_ids_travel_as_guuids():
    for i in ("18b2c3d4e5f-12345", "1-0", "a1b2c3d4e5f6-99"):
        assert pp.id_of(*pp.uuid_of(i)) == i
    u = "0f8fad5b-d9cb-469f-a165-70867728950e"
    assert pp.id_of(*pp.uuid_of(u)) == u
