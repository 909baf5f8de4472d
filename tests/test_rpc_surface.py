"""RPC surface parity: every RPC of the reference's gRPC services (``sitewhere-grpc-*/src/main/proto/
*.proto``, 178 RPCs) resolves to a callable on our service implementation, through the
same snake_case mapping the transport uses, and every one of them is *invoked* over gRPC on its
reference path and schema (``/com.sitewhere.grpc.service.<Service>/<Rpc>``, ``rpc/protoplane.py``)."""
from __future__ import annotations

import pytest

from sitewhere_amd.rpc.transport import snake_method

REFERENCE_RPCS = {
    "AssetManagement": "CreateAssetType UpdateAssetType GetAssetTypeById GetAssetTypeByToken DeleteAssetType "
                       "ListAssetTypes CreateAsset UpdateAsset GetAssetById GetAssetByToken DeleteAsset ListAssets",
    "BatchManagement": "CreateBatchOperation CreateBatchCommandInvocation UpdateBatchOperation GetBatchOperation "
                       "GetBatchOperationByToken ListBatchOperations DeleteBatchOperation ListBatchOperationElements "
                       "UpdateBatchOperationElement",
    "ScheduleManagement": "CreateSchedule UpdateSchedule GetScheduleByToken ListSchedules DeleteSchedule "
                          "CreateScheduledJob UpdateScheduledJob GetScheduledJobByToken ListScheduledJobs "
                          "DeleteScheduledJob",
    "DeviceEventManagement": "AddDeviceEventBatch GetDeviceEventById GetDeviceEventByAlternateId AddMeasurements "
                             "ListMeasurementsForIndex AddLocations ListLocationsForIndex AddAlerts ListAlertsForIndex "
                             "AddCommandInvocations ListCommandInvocationsForIndex AddCommandResponses "
                             "ListCommandResponsesForInvocation ListCommandResponsesForIndex AddStateChanges "
                             "ListStateChangesForIndex",
    "UserManagement": "CreateUser ImportUser Authenticate UpdateUser GetUserByUsername ListUsers DeleteUser "
                      "CreateGrantedAuthority GetGrantedAuthorityByName UpdateGrantedAuthority ListGrantedAuthorities "
                      "DeleteGrantedAuthority GetGrantedAuthoritiesForUser AddGrantedAuthoritiesForUser "
                      "RemoveGrantedAuthoritiesForUser",
    "DeviceManagement": "CreateCustomerType GetCustomerType GetCustomerTypeByToken UpdateCustomerType ListCustomerTypes "
                        "DeleteCustomerType CreateCustomer GetCustomer GetCustomerByToken GetCustomerChildren "
                        "UpdateCustomer ListCustomers DeleteCustomer CreateAreaType GetAreaType GetAreaTypeByToken "
                        "UpdateAreaType ListAreaTypes DeleteAreaType CreateArea GetArea GetAreaByToken GetAreaChildren "
                        "UpdateArea ListAreas DeleteArea CreateZone GetZone GetZoneByToken UpdateZone ListZones "
                        "DeleteZone CreateDeviceType GetDeviceType GetDeviceTypeByToken UpdateDeviceType "
                        "ListDeviceTypes DeleteDeviceType CreateDeviceCommand GetDeviceCommand GetDeviceCommandByToken "
                        "UpdateDeviceCommand ListDeviceCommands DeleteDeviceCommand CreateDeviceStatus GetDeviceStatus "
                        "GetDeviceStatusByToken UpdateDeviceStatus ListDeviceStatuses DeleteDeviceStatus CreateDevice "
                        "GetDevice GetDeviceByToken UpdateDevice ListDevices CreateDeviceElementMapping "
                        "DeleteDeviceElementMapping DeleteDevice CreateDeviceGroup GetDeviceGroup GetDeviceGroupByToken "
                        "UpdateDeviceGroup ListDeviceGroups ListDeviceGroupsWithRole DeleteDeviceGroup "
                        "AddDeviceGroupElements RemoveDeviceGroupElements ListDeviceGroupElements "
                        "CreateDeviceAssignment GetDeviceAssignment GetDeviceAssignmentByToken "
                        "GetCurrentAssignmentForDevice DeleteDeviceAssignment UpdateDeviceAssignment "
                        "ListDeviceAssignments EndDeviceAssignment CreateDeviceStream GetDeviceStreamByStreamId "
                        "ListDeviceStreams CreateDeviceAlarm GetDeviceAlarm UpdateDeviceAlarm SearchDeviceAlarms "
                        "DeleteDeviceAlarm",
    "DeviceStateManagement": "CreateDeviceState GetDeviceState GetDeviceStateByDeviceAssignmentId SearchDeviceStates "
                             "UpdateDeviceState DeleteDeviceState",
    "LabelGeneration": "GetCustomerTypeLabel GetCustomerLabel GetAreaTypeLabel GetAreaLabel GetDeviceTypeLabel "
                       "GetDeviceLabel GetDeviceGroupLabel GetDeviceAssignmentLabel GetAssetTypeLabel GetAssetLabel",
    "MultitenantManagement": "CheckTenantEngineAvailable",
    "MicroserviceManagement": "GetConfigurationModel GetGlobalConfiguration GetTenantConfiguration "
                              "UpdateGlobalConfiguration UpdateTenantConfiguration GetScriptTemplates "
                              "GetScriptTemplateContent",
    "TenantManagement": "CreateTenant UpdateTenant GetTenantById GetTenantByToken ListTenants DeleteTenant "
                        "GetTenantTemplates GetDatasetTemplates",
}


def implementations():
    from sitewhere_amd.runtime.microservice import MicroserviceManagementApi, MultitenantManagementApi
    from sitewhere_amd.services.asset_management import AssetManagement
    from sitewhere_amd.services.batch_operations import BatchManagement
    from sitewhere_amd.services.device_management import DeviceManagement
    from sitewhere_amd.services.device_state import DeviceStateManagement
    from sitewhere_amd.services.event_management import DeviceEventManagement
    from sitewhere_amd.services.labels_media_search import LabelGeneration
    from sitewhere_amd.services.schedule_management import ScheduleManagement
    from sitewhere_amd.services.tenant_management import TenantManagement
    from sitewhere_amd.services.user_management import UserManagement
    return {"AssetManagement": AssetManagement, "BatchManagement": BatchManagement,
            "ScheduleManagement": ScheduleManagement, "DeviceEventManagement": DeviceEventManagement,
            "UserManagement": UserManagement, "DeviceManagement": DeviceManagement,
            "DeviceStateManagement": DeviceStateManagement, "LabelGeneration": LabelGeneration,
            "MultitenantManagement": MultitenantManagementApi, "MicroserviceManagement": MicroserviceManagementApi,
            "TenantManagement": TenantManagement}


def test_reference_rpc_count():
    assert sum(len(v.split()) for v in REFERENCE_RPCS.values()) == 178


@pytest.mark.parametrize("service", sorted(REFERENCE_RPCS))
def test_every_reference_rpc_is_implemented(service):
    impl = implementations()[service]
    missing = [m for m in REFERENCE_RPCS[service].split() if not callable(getattr(impl, snake_method(m), None))]
    assert not missing, f"{service} missing {missing}"


def test_schema_declares_the_reference_rpcs():
    from sitewhere_amd.rpc import protoplane as pp
    alias = {v: k for k, v in pp.SERVICE_ALIASES.items()}
    declared = {name: {m.name for m in sv.methods} for name, sv in pp.services().items()}
    for service, rpcs in REFERENCE_RPCS.items():
        assert declared[alias.get(service, service)] == set(rpcs.split()), service


def test_every_reference_rpc_is_invoked_over_grpc():
    """Each of the 178 RPCs is called with an empty request over a real gRPC socket: the answer is
    a response or a domain error status (not found, invalid argument, unauthenticated, ...) --
    never UNIMPLEMENTED, never an INTERNAL error, never an argument mismatch."""
    import logging

    import grpc

    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.rpc import protoplane as pp
    logging.getLogger("sitewhere").setLevel(logging.CRITICAL)
    sw = SiteWhereInstance(network_rpc=True).start()
    try:
        sw.wait_for_tenant("default", 60)
        c = pp.ReferenceClient(sw["device-management"].rpc_server.address, jwt=sw.instance.system_jwt(),
                               tenant="default")
        codes, bad, n = {}, [], 0
        for name, sv in pp.services().items():
            for m in sv.methods:
                n += 1
                try:
                    c.call(name, m.name, pp.message_class(m.input_type.full_name)(), timeout=20)
                    code = "OK"
                except grpc.RpcError as e:
                    code = e.code().name
                    det = e.details() or ""
                    if e.code() in (grpc.StatusCode.INTERNAL, grpc.StatusCode.UNIMPLEMENTED, grpc.StatusCode.UNKNOWN) \
                            or "positional argument" in det or "unexpected keyword" in det:
                        bad.append((name, m.name, code, det[:200]))
                codes[code] = codes.get(code, 0) + 1
        c.close()
        assert n == 178 and not bad, bad
        assert codes.get("OK", 0) >= 60, codes
    finally:
        sw.stop()
