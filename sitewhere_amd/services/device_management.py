"""service-device-management: the device registry (multitenant).

Reference: ``service-device-management`` -- ``DeviceManagementImpl`` (2,377 LoC) routed per tenant by
``DeviceManagementRouter`` over ``MongoDeviceManagement`` (2,474), decorated by
``CacheAwareDeviceManagement`` (near-cache writes) and ``DeviceManagementTriggers`` (state-change
events on assignment create/update/end, ``DeviceManagementTriggers.java:30-80``).  RPC surface:
``sitewhere-grpc-device-management/src/main/proto/device-management.proto`` (84 RPCs), all
implemented below as methods of :class:`DeviceManagement` (snake_case of the RPC names).

Registry changes are also published as a change feed (``device-model-updates``) so the GPU
inbound engine can mirror devices/assignments into HBM (new capability).
"""
from __future__ import annotations

import json
import logging
import threading

from ..core.errors import ErrorCode, NotFoundException, SiteWhereSystemException
from ..models.domain import (Area, AreaType, Customer, CustomerType, Device, DeviceAlarm, DeviceAlarmState,
                             DeviceAssignment, DeviceAssignmentStatus, DeviceCommand, DeviceElementMapping,
                             DeviceGroup, DeviceGroupElement, DeviceStatus, DeviceStream, DeviceType, SearchResults,
                             Zone, now_ms)
from ..persistence.query import Query
from ..persistence.store import EntityStore, create_store
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from .common import Crud


def _ids(v):
    return set(v or [])


class DeviceManagement:
    def __init__(self, store: EntityStore | None = None):
        s = self._store = store or create_store("memory")
        # indexed: the fields list / search criteria filter and sort on, pushed down into the store
        # (persistence/query.py; the reference's MongoDeviceManagement list* queries)
        self.device_types = Crud(s, "deviceTypes", DeviceType, ErrorCode.InvalidDeviceTypeToken, indexed=("name",))
        self.commands = Crud(s, "deviceCommands", DeviceCommand, ErrorCode.InvalidDeviceCommandToken,
                             indexed=("device_type_id",))
        self.statuses = Crud(s, "deviceStatuses", DeviceStatus, ErrorCode.InvalidDeviceStatusCode,
                             indexed=("device_type_id",))
        self.devices = Crud(s, "devices", Device, ErrorCode.InvalidDeviceToken,
                            indexed=("device_type_id", "device_assignment_id", "parent_device_id", "created_date"))
        self.assignments = Crud(s, "assignments", DeviceAssignment, ErrorCode.InvalidDeviceAssignmentToken,
                                indexed=("device_id", "device_type_id", "customer_id", "area_id", "asset_id", "status",
                                         "active_date"))
        self.groups = Crud(s, "deviceGroups", DeviceGroup, ErrorCode.InvalidDeviceGroupToken, indexed=("name",))
        self.group_elements = Crud(s, "deviceGroupElements", DeviceGroupElement, ErrorCode.InvalidDeviceGroupToken, (),
                                   indexed=("group_id",))
        self.streams = Crud(s, "deviceStreams", DeviceStream, ErrorCode.InvalidStreamId, indexed=("assignment_id",))
        self.alarms = Crud(s, "deviceAlarms", DeviceAlarm, ErrorCode.InvalidAlarmId,
                           indexed=("device_id", "device_assignment_id", "customer_id", "area_id", "asset_id",
                                    "triggering_event_id", "state", "triggered_date"))
        self.customer_types = Crud(s, "customerTypes", CustomerType, ErrorCode.InvalidCustomerTypeToken,
                                   indexed=("name",))
        self.customers = Crud(s, "customers", Customer, ErrorCode.InvalidCustomerToken,
                              indexed=("parent_customer_id", "customer_type_id", "name"))
        self.area_types = Crud(s, "areaTypes", AreaType, ErrorCode.InvalidAreaTypeToken, indexed=("name",))
        self.areas = Crud(s, "areas", Area, ErrorCode.InvalidAreaToken, indexed=("parent_area_id", "area_type_id", "name"))
        self.zones = Crud(s, "zones", Zone, ErrorCode.InvalidZoneToken, indexed=("area_id", "name"))
        self._listeners = []
        self._lock = threading.RLock()

    # ------------------------------------------------------------------ change feed
    def _add_listener(self, cb, many=None):
        """``cb(kind, entity)`` per change; ``many(kind, entities)``, when given, takes a bulk
        operation's changes at once (one change-feed publish, one durable add)."""
        self._listeners.append((cb, many))

    def _emit(self, kind: str, entity):
        self._emit_many(kind, [entity])

    def _emit_many(self, kind: str, entities: list):
        if not entities:
            return
        for cb, many in list(self._listeners):
            try:
                if many is not None and len(entities) > 1:
                    many(kind, entities)
                else:
                    for e in entities:
                        cb(kind, e)
            except Exception:   # one listener must not block the others; make the failure visible
                logging.getLogger(__name__).warning("device-model listener failed on %s", kind, exc_info=True)

    # ================================================================== device types
    def create_device_type(self, request: dict) -> DeviceType:
        t = self.device_types.create(request)
        self._emit("deviceType.created", t)
        return t

    def get_device_type(self, id: str) -> DeviceType | None:
        return self.device_types.get(id)

    def get_device_type_by_token(self, token: str) -> DeviceType | None:
        return self.device_types.get_by_token(token)

    def update_device_type(self, id: str, request: dict) -> DeviceType:
        return self.device_types.update(id, request)

    def list_device_types(self, criteria=None) -> SearchResults:
        return self.device_types.search(Query().order("name"), criteria)

    def delete_device_type(self, id: str) -> DeviceType:
        if self.devices.s.find(self.devices.c, Query(limit=1).eq("device_type_id", id))[0]:
            raise SiteWhereSystemException(ErrorCode.DeviceTypeInUse, detail=id)
        return self.device_types.delete(id)

    # ================================================================== commands
    def create_device_command(self, request: dict) -> DeviceCommand:
        dt = self._device_type_from(request)
        ns, name = request.get("namespace", ""), request.get("name", "")
        if any(c.namespace == ns and c.name == name for c in self.commands.query(lambda c: c.device_type_id == dt.id)):
            raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=f"command {ns}:{name} exists")
        return self.commands.create(request, device_type_id=dt.id)

    def get_device_command(self, id: str):
        return self.commands.get(id)

    def get_device_command_by_token(self, token: str):
        return self.commands.get_by_token(token)

    def update_device_command(self, id: str, request: dict):
        return self.commands.update(id, request)

    def list_device_commands(self, criteria=None):
        c = criteria or {}
        dt = c.get("deviceTypeId") if isinstance(c, dict) else None
        if isinstance(c, dict) and c.get("deviceTypeToken"):
            dt = self.device_types.require_token(c["deviceTypeToken"]).id
        return self.commands.search(Query().eq("device_type_id", dt).order("namespace").order("name"), c)

    def delete_device_command(self, id: str):
        return self.commands.delete(id)

    # ================================================================== statuses
    def create_device_status(self, request: dict) -> DeviceStatus:
        dt = self._device_type_from(request)
        code = request.get("code")
        if any(s.code == code for s in self.statuses.query(lambda s: s.device_type_id == dt.id)):
            raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=f"status code {code} exists")
        return self.statuses.create(request, device_type_id=dt.id)

    def get_device_status(self, id: str):
        return self.statuses.get(id)

    def get_device_status_by_token(self, token: str):
        return self.statuses.get_by_token(token)

    def update_device_status(self, id: str, request: dict):
        return self.statuses.update(id, request)

    def list_device_statuses(self, criteria=None):
        c = criteria or {}
        dt = c.get("deviceTypeId") if isinstance(c, dict) else None
        if isinstance(c, dict) and c.get("deviceTypeToken"):
            dt = self.device_types.require_token(c["deviceTypeToken"]).id
        code = c.get("code") if isinstance(c, dict) else None
        return self.statuses.search(Query().eq("device_type_id", dt).eq("code", code).order("code"), c)

    def delete_device_status(self, id: str):
        return self.statuses.delete(id)

    # ================================================================== devices
    def _device_type_from(self, request: dict) -> DeviceType:
        if request.get("deviceTypeId"):
            return self.device_types.require(request["deviceTypeId"])
        tok = request.get("deviceTypeToken")
        if not tok:
            raise SiteWhereSystemException(ErrorCode.IncompleteData, detail="device type required")
        return self.device_types.require_token(tok)

    def _new_device(self, request: dict) -> Device:
        dt = self._device_type_from(request)
        parent = None
        if request.get("parentDeviceToken"):
            parent = self.devices.require_token(request["parentDeviceToken"]).id
        maps = [DeviceElementMapping.from_dict(m) if isinstance(m, dict) else m
                for m in request.get("deviceElementMappings", [])]
        return self.devices.create({k: v for k, v in request.items() if k != "deviceElementMappings"},
                                   device_type_id=dt.id, parent_device_id=parent, device_element_mappings=maps,
                                   device_assignment_id=None)

    def create_device(self, request: dict) -> Device:
        d = self._new_device(request)
        self._emit("device.created", d)
        return d

    def create_devices(self, requests: list) -> list:
        """Bulk device creation (fleet provisioning; an extension of the reference's one-at-a-time
        ``createDevice``): the same validation per device, then ONE change-feed publish for the batch
        (engine tenants register the whole batch in one table upload).  A request that fails
        validation stops the batch; the devices before it are created and announced.  Returns the
        new devices' ids (not the entities: a bulk call's reply stays small)."""
        out = []
        try:
            for r in requests:
                out.append(self._new_device(r))
        finally:
            self._emit_many("device.created", out)
        return [d.id for d in out]

    def get_device(self, id: str):
        return self.devices.get(id)

    def get_device_by_token(self, token: str):
        return self.devices.get_by_token(token)

    def get_devices(self, ids: list) -> list:
        """Devices by id, in order (None where unknown): one call for a consumer's poll batch."""
        return [self.devices.get(i) if i else None for i in ids]

    def get_devices_by_tokens(self, tokens: list) -> list:
        """Devices by token, in order (None where unknown)."""
        return [self.devices.get_by_token(t) if t else None for t in tokens]

    def update_device(self, id: str, request: dict) -> Device:
        fixed = {}
        if request.get("deviceTypeToken") or request.get("deviceTypeId"):
            fixed["device_type_id"] = self._device_type_from(request).id
        if "parentDeviceToken" in request:
            tok = request["parentDeviceToken"]
            if tok:
                pid = self.devices.require_token(tok).id
                self._check_cycle(id, pid)
                fixed["parent_device_id"] = pid
            else:
                fixed["parent_device_id"] = None
        req = {k: v for k, v in request.items() if k not in ("deviceAssignmentId", "deviceTypeToken", "parentDeviceToken")}
        d = self.devices.update(id, req, **fixed)
        self._emit("device.updated", d)
        return d

    def _check_cycle(self, child: str, parent: str):
        seen = set()
        cur = parent
        while cur:
            if cur == child or cur in seen:
                raise SiteWhereSystemException(ErrorCode.DeviceParentCycle, detail=child)
            seen.add(cur)
            p = self.devices.get(cur)
            cur = p.parent_device_id if p else None

    def list_devices(self, criteria=None) -> SearchResults:
        c = criteria or {}
        dt = c.get("deviceTypeId") if isinstance(c, dict) else None
        if isinstance(c, dict) and c.get("deviceTypeToken"):
            dt = self.device_types.require_token(c["deviceTypeToken"]).id
        excl = bool(c.get("excludeAssigned")) if isinstance(c, dict) else False
        after = c.get("createdAfter") if isinstance(c, dict) else None
        before = c.get("createdBefore") if isinstance(c, dict) else None
        q = Query().eq("device_type_id", dt).gte("created_date", after or None).lte("created_date", before or None)
        if excl:
            q.null("device_assignment_id")
        return self.devices.search(q.order("created_date", True).order("token", True), c)

    def create_device_element_mapping(self, device_id: str, mapping) -> Device:
        """Nest a child device under a path of the parent's element schema (reference NestedDeviceSupport)."""
        m = DeviceElementMapping.from_dict(mapping) if isinstance(mapping, dict) else mapping
        d = self.devices.require(device_id)
        if any(x.device_element_schema_path == m.device_element_schema_path for x in d.device_element_mappings):
            raise SiteWhereSystemException(ErrorCode.DeviceElementMappingExists, detail=m.device_element_schema_path)
        child = self.devices.require_token(m.device_token)
        self._check_cycle(child.id, d.id)
        d.device_element_mappings.append(m)
        child.parent_device_id = d.id
        self.devices.put(child)
        return self.devices.put(d)

    def delete_device_element_mapping(self, device_id: str, path: str) -> Device:
        d = self.devices.require(device_id)
        keep = [m for m in d.device_element_mappings if m.device_element_schema_path != path]
        if len(keep) == len(d.device_element_mappings):
            raise NotFoundException(ErrorCode.InvalidDeviceElementPath, path)
        gone = [m for m in d.device_element_mappings if m.device_element_schema_path == path][0]
        child = self.devices.get_by_token(gone.device_token)
        if child is not None and child.parent_device_id == d.id:
            child.parent_device_id = None
            self.devices.put(child)
        d.device_element_mappings = keep
        return self.devices.put(d)

    def delete_device(self, id: str) -> Device:
        d = self.devices.require(id)
        a = self.assignments.get(d.device_assignment_id) if d.device_assignment_id else None
        if a is not None and a.status == DeviceAssignmentStatus.Active:
            raise SiteWhereSystemException(ErrorCode.DeviceAlreadyAssigned, detail="end the assignment first")
        self.devices.delete(id)
        self._emit("device.deleted", d)
        return d

    # ================================================================== groups
    def create_device_group(self, request: dict):
        return self.groups.create(request)

    def get_device_group(self, id: str):
        return self.groups.get(id)

    def get_device_group_by_token(self, token: str):
        return self.groups.get_by_token(token)

    def update_device_group(self, id: str, request: dict):
        return self.groups.update(id, request)

    def list_device_groups(self, criteria=None):
        return self.groups.search(Query().order("name"), criteria)

    def list_device_groups_with_role(self, role: str, criteria=None):
        return self.groups.list(criteria, lambda g: role in g.roles, sort=lambda g: g.name)

    def delete_device_group(self, id: str):
        g = self.groups.delete(id)
        for e in self.group_elements.query(lambda e: e.group_id == id):
            self._store.delete("deviceGroupElements", e.id)
        return g

    def add_device_group_elements(self, group_id: str, elements: list, ignore_duplicates: bool = True):
        self.groups.require(group_id)
        out = []
        existing = {(e.device_id, e.nested_group_id) for e in self.group_elements.query(lambda e: e.group_id == group_id)}
        for req in elements:
            dev = self.devices.require_token(req["deviceToken"]).id if req.get("deviceToken") else None
            nested = self.groups.require_token(req["nestedGroupToken"]).id if req.get("nestedGroupToken") else None
            if (dev, nested) in existing:
                if ignore_duplicates:
                    continue
                raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail="group element exists")
            e = DeviceGroupElement(group_id=group_id, device_id=dev, nested_group_id=nested,
                                   roles=list(req.get("roles", [])))
            self._store.put("deviceGroupElements", e)
            existing.add((dev, nested))
            out.append(e)
        return out

    def remove_device_group_elements(self, element_ids: list[str]):
        out = []
        for i in element_ids:
            e = self._store.delete("deviceGroupElements", i)
            if e is not None:
                out.append(e)
        return out

    def list_device_group_elements(self, group_id: str, criteria=None):
        self.groups.require(group_id)
        return self.group_elements.search(Query().eq("group_id", group_id).order("id"), criteria)

    def expand_group_devices(self, group_id: str, roles: list[str] | None = None) -> list[str]:
        """Device ids of a group, recursing into nested groups (reference GroupUtils)."""
        out, seen, stack = [], set(), [group_id]
        while stack:
            g = stack.pop()
            if g in seen:
                continue
            seen.add(g)
            for e in self.group_elements.query(lambda e, g=g: e.group_id == g):
                if roles and not (set(roles) & set(e.roles)):
                    continue
                if e.device_id:
                    out.append(e.device_id)
                if e.nested_group_id:
                    stack.append(e.nested_group_id)
        return sorted(set(out))

    # ================================================================== assignments
    def create_device_assignment(self, request: dict) -> DeviceAssignment:
        with self._lock:
            a = self._new_assignment(request)
        self._emit("assignment.created", a)
        return a

    def create_device_assignments(self, requests: list, record_state_changes: bool = True) -> list:
        """Bulk assignment creation (see :meth:`create_devices`): one change-feed publish and ONE
        durable add of the assignments' state-change events for the batch.  ``record_state_changes``
        False: an import of assignments whose activation already happened elsewhere (a fleet
        migrated from another system) -- no "assignment Active" state-change event is recorded.
        Returns the new assignments' ids."""
        out = []
        try:
            with self._lock:
                for r in requests:
                    out.append(self._new_assignment(r))
        finally:
            self._emit_many("assignment.created" if record_state_changes else "assignment.imported", out)
        return [a.id for a in out]

    def _new_assignment(self, request: dict) -> DeviceAssignment:
        """Validate and store one assignment (caller holds the lock; the caller announces it)."""
        d = (self.devices.require(request["deviceId"]) if request.get("deviceId")
             else self.devices.require_token(request.get("deviceToken")))
        if d.device_assignment_id:
            cur = self.assignments.get(d.device_assignment_id)
            if cur is not None and cur.status != DeviceAssignmentStatus.Released:
                raise SiteWhereSystemException(ErrorCode.DeviceAlreadyAssigned, detail=d.token)
        fixed = dict(device_id=d.id, device_type_id=d.device_type_id,
                     status=DeviceAssignmentStatus(request.get("status", "Active")),
                     active_date=now_ms(), released_date=None,
                     customer_id=self._opt_token(self.customers, request.get("customerToken"), request.get("customerId")),
                     area_id=self._opt_token(self.areas, request.get("areaToken"), request.get("areaId")),
                     asset_id=request.get("assetId") or None)
        if request.get("assetToken"):
            fixed["asset_id"] = request["assetToken"]  # resolved by the asset service (reference: token ref)
        req = {k: v for k, v in request.items() if k in ("token", "metadata")}
        a = self.assignments.create(req, **fixed)
        d.device_assignment_id = a.id
        self.devices.put(d)
        return a

    def _opt_token(self, crud, token, id_):
        if token:
            return crud.require_token(token).id
        return id_ or None

    def get_device_assignment(self, id: str):
        return self.assignments.get(id)

    def get_device_assignments(self, ids: list) -> list:
        """Assignments by id, in order (None where unknown)."""
        return [self.assignments.get(i) if i else None for i in ids]

    def get_device_assignment_by_token(self, token: str):
        return self.assignments.get_by_token(token)

    def get_current_assignment_for_device(self, device_id: str):
        d = self.devices.require(device_id)
        return self.assignments.get(d.device_assignment_id) if d.device_assignment_id else None

    def delete_device_assignment(self, id: str):
        a = self.assignments.delete(id)
        d = self.devices.get(a.device_id)
        if d is not None and d.device_assignment_id == id:
            d.device_assignment_id = None
            self.devices.put(d)
        self._emit("assignment.deleted", a)
        return a

    def update_device_assignment(self, id: str, request: dict):
        fixed = {}
        if "customerToken" in request:
            fixed["customer_id"] = self._opt_token(self.customers, request["customerToken"], None)
        if "areaToken" in request:
            fixed["area_id"] = self._opt_token(self.areas, request["areaToken"], None)
        if "assetToken" in request:
            fixed["asset_id"] = request["assetToken"]
        req = {k: v for k, v in request.items() if k in ("metadata", "status", "token")}
        a = self.assignments.update(id, req, **fixed)
        self._emit("assignment.updated", a)
        return a

    def list_device_assignments(self, criteria=None):
        c = criteria or {}
        st = c.get("status") if isinstance(c, dict) else None
        dev = c.get("deviceId") if isinstance(c, dict) else None
        # reference criteria carry id lists (DeviceAssignmentSearchCriteria); REST / client filters
        # name one entity (customerId, areaId, ...) -- both narrow the result
        q = Query().eq("status", st or None).eq("device_id", dev or None)
        for k, f in (("deviceTypeId", "device_type_id"), ("customerId", "customer_id"), ("areaId", "area_id"),
                     ("assetId", "asset_id")):
            # reference criteria carry id lists (DeviceAssignmentSearchCriteria); REST / client
            # filters name one entity (customerId, areaId, ...) -- both narrow the result
            ids = (_ids(c.get(k + "s")) | ({c[k]} if c.get(k) else set())) if isinstance(c, dict) else set()
            if ids:
                q.in_(f, sorted(ids))
        return self.assignments.search(q.order("active_date", True).order("id", True), c)

    def end_device_assignment(self, id: str):
        with self._lock:
            a = self.assignments.require(id)
            a.status = DeviceAssignmentStatus.Released
            a.released_date = now_ms()
            self.assignments.put(a)
            d = self.devices.get(a.device_id)
            if d is not None and d.device_assignment_id == id:
                d.device_assignment_id = None
                self.devices.put(d)
        self._emit("assignment.ended", a)
        return a

    def mark_assignment_missing(self, id: str):
        a = self.assignments.require(id)
        a.status = DeviceAssignmentStatus.Missing
        self.assignments.put(a)
        self._emit("assignment.updated", a)
        return a

    # ================================================================== streams
    def create_device_stream(self, assignment_id: str, request: dict) -> DeviceStream:
        self.assignments.require(assignment_id)
        sid = request.get("streamId")
        if any(s.stream_id == sid for s in self.streams.query(lambda s: s.assignment_id == assignment_id)):
            raise SiteWhereSystemException(ErrorCode.DuplicateStreamId, detail=sid)
        return self.streams.create(request, assignment_id=assignment_id)

    def get_device_stream_by_stream_id(self, assignment_id: str, stream_id: str):
        r = self.streams.query(lambda s: s.assignment_id == assignment_id and s.stream_id == stream_id)
        return r[0] if r else None

    def list_device_streams(self, assignment_id: str, criteria=None):
        return self.streams.search(Query().eq("assignment_id", assignment_id).order("stream_id"), criteria)

    # ================================================================== alarms
    def create_device_alarm(self, request: dict) -> DeviceAlarm:
        a = self.assignments.require(request["deviceAssignmentId"]) if request.get("deviceAssignmentId") else None
        fixed = {"triggered_date": now_ms(), "state": DeviceAlarmState(request.get("state", "Triggered"))}
        if a is not None:
            fixed.update(device_id=a.device_id, customer_id=a.customer_id, area_id=a.area_id, asset_id=a.asset_id)
        return self.alarms.create(request, **fixed)

    def get_device_alarm(self, id: str):
        return self.alarms.get(id)

    def update_device_alarm(self, id: str, request: dict):
        al = self.alarms.require(id)
        st = request.get("state")
        fixed = {}
        if st and st != al.state.value:
            if st == "Acknowledged":
                fixed["acknowledged_date"] = now_ms()
            if st == "Resolved":
                fixed["resolved_date"] = now_ms()
        return self.alarms.update(id, request, **fixed)

    def search_device_alarms(self, criteria=None):
        c = criteria or {}
        keys = {"deviceId": "device_id", "deviceAssignmentId": "device_assignment_id", "customerId": "customer_id",
                "areaId": "area_id", "assetId": "asset_id", "triggeringEventId": "triggering_event_id"}
        q = Query()
        for k, f in keys.items():
            if isinstance(c, dict) and c.get(k):
                q.eq(f, c[k])
        st = c.get("state") if isinstance(c, dict) else None
        return self.alarms.search(q.eq("state", st or None).order("triggered_date", True), c)

    def delete_device_alarm(self, id: str):
        return self.alarms.delete(id)

    # ================================================================== customers
    def create_customer_type(self, request: dict):
        ids = [self.customer_types.require_token(t).id for t in request.get("containedCustomerTypeTokens", [])]
        return self.customer_types.create({k: v for k, v in request.items() if k != "containedCustomerTypeTokens"},
                                          contained_customer_type_ids=ids)

    def get_customer_type(self, id: str):
        return self.customer_types.get(id)

    def get_customer_type_by_token(self, token: str):
        return self.customer_types.get_by_token(token)

    def update_customer_type(self, id: str, request: dict):
        fixed = {}
        if "containedCustomerTypeTokens" in request:
            fixed["contained_customer_type_ids"] = [self.customer_types.require_token(t).id
                                                    for t in request["containedCustomerTypeTokens"]]
        return self.customer_types.update(id, {k: v for k, v in request.items()
                                               if k != "containedCustomerTypeTokens"}, **fixed)

    def list_customer_types(self, criteria=None):
        return self.customer_types.search(Query().order("name"), criteria)

    def delete_customer_type(self, id: str):
        return self.customer_types.delete(id)

    def create_customer(self, request: dict):
        ct = self.customer_types.require_token(request["customerTypeToken"]).id if request.get("customerTypeToken") else None
        parent = self.customers.require_token(request["parentCustomerToken"]).id if request.get("parentCustomerToken") else None
        return self.customers.create(request, customer_type_id=ct, parent_customer_id=parent)

    def get_customer(self, id: str):
        return self.customers.get(id)

    def get_customer_by_token(self, token: str):
        return self.customers.get_by_token(token)

    def get_customer_children(self, token: str) -> list:
        p = self.customers.require_token(token)
        return self.customers.query(lambda c: c.parent_customer_id == p.id, sort=lambda c: c.name)

    def update_customer(self, id: str, request: dict):
        fixed = {}
        if request.get("customerTypeToken"):
            fixed["customer_type_id"] = self.customer_types.require_token(request["customerTypeToken"]).id
        if "parentCustomerToken" in request:
            fixed["parent_customer_id"] = (self.customers.require_token(request["parentCustomerToken"]).id
                                           if request["parentCustomerToken"] else None)
        return self.customers.update(id, request, **fixed)

    def list_customers(self, criteria=None):
        c = criteria or {}
        root = bool(c.get("rootOnly")) if isinstance(c, dict) else False
        parent = c.get("parentCustomerId") if isinstance(c, dict) else None
        ct = c.get("customerTypeId") if isinstance(c, dict) else None
        q = Query().eq("parent_customer_id", parent or None).eq("customer_type_id", ct or None)
        if root:
            q.null("parent_customer_id")
        return self.customers.search(q.order("name"), c)

    def delete_customer(self, id: str):
        return self.customers.delete(id)

    def get_customers_tree(self) -> list[dict]:
        return _tree(self.customers.query(sort=lambda e: e.name), "parent_customer_id")

    # ================================================================== areas
    def create_area_type(self, request: dict):
        ids = [self.area_types.require_token(t).id for t in request.get("containedAreaTypeTokens", [])]
        return self.area_types.create({k: v for k, v in request.items() if k != "containedAreaTypeTokens"},
                                      contained_area_type_ids=ids)

    def get_area_type(self, id: str):
        return self.area_types.get(id)

    def get_area_type_by_token(self, token: str):
        return self.area_types.get_by_token(token)

    def update_area_type(self, id: str, request: dict):
        fixed = {}
        if "containedAreaTypeTokens" in request:
            fixed["contained_area_type_ids"] = [self.area_types.require_token(t).id
                                                for t in request["containedAreaTypeTokens"]]
        return self.area_types.update(id, {k: v for k, v in request.items() if k != "containedAreaTypeTokens"}, **fixed)

    def list_area_types(self, criteria=None):
        return self.area_types.search(Query().order("name"), criteria)

    def delete_area_type(self, id: str):
        return self.area_types.delete(id)

    def create_area(self, request: dict):
        at = self.area_types.require_token(request["areaTypeToken"]).id if request.get("areaTypeToken") else None
        parent = self.areas.require_token(request["parentAreaToken"]).id if request.get("parentAreaToken") else None
        return self.areas.create(request, area_type_id=at, parent_area_id=parent)

    def get_area(self, id: str):
        return self.areas.get(id)

    def get_area_by_token(self, token: str):
        return self.areas.get_by_token(token)

    def get_area_children(self, token: str) -> list:
        p = self.areas.require_token(token)
        return self.areas.query(lambda a: a.parent_area_id == p.id, sort=lambda a: a.name)

    def update_area(self, id: str, request: dict):
        fixed = {}
        if request.get("areaTypeToken"):
            fixed["area_type_id"] = self.area_types.require_token(request["areaTypeToken"]).id
        if "parentAreaToken" in request:
            fixed["parent_area_id"] = (self.areas.require_token(request["parentAreaToken"]).id
                                       if request["parentAreaToken"] else None)
        return self.areas.update(id, request, **fixed)

    def list_areas(self, criteria=None):
        c = criteria or {}
        root = bool(c.get("rootOnly")) if isinstance(c, dict) else False
        parent = c.get("parentAreaId") if isinstance(c, dict) else None
        at = c.get("areaTypeId") if isinstance(c, dict) else None
        q = Query().eq("parent_area_id", parent or None).eq("area_type_id", at or None)
        if root:
            q.null("parent_area_id")
        return self.areas.search(q.order("name"), c)

    def delete_area(self, id: str):
        return self.areas.delete(id)

    def get_areas_tree(self) -> list[dict]:
        return _tree(self.areas.query(sort=lambda e: e.name), "parent_area_id")

    # ================================================================== zones
    def create_zone(self, request: dict):
        area = self.areas.require_token(request["areaToken"]).id if request.get("areaToken") else request.get("areaId")
        z = self.zones.create(request, area_id=area)
        self._emit("zone.created", z)
        return z

    def get_zone(self, id: str):
        return self.zones.get(id)

    def get_zone_by_token(self, token: str):
        return self.zones.get_by_token(token)

    def update_zone(self, id: str, request: dict):
        z = self.zones.update(id, request)
        self._emit("zone.updated", z)
        return z

    def list_zones(self, criteria=None):
        c = criteria or {}
        area = c.get("areaId") if isinstance(c, dict) else None
        if isinstance(c, dict) and c.get("areaToken"):
            area = self.areas.require_token(c["areaToken"]).id
        return self.zones.search(Query().eq("area_id", area or None).order("name"), c)

    def delete_zone(self, id: str):
        z = self.zones.delete(id)
        self._emit("zone.deleted", z)
        return z


def _tree(items, parent_field: str) -> list[dict]:
    by_parent: dict = {}
    for e in items:
        by_parent.setdefault(getattr(e, parent_field), []).append(e)

    def build(pid):
        return [{"id": e.id, "token": e.token, "name": e.name, "children": build(e.id)} for e in by_parent.get(pid, [])]
    return build(None)


class DeviceManagementTriggers:
    """State-change events on assignment create/end (reference DeviceManagementTriggers.java:30-80)."""

    def __init__(self, dm: DeviceManagement, event_api_factory):
        self.dm = dm
        self.events = event_api_factory
        dm._add_listener(self._on_change, self._on_changes)

    @staticmethod
    def _state_change(kind) -> dict:
        return {"attribute": "assignment", "type": "automated",
                "previousState": None if kind == "assignment.created" else "Active",
                "newState": "Active" if kind == "assignment.created" else "Released"}

    def _on_changes(self, kind, entities):
        """A bulk operation's assignments: their state changes in one durable add."""
        if kind not in ("assignment.created", "assignment.ended"):
            return
        try:
            api = self.events()
            if api is None:
                return
            if hasattr(api, "add_event_batch"):
                api.add_event_batch([(e.id, "StateChange", self._state_change(kind)) for e in entities],
                                    assignments=entities)
            else:
                for e in entities:
                    api.add_state_changes(e.id, self._state_change(kind))
        except Exception:
            logging.getLogger(__name__).warning("assignment state-change events for %s not recorded", kind,
                                                exc_info=True)

    def _on_change(self, kind, e):
        if kind not in ("assignment.created", "assignment.ended"):
            return
        try:
            api = self.events()
            if api is None:
                return
            api.add_state_changes(e.id, {"attribute": "assignment", "type": "automated",
                                         "previousState": None if kind == "assignment.created" else "Active",
                                         "newState": "Active" if kind == "assignment.created" else "Released"})
        except Exception:
            logging.getLogger(__name__).warning("assignment state-change event for %s not recorded", kind,
                                                exc_info=True)


class DeviceManagementTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ds = self.config.get("datastore", {"type": "memory"})
        store = create_store(ds.get("type", "memory"), **{k: v for k, v in ds.items() if k != "type"})
        self.management = DeviceManagement(store)
        self.management._add_listener(self._publish_change, self._publish_changes)
        self.triggers = DeviceManagementTriggers(
            self.management, lambda: self.ms.api("DeviceEventManagement", self.tenant.token)
            if "DeviceEventManagement" in self.ms.instance.resolver.names() else None)
        self.api = {"DeviceManagement": self.management}

    def _publish_change(self, kind, entity):
        topic = self.ms.instance.naming.tenant_prefix(self.tenant.token) + "device-model-updates"
        from ..rpc import codec
        self.ms.producer.send(topic, getattr(entity, "token", None) or entity.id,
                              json.dumps({"kind": kind, "entity": codec.to_wire(entity)}).encode())

    # entities per bulk change record (a bulk create of 1M devices is ~250 records, not 1M)
    BULK_RECORD = 4096

    def _publish_changes(self, kind, entities):
        """A bulk operation's changes as ``{"kind": "bulk", "of": kind, "entities": [...]}`` records
        (consumers expand them, ``inbound_processing.model_changes``): one record per entity made every
        consumer decode and dispatch a million records for a fleet provisioning."""
        topic = self.ms.instance.naming.tenant_prefix(self.tenant.token) + "device-model-updates"
        from ..rpc import codec
        n = self.BULK_RECORD
        self.ms.producer.send_batch(topic, [
            (f"bulk-{kind}-{i}", json.dumps({"kind": "bulk", "of": kind,
                                            "entities": [codec.to_wire(e) for e in entities[i:i + n]]}).encode())
            for i in range(0, len(entities), n)])

    def tenant_bootstrap(self, dataset_template, monitor):
        from .builders import DeviceBuilder, EventBuilder
        from .dataset_runner import run_initializers
        token = self.tenant.token
        run_initializers(self, "deviceManagement", dataset_template, {
            "device_builder": DeviceBuilder(self.management, self.ms.logger),
            "event_builder": EventBuilder(lambda: self.ms.api("DeviceEventManagement", token), self.management,
                                          logger=self.ms.logger)})


class DeviceManagementMicroservice(MultitenantMicroservice):
    identifier = "device-management"
    name = "Device Management"

    def service_names(self):
        return ["DeviceManagement"]

    def create_tenant_engine(self, tenant):
        return DeviceManagementTenantEngine(self, tenant)
