"""Domain model: every persistent entity and event of the platform (L0 contracts).

Field parity with ``sitewhere-core-api/.../spi/**`` and ``rest/model/**`` (e.g. ``IDevice``,
``IDeviceAssignment``, ``IDeviceType``...) as serialized by the protobuf messages in
``sitewhere-grpc-*/src/main/proto/*-model.proto``.  JSON uses the reference's camelCase names.
"""
from __future__ import annotations

import dataclasses
import functools
import enum
import re
import time
from dataclasses import dataclass, field
from typing import get_type_hints
from ..utils import fast_uuid4

_camel_re = re.compile(r"_([a-z0-9])")


@functools.lru_cache(maxsize=4096)
def camel(s: str) -> str:
    return _camel_re.sub(lambda m: m.group(1).upper(), s)


@functools.lru_cache(maxsize=4096)
def snake(s: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", s).lower()


_field_cache: dict = {}


def _fields(cls):
    """(name, camelName) per dataclass field, computed once per class."""
    f = _field_cache.get(cls)
    if f is None:
        f = _field_cache[cls] = tuple((x.name, camel(x.name)) for x in dataclasses.fields(cls))
    return f


def now_ms() -> int:
    return int(time.time() * 1000)


def new_id() -> str:
    return fast_uuid4()


class Model:
    """Mixin: camelCase dict (de)serialization for dataclasses."""

    def to_dict(self) -> dict:
        return {c: _ser(getattr(self, n)) for n, c in _fields(type(self))}

    @classmethod
    def from_dict(cls, d: dict | None):
        if d is None:
            return None
        hints = _hints(cls)
        kw = {}
        names = _names(cls)
        for k, v in d.items():
            n = snake(k) if k not in names else k
            if n in names:
                kw[n] = _deser(hints.get(n), v)
        return cls(**kw)

    def copy(self, **changes):
        return dataclasses.replace(self, **changes)


_hint_cache: dict = {}
_names_cache: dict = {}


def _names(cls) -> frozenset:
    n = _names_cache.get(cls)
    if n is None:
        n = _names_cache[cls] = frozenset(x.name for x in dataclasses.fields(cls))
    return n


def _hints(cls):
    h = _hint_cache.get(cls)
    if h is None:
        h = get_type_hints(cls)
        _hint_cache[cls] = h
    return h


_PLAIN = (str, int, float, bool, type(None))


def _ser(v):
    if type(v) in _PLAIN:
        return v
    if isinstance(v, Model):
        return v.to_dict()
    if isinstance(v, enum.Enum):
        return v.value
    if isinstance(v, (list, tuple)):
        return [_ser(x) for x in v]
    if isinstance(v, dict):
        return {k: _ser(x) for k, x in v.items()}
    return v


def _deser(t, v):
    if v is None or t is None:
        return v
    origin = getattr(t, "__origin__", None)
    args = getattr(t, "__args__", ())
    if origin is list and args:
        return [_deser(args[0], x) for x in v]
    if origin is dict:
        return dict(v)
    if origin is not None and type(None) in args:  # Optional[X]
        inner = [a for a in args if a is not type(None)]
        return _deser(inner[0], v) if inner else v
    if isinstance(t, type):
        if issubclass(t, Model) and isinstance(v, dict):
            return t.from_dict(v)
        if issubclass(t, enum.Enum):
            return t(v)
    return v


# ============================================================================ base entities
@dataclass
class PersistentEntity(Model):
    id: str = field(default_factory=new_id)
    token: str | None = None
    created_date: int | None = None
    created_by: str | None = None
    updated_date: int | None = None
    updated_by: str | None = None
    metadata: dict = field(default_factory=dict)


@dataclass
class BrandedEntity(PersistentEntity):
    image_url: str | None = None
    icon: str | None = None
    background_color: str | None = None
    foreground_color: str | None = None
    border_color: str | None = None


@dataclass
class Location(Model):
    latitude: float = 0.0
    longitude: float = 0.0
    elevation: float | None = None


@dataclass
class SearchCriteria(Model):
    page_number: int = 1
    page_size: int = 100     # 0 = all

    def slice(self, items: list) -> list:
        if self.page_size <= 0:
            return items
        start = (max(1, self.page_number) - 1) * self.page_size
        return items[start:start + self.page_size]


@dataclass
class DateRangeSearchCriteria(SearchCriteria):
    start_date: int | None = None
    end_date: int | None = None


@dataclass
class SearchResults(Model):
    num_results: int = 0
    results: list = field(default_factory=list)

    def to_dict(self) -> dict:
        return {"numResults": self.num_results, "results": [_ser(r) for r in self.results]}


# ============================================================================ device management
class DeviceContainerPolicy(str, enum.Enum):
    Standalone = "Standalone"
    Composite = "Composite"


@dataclass
class DeviceSlot(Model):
    name: str = ""
    path: str = ""


@dataclass
class DeviceUnit(Model):
    name: str = ""
    path: str = ""
    device_units: list["DeviceUnit"] = field(default_factory=list)
    device_slots: list[DeviceSlot] = field(default_factory=list)


@dataclass
class DeviceElementSchema(Model):
    device_units: list[DeviceUnit] = field(default_factory=list)
    device_slots: list[DeviceSlot] = field(default_factory=list)


@dataclass
class DeviceType(BrandedEntity):
    name: str = ""
    description: str = ""
    container_policy: DeviceContainerPolicy = DeviceContainerPolicy.Standalone
    device_element_schema: DeviceElementSchema | None = None


class ParameterType(str, enum.Enum):
    Double = "Double"
    Float = "Float"
    Int32 = "Int32"
    Int64 = "Int64"
    UInt32 = "UInt32"
    UInt64 = "UInt64"
    SInt32 = "SInt32"
    SInt64 = "SInt64"
    Fixed32 = "Fixed32"
    Fixed64 = "Fixed64"
    SFixed32 = "SFixed32"
    SFixed64 = "SFixed64"
    Bool = "Bool"
    String = "String"
    Bytes = "Bytes"


@dataclass
class CommandParameter(Model):
    name: str = ""
    type: ParameterType = ParameterType.String
    required: bool = False


@dataclass
class DeviceCommand(PersistentEntity):
    device_type_id: str | None = None
    namespace: str = ""
    name: str = ""
    description: str = ""
    parameters: list[CommandParameter] = field(default_factory=list)


@dataclass
class DeviceStatus(PersistentEntity):
    device_type_id: str | None = None
    code: str = ""
    name: str = ""
    background_color: str | None = None
    foreground_color: str | None = None
    border_color: str | None = None
    icon: str | None = None


@dataclass
class DeviceElementMapping(Model):
    device_element_schema_path: str = ""
    device_token: str = ""


@dataclass
class Device(PersistentEntity):
    device_type_id: str | None = None
    device_assignment_id: str | None = None
    parent_device_id: str | None = None
    device_element_mappings: list[DeviceElementMapping] = field(default_factory=list)
    comments: str | None = None
    status: str | None = None


class DeviceAssignmentStatus(str, enum.Enum):
    Active = "Active"
    Missing = "Missing"
    Released = "Released"


@dataclass
class DeviceAssignment(PersistentEntity):
    device_id: str | None = None
    device_type_id: str | None = None
    customer_id: str | None = None
    area_id: str | None = None
    asset_id: str | None = None
    status: DeviceAssignmentStatus = DeviceAssignmentStatus.Active
    active_date: int | None = None
    released_date: int | None = None


class DeviceAlarmState(str, enum.Enum):
    Triggered = "Triggered"
    Acknowledged = "Acknowledged"
    Resolved = "Resolved"


@dataclass
class DeviceAlarm(PersistentEntity):
    device_id: str | None = None
    device_assignment_id: str | None = None
    customer_id: str | None = None
    area_id: str | None = None
    asset_id: str | None = None
    alarm_message: str = ""
    triggering_event_id: str | None = None
    state: DeviceAlarmState = DeviceAlarmState.Triggered
    triggered_date: int | None = None
    acknowledged_date: int | None = None
    resolved_date: int | None = None


@dataclass
class DeviceGroup(BrandedEntity):
    name: str = ""
    description: str = ""
    roles: list[str] = field(default_factory=list)


@dataclass
class DeviceGroupElement(Model):
    id: str = field(default_factory=new_id)
    group_id: str | None = None
    device_id: str | None = None
    nested_group_id: str | None = None
    roles: list[str] = field(default_factory=list)


@dataclass
class DeviceStream(PersistentEntity):
    assignment_id: str | None = None
    stream_id: str = ""
    content_type: str = ""


@dataclass
class DeviceStreamData(Model):
    id: str = field(default_factory=new_id)
    device_assignment_id: str | None = None
    stream_id: str = ""
    sequence_number: int = 0
    data: bytes = b""
    event_date: int | None = None
    received_date: int | None = None

    def to_dict(self):
        d = super().to_dict()
        import base64
        d["data"] = base64.b64encode(self.data or b"").decode()
        return d

    @classmethod
    def from_dict(cls, d: dict | None):
        m = super().from_dict(d)
        if m is not None and isinstance(m.data, str):      # stored documents carry the chunk as base64
            import base64
            m.data = base64.b64decode(m.data)
        return m


@dataclass
class CustomerType(BrandedEntity):
    name: str = ""
    description: str = ""
    contained_customer_type_ids: list[str] = field(default_factory=list)


@dataclass
class Customer(BrandedEntity):
    customer_type_id: str | None = None
    parent_customer_id: str | None = None
    name: str = ""
    description: str = ""


@dataclass
class AreaType(BrandedEntity):
    name: str = ""
    description: str = ""
    contained_area_type_ids: list[str] = field(default_factory=list)


@dataclass
class Area(BrandedEntity):
    area_type_id: str | None = None
    parent_area_id: str | None = None
    name: str = ""
    description: str = ""
    bounds: list[Location] = field(default_factory=list)


@dataclass
class Zone(PersistentEntity):
    area_id: str | None = None
    name: str = ""
    bounds: list[Location] = field(default_factory=list)
    border_color: str | None = None
    fill_color: str | None = None
    opacity: float | None = None


@dataclass
class DeviceState(PersistentEntity):
    device_id: str | None = None
    device_type_id: str | None = None
    device_assignment_id: str | None = None
    customer_id: str | None = None
    area_id: str | None = None
    asset_id: str | None = None
    last_interaction_date: int | None = None
    presence_missing_date: int | None = None
    last_location_event_id: str | None = None
    last_measurement_event_ids: dict = field(default_factory=dict)
    last_alert_event_ids: dict = field(default_factory=dict)


# ============================================================================ assets
class AssetCategory(str, enum.Enum):
    Device = "Device"
    Person = "Person"
    Hardware = "Hardware"


@dataclass
class AssetType(BrandedEntity):
    name: str = ""
    description: str = ""
    asset_category: AssetCategory = AssetCategory.Device


@dataclass
class Asset(BrandedEntity):
    asset_type_id: str | None = None
    name: str = ""


# ============================================================================ events
class DeviceEventType(str, enum.Enum):
    Measurement = "Measurement"
    Location = "Location"
    Alert = "Alert"
    CommandInvocation = "CommandInvocation"
    CommandResponse = "CommandResponse"
    StateChange = "StateChange"


class AlertSource(str, enum.Enum):
    Device = "Device"
    System = "System"


class AlertLevel(str, enum.Enum):
    Info = "Info"
    Warning = "Warning"
    Error = "Error"
    Critical = "Critical"


ALERT_LEVEL_INDEX = {AlertLevel.Info: 0, AlertLevel.Warning: 1, AlertLevel.Error: 2, AlertLevel.Critical: 3}


class CommandInitiator(str, enum.Enum):
    REST = "REST"
    BatchOperation = "BatchOperation"
    Script = "Script"
    Scheduler = "Scheduler"


class CommandTarget(str, enum.Enum):
    Assignment = "Assignment"


class DeviceEventIndex(str, enum.Enum):
    Assignment = "Assignment"
    Customer = "Customer"
    Area = "Area"
    Asset = "Asset"


@dataclass
class DeviceEvent(Model):
    id: str = field(default_factory=new_id)
    alternate_id: str | None = None
    event_type: DeviceEventType = DeviceEventType.Measurement
    device_id: str | None = None
    device_assignment_id: str | None = None
    customer_id: str | None = None
    area_id: str | None = None
    asset_id: str | None = None
    event_date: int | None = None
    received_date: int | None = None
    metadata: dict = field(default_factory=dict)


@dataclass
class DeviceMeasurement(DeviceEvent):
    event_type: DeviceEventType = DeviceEventType.Measurement
    name: str = ""
    value: float = 0.0


@dataclass
class DeviceLocation(DeviceEvent):
    event_type: DeviceEventType = DeviceEventType.Location
    latitude: float = 0.0
    longitude: float = 0.0
    elevation: float | None = None


@dataclass
class DeviceAlert(DeviceEvent):
    event_type: DeviceEventType = DeviceEventType.Alert
    source: AlertSource = AlertSource.Device
    level: AlertLevel = AlertLevel.Info
    type: str = ""
    message: str = ""


@dataclass
class DeviceCommandInvocation(DeviceEvent):
    event_type: DeviceEventType = DeviceEventType.CommandInvocation
    initiator: CommandInitiator = CommandInitiator.REST
    initiator_id: str | None = None
    target: CommandTarget = CommandTarget.Assignment
    target_id: str | None = None
    device_command_id: str | None = None
    command_token: str | None = None
    parameter_values: dict = field(default_factory=dict)


@dataclass
class DeviceCommandResponse(DeviceEvent):
    event_type: DeviceEventType = DeviceEventType.CommandResponse
    originating_event_id: str | None = None
    response_event_id: str | None = None
    response: str | None = None


@dataclass
class DeviceStateChange(DeviceEvent):
    event_type: DeviceEventType = DeviceEventType.StateChange
    attribute: str = ""
    type: str = ""
    previous_state: str | None = None
    new_state: str | None = None


EVENT_CLASSES = {
    DeviceEventType.Measurement: DeviceMeasurement, DeviceEventType.Location: DeviceLocation,
    DeviceEventType.Alert: DeviceAlert, DeviceEventType.CommandInvocation: DeviceCommandInvocation,
    DeviceEventType.CommandResponse: DeviceCommandResponse, DeviceEventType.StateChange: DeviceStateChange,
}


def event_from_dict(d: dict) -> DeviceEvent:
    et = DeviceEventType(d.get("eventType", "Measurement"))
    return EVENT_CLASSES[et].from_dict(d)


@dataclass
class DeviceEventBatch(Model):
    """Batch of event create requests for one device (reference DeviceEventBatch)."""
    device_token: str = ""
    measurements: list[dict] = field(default_factory=list)
    locations: list[dict] = field(default_factory=list)
    alerts: list[dict] = field(default_factory=list)


@dataclass
class DeviceEventContext(Model):
    """Context attached to enriched events (reference IDeviceEventContext)."""
    device_id: str | None = None
    device_token: str | None = None
    device_type_id: str | None = None
    device_type_token: str | None = None
    parent_device_id: str | None = None
    device_status: str | None = None
    device_metadata: dict = field(default_factory=dict)
    assignment_status: str | None = None
    assignment_metadata: dict = field(default_factory=dict)


# ============================================================================ batch / schedule
class BatchOperationStatus(str, enum.Enum):
    Unprocessed = "Unprocessed"
    Initializing = "Initializing"
    InitializedSuccessfully = "InitializedSuccessfully"
    InitializedWithErrors = "InitializedWithErrors"
    Processing = "Processing"
    FinishedSuccessfully = "FinishedSuccessfully"
    FinishedWithErrors = "FinishedWithErrors"


class ElementProcessingStatus(str, enum.Enum):
    Unprocessed = "Unprocessed"
    Processing = "Processing"
    Failed = "Failed"
    Succeeded = "Succeeded"


@dataclass
class BatchOperation(PersistentEntity):
    operation_type: str = "InvokeCommand"
    parameters: dict = field(default_factory=dict)
    processing_status: BatchOperationStatus = BatchOperationStatus.Unprocessed
    processing_started_date: int | None = None
    processing_ended_date: int | None = None


@dataclass
class BatchElement(Model):
    id: str = field(default_factory=new_id)
    batch_operation_id: str | None = None
    device_id: str | None = None
    processing_status: ElementProcessingStatus = ElementProcessingStatus.Unprocessed
    processed_date: int | None = None
    metadata: dict = field(default_factory=dict)


class TriggerType(str, enum.Enum):
    SimpleTrigger = "SimpleTrigger"
    CronTrigger = "CronTrigger"


class ScheduledJobType(str, enum.Enum):
    CommandInvocation = "CommandInvocation"
    BatchCommandInvocation = "BatchCommandInvocation"


class ScheduledJobState(str, enum.Enum):
    Unsubmitted = "Unsubmitted"
    Active = "Active"
    Complete = "Complete"


@dataclass
class Schedule(PersistentEntity):
    name: str = ""
    trigger_type: TriggerType = TriggerType.SimpleTrigger
    trigger_configuration: dict = field(default_factory=dict)
    start_date: int | None = None
    end_date: int | None = None


@dataclass
class ScheduledJob(PersistentEntity):
    schedule_id: str | None = None
    job_type: ScheduledJobType = ScheduledJobType.CommandInvocation
    job_configuration: dict = field(default_factory=dict)
    job_state: ScheduledJobState = ScheduledJobState.Unsubmitted


# ============================================================================ users / tenants
class AccountStatus(str, enum.Enum):
    Active = "Active"
    Expired = "Expired"
    Locked = "Locked"


@dataclass
class GrantedAuthority(Model):
    authority: str = ""
    description: str = ""
    parent: str | None = None
    group: bool = False


@dataclass
class User(PersistentEntity):
    username: str = ""
    hashed_password: str = ""
    first_name: str = ""
    last_name: str = ""
    email: str | None = None
    last_login: int | None = None
    status: AccountStatus = AccountStatus.Active
    authorities: list[str] = field(default_factory=list)

    def public_dict(self):
        d = self.to_dict()
        d.pop("hashedPassword", None)
        return d


@dataclass
class Tenant(BrandedEntity):
    name: str = ""
    authentication_token: str = ""
    authorized_user_ids: list[str] = field(default_factory=list)
    configuration_template_id: str = "default"
    dataset_template_id: str = "empty"


# ============================================================================ misc
@dataclass
class ScriptMetadata(Model):
    id: str = ""
    name: str = ""
    description: str = ""
    interpreter_type: str = "python"
    active_version: str | None = None
    versions: list[dict] = field(default_factory=list)


@dataclass
class Label(Model):
    content_type: str = "image/png"
    content: bytes = b""

    def to_dict(self):
        import base64
        return {"contentType": self.content_type, "content": base64.b64encode(self.content).decode()}


def stamp_created(e: PersistentEntity, user: str | None = None):
    e.created_date = e.created_date or now_ms()
    e.created_by = e.created_by or user
    return e


def stamp_updated(e: PersistentEntity, user: str | None = None):
    e.updated_date = now_ms()
    e.updated_by = user
    return e
