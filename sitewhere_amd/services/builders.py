"""Builder API for dataset initializer scripts.

Reference: the ``deviceBuilder`` / ``eventBuilder`` / ``assetBuilder`` / ``scheduleBuilder`` objects
bound into the Groovy initializers of a dataset template
(``service-tenant-management/dockerimage/datasets/*/scripts/*/content/initializer/*.groovy``, e.g.
``construction/.../deviceModel.groovy:29-342``): fluent request builders (``newDeviceType(...)
.withDescription(...).metadata(...)``) persisted through the management APIs, composite device
element schemas, device groups, and historical measurements / alerts / locations per assignment.

Here the builders are plain Python objects with snake_case fluent methods, bound into initializer
scripts as ``device_builder``, ``event_builder``, ``asset_builder`` and ``schedule_builder``
(``services/dataset_runner.py``).  Every ``persist`` goes through the tenant's management API, so
an initializer exercises the same validation and change feed as any client."""
from __future__ import annotations

import time


class _Req:
    """A request under construction: fluent setters collect camelCase request keys."""

    kind = ""

    def __init__(self, **fields):
        self.req = {k: v for k, v in fields.items() if v is not None}

    def _set(self, key, value):
        self.req[key] = value
        return self

    def with_description(self, d: str):
        return self._set("description", d)

    def with_image_url(self, u: str):
        return self._set("imageUrl", u)

    def with_icon(self, i: str):
        return self._set("icon", i)

    def with_background_color(self, c: str):
        return self._set("backgroundColor", c)

    def with_foreground_color(self, c: str):
        return self._set("foregroundColor", c)

    def with_border_color(self, c: str):
        return self._set("borderColor", c)

    def metadata(self, key: str, value: str):
        self.req.setdefault("metadata", {})[key] = str(value)
        return self

    @property
    def token(self):
        return self.req.get("token")


class _Bounded(_Req):
    def coord(self, latitude: float, longitude: float):
        self.req.setdefault("bounds", []).append({"latitude": float(latitude), "longitude": float(longitude)})
        return self


class _Slotted:
    def __init__(self, name: str, path: str):
        self.name, self.path = name, path
        self.slots: list[dict] = []
        self.units: list["_Unit"] = []

    def add_slot(self, name: str, path: str):
        self.slots.append({"name": name, "path": path})
        return self

    def add_unit(self, name: str, path: str) -> "_Unit":
        u = _Unit(name, path)
        self.units.append(u)
        return u

    def to_dict(self) -> dict:
        return {"deviceSlots": list(self.slots), "deviceUnits": [u.to_dict() for u in self.units]}


class _Unit(_Slotted):
    def to_dict(self) -> dict:
        return dict(super().to_dict(), name=self.name, path=self.path)


class _DeviceType(_Req):
    kind = "deviceType"

    def make_composite(self):
        self.req["containerPolicy"] = "Composite"
        return self

    def new_schema(self) -> _Slotted:
        self._schema = _Slotted("", "")
        return self._schema

    def request(self) -> dict:
        r = dict(self.req)
        if getattr(self, "_schema", None) is not None:
            r["deviceElementSchema"] = self._schema.to_dict()
        return r


class _Command(_Req):
    kind = "command"

    def _param(self, name, ptype, required):
        self.req.setdefault("parameters", []).append({"name": name, "type": ptype, "required": bool(required)})
        return self

    def with_string_parameter(self, name: str, required: bool = False):
        return self._param(name, "String", required)

    def with_boolean_parameter(self, name: str, required: bool = False):
        return self._param(name, "Bool", required)

    def with_double_parameter(self, name: str, required: bool = False):
        return self._param(name, "Double", required)

    def with_int32_parameter(self, name: str, required: bool = False):
        return self._param(name, "Int32", required)


class _AreaType(_Req):
    kind = "areaType"

    def with_contained_area_type(self, token: str):
        self.req.setdefault("containedAreaTypeTokens", []).append(token)
        return self


class _Zone(_Bounded):
    kind = "zone"

    def with_fill_color(self, c: str):
        return self._set("fillColor", c)

    def with_opacity(self, o: float):
        return self._set("opacity", float(o))


class _Group(_Req):
    kind = "group"

    def with_role(self, role: str):
        self.req.setdefault("roles", []).append(role)
        return self


class _Device(_Req):
    kind = "device"

    def with_comment(self, c: str):
        return self._set("comments", c)


class _Alarm(_Req):
    kind = "alarm"

    def with_triggering_event_id(self, eid: str):
        return self._set("triggeringEventId", eid)


class _Simple(_Req):
    def __init__(self, kind, **fields):
        super().__init__(**fields)
        self.kind = kind


class DeviceBuilder:
    """``deviceBuilder`` of the reference initializers, over a DeviceManagement API."""

    def __init__(self, dm, logger=None):
        self.dm = dm
        self.log = logger

    def new_customer_type(self, token, name):
        return _Simple("customerType", token=token, name=name)

    def new_customer(self, type_token, parent_token, token, name):
        return _Simple("customer", token=token, name=name, customerTypeToken=type_token,
                       parentCustomerToken=parent_token)

    def new_area_type(self, token, name):
        return _AreaType(token=token, name=name)

    def new_area(self, type_token, parent_token, token, name):
        a = _Bounded(token=token, name=name, areaTypeToken=type_token, parentAreaToken=parent_token)
        a.kind = "area"
        return a

    def new_zone(self, token, name, area):
        return _Zone(token=token, name=name, areaToken=area if isinstance(area, str) else area.token)

    def new_device_type(self, token, name):
        return _DeviceType(token=token, name=name)

    def new_command(self, type_token, token, namespace, name):
        return _Command(token=token, deviceTypeToken=type_token, namespace=namespace, name=name)

    def new_device_status(self, type_token, code, name):
        return _Simple("status", token=f"{type_token}-{code}", deviceTypeToken=type_token, code=code, name=name)

    def new_group(self, token, name):
        return _Group(token=token, name=name)

    def new_group_element(self, device_token, roles=()):
        return {"deviceToken": device_token, "roles": list(roles)}

    def new_device(self, type_token, token):
        return _Device(token=token, deviceTypeToken=type_token)

    def new_assignment(self, device_token, customer_token=None, area_token=None, asset_token=None):
        return _Simple("assignment", deviceToken=device_token, customerToken=customer_token, areaToken=area_token,
                       assetToken=asset_token)

    def new_device_alarm(self, assignment, message):
        a = assignment if isinstance(assignment, str) else assignment.id
        return _Alarm(deviceAssignmentId=a, alarmMessage=message)

    def persist(self, item, elements=None):
        """Create the entity (``elements``: a group's members, added after the group)."""
        dm = self.dm
        k = item.kind
        r = item.request() if hasattr(item, "request") else item.req
        if k == "group" and elements is not None:
            g = dm.get_device_group_by_token(r["token"]) if r.get("token") else None
            g = g or dm.create_device_group(r)
            if elements:
                dm.add_device_group_elements(g.id, list(elements))
            return g
        fn = {"customerType": dm.create_customer_type, "customer": dm.create_customer,
              "areaType": dm.create_area_type, "area": dm.create_area, "zone": dm.create_zone,
              "deviceType": dm.create_device_type, "command": dm.create_device_command,
              "status": dm.create_device_status, "group": dm.create_device_group, "device": dm.create_device,
              "assignment": dm.create_device_assignment, "alarm": dm.create_device_alarm}[k]
        return fn(r)


class _Event(_Req):
    def on(self, date_ms):
        return self._set("eventDate", int(date_ms))

    def track_state(self, on: bool = True):
        return self._set("updateState", bool(on))

    def with_alternate_id(self, alt: str):
        return self._set("alternateId", alt)


class _Measurements(_Event):
    kind = "measurements"

    def measurement(self, name, value):
        self.req.setdefault("_mx", []).append((name, float(value)))
        return self


class _Alert(_Event):
    kind = "alert"

    def _level(self, lv):
        return self._set("level", lv)

    def info(self):
        return self._level("Info")

    def warning(self):
        return self._level("Warning")

    def error(self):
        return self._level("Error")

    def critical(self):
        return self._level("Critical")


class _AssignmentEvents:
    def __init__(self, eb: "EventBuilder", assignment):
        self.eb, self.assignment = eb, assignment

    def _aid(self):
        a = self.assignment
        if not isinstance(a, str):
            return a.id
        found = self.eb.dm.get_device_assignment_by_token(a)
        return found.id if found is not None else a

    def persist_measurements(self, requests):
        reqs = []
        for r in requests:
            base = {k: v for k, v in r.req.items() if k != "_mx"}
            reqs += [dict(base, name=n, value=v) for n, v in r.req.get("_mx", [])]
        return self.eb.call("add_measurements", self._aid(), reqs) if reqs else []

    def persist_alerts(self, requests):
        return self.eb.call("add_alerts", self._aid(), [r.req for r in requests]) if requests else []

    def persist_locations(self, requests):
        return self.eb.call("add_locations", self._aid(), [r.req for r in requests]) if requests else []


class EventBuilder:
    """``eventBuilder`` of the reference initializers, over the tenant's DeviceEventManagement API
    (reached lazily: event management may start after device management bootstraps)."""

    def __init__(self, em_factory, dm, wait_s: float = 60.0, logger=None):
        self._em_factory, self.dm, self.wait_s = em_factory, dm, wait_s
        self.log = logger
        self.disabled = False

    def call(self, method, *args):
        """Call event management; if it never becomes reachable (a deployment without it) the
        history is skipped with a warning rather than failing the tenant's bootstrap."""
        if self.disabled:
            return []
        deadline = time.time() + self.wait_s
        while True:
            try:
                return getattr(self._em_factory(), method)(*args)
            except Exception as e:  # noqa: BLE001 -- the tenant's event management engine is still starting
                if time.time() > deadline:
                    self.disabled = True
                    if self.log is not None:
                        self.log.warning("event management unreachable, skipping dataset events: %s", e)
                    return []
                time.sleep(0.1)

    def new_measurements(self):
        return _Measurements()

    def new_alert(self, alert_type, message):
        return _Alert(type=alert_type, message=message, source="Device", level="Info")

    def new_location(self, latitude, longitude, elevation=None):
        r = _Event(latitude=float(latitude), longitude=float(longitude), elevation=elevation)
        r.kind = "location"
        return r

    def for_assignment(self, assignment):
        return _AssignmentEvents(self, assignment)


class AssetBuilder:
    def __init__(self, am):
        self.am = am

    def new_asset_type(self, token, name, category="Device"):
        return _Simple("assetType", token=token, name=name, assetCategory=category)

    def new_asset(self, type_token, token, name):
        return _Simple("asset", token=token, name=name, assetTypeToken=type_token)

    def persist(self, item):
        fn = {"assetType": self.am.create_asset_type, "asset": self.am.create_asset}[item.kind]
        return fn(item.req)


class ScheduleBuilder:
    def __init__(self, sm):
        self.sm = sm

    def new_cron_schedule(self, token, name, expression):
        return _Simple("schedule", token=token, name=name, triggerType="CronTrigger",
                       triggerConfiguration={"cronExpression": expression})

    def new_simple_schedule(self, token, name, interval_ms, repeat_count=-1):
        return _Simple("schedule", token=token, name=name, triggerType="SimpleTrigger",
                       triggerConfiguration={"repeatInterval": int(interval_ms), "repeatCount": int(repeat_count)})

    def persist(self, item):
        return self.sm.create_schedule(item.req)
