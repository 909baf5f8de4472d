"""service-web-rest: the REST API (25 controllers), JWT issue, tenant headers, WebSocket topology feed.

Reference: ``service-web-rest/.../web/rest/controllers/*.java`` (193 endpoint methods under
``/sitewhere/api``), ``LimitedBasicAuthFilter.java:36`` (``GET /sitewhere/authapi/jwt`` with HTTP
basic credentials -> ``X-Sitewhere-JWT`` header), ``TokenAuthenticationFilter.java:74-117``
(``Authorization: Bearer`` + ``X-SiteWhere-Tenant-Id`` / ``X-SiteWhere-Tenant-Auth``),
``ISiteWhereWebConstants.java:18-30`` (header names), ``TopologyBroadcaster`` (WebSocket feed).

Every controller call goes through the same RPC dispatch (auth, tenant resolution, tracing span,
codec) as service-to-service calls -- the in-process channel when co-located, gRPC otherwise.
REST event writes call event management directly (``Assignments.java:360-369``).
"""
from __future__ import annotations

import asyncio
import base64
import datetime as _dt
import json
import threading

from fastapi import APIRouter, Body, Depends, FastAPI, Header, Request, WebSocket, WebSocketDisconnect
from fastapi.responses import JSONResponse, Response

from ..core.errors import (ErrorCode, NotFoundException, SiteWhereException, SiteWhereSystemException,
                           UnauthorizedException)
from ..core.security import Authentication, SiteWhereAuthority, security_context
from ..models.domain import Model, SearchResults
from ..runtime.microservice import GlobalMicroservice

API = "/sitewhere/api"
HEADER_JWT = "X-Sitewhere-JWT"
HEADER_TENANT_ID = "X-SiteWhere-Tenant-Id"
HEADER_TENANT_AUTH = "X-SiteWhere-Tenant-Auth"
HEADER_ERROR = "X-SiteWhere-Error"
HEADER_ERROR_CODE = "X-SiteWhere-Error-Code"
VERSION = {"edition": "MI355X", "editionIdentifier": "MI355X", "versionIdentifier": "3.0.0-mi355x",
           "buildTimestamp": "2026-10-15"}


# ------------------------------------------------------------------------------ serialization
def out(v):
    if isinstance(v, SearchResults):
        return {"numResults": v.num_results, "results": [out(r) for r in v.results]}
    if isinstance(v, Model):
        d = v.public_dict() if hasattr(v, "public_dict") else v.to_dict()
        return d
    if isinstance(v, (list, tuple)):
        return [out(x) for x in v]
    if isinstance(v, dict):
        return {k: out(x) for k, x in v.items()}
    if isinstance(v, bytes):
        return base64.b64encode(v).decode()
    if hasattr(v, "value") and hasattr(v, "name") and isinstance(getattr(v, "value"), str):
        return v.value
    return v


def _date(s):
    if s is None or s == "":
        return None
    try:
        return int(s)
    except (TypeError, ValueError):
        return int(_dt.datetime.fromisoformat(str(s).replace("Z", "+00:00")).timestamp() * 1000)


_QUERY_ALIASES = {"deviceType": "deviceTypeToken", "customer": "customerToken", "area": "areaToken",
                  "asset": "assetToken", "areaType": "areaTypeToken", "customerType": "customerTypeToken",
                  "assetType": "assetTypeToken"}


def query_criteria(request: Request, page: int, pageSize: int) -> dict:
    """Query string -> search criteria: the reference's parameter names (``deviceType``, ...) map
    to token criteria, ``true``/``false`` become booleans and epoch / ISO-8601 dates integers
    (query values are strings: ``excludeAssigned=false`` must not read as true)."""
    crit: dict = {}
    for k, v in request.query_params.items():
        k = _QUERY_ALIASES.get(k, k)
        if isinstance(v, str) and v.lower() in ("true", "false"):
            v = v.lower() == "true"
        elif k.endswith(("Date", "After", "Before")) and v:
            v = _date(v)
        crit[k] = v
    crit.update(paging(page, pageSize))
    return crit


def paging(page: int = 1, pageSize: int = 100) -> dict:
    return {"pageNumber": page, "pageSize": pageSize}


def date_paging(page: int = 1, pageSize: int = 100, startDate: str | None = None, endDate: str | None = None) -> dict:
    return {"pageNumber": page, "pageSize": pageSize, "startDate": _date(startDate), "endDate": _date(endDate)}


# ------------------------------------------------------------------------------ request context
class _Bound:
    """Service proxy that runs every call inside the caller's security context."""

    def __init__(self, proxy, auth):
        self._p, self._a = proxy, auth

    def __getattr__(self, name):
        fn = getattr(self._p, name)

        def call(*a, **k):
            with security_context(self._a):
                return fn(*a, **k)
        return call


class Ctx:
    def __init__(self, web: "WebRest", auth: Authentication):
        self.web, self.auth = web, auth

    def svc(self, name: str) -> _Bound:
        return _Bound(self.web.channel.proxy(name, self.auth.tenant), self.auth)

    def require(self, authority: str):
        if not self.auth.has(authority):
            raise SiteWhereSystemException(ErrorCode.NotAuthorized, detail=f"missing authority {authority}",
                                           http_status=403)

    @property
    def dm(self):
        return self.svc("DeviceManagement")

    @property
    def em(self):
        return self.svc("DeviceEventManagement")

    @property
    def am(self):
        return self.svc("AssetManagement")


class WebRest:
    def __init__(self, instance, topology=None):
        self.instance = instance
        self.channel = instance.router
        self.tokens = instance.tokens
        self.topology = topology

    def system(self, tenant=None) -> Authentication:
        return self.instance.system_user.authentication(tenant)

    def authenticate_jwt(self, authorization: str | None, tenant_id: str | None, tenant_auth: str | None,
                         tenant_required: bool) -> Ctx:
        if not authorization or not authorization.lower().startswith("bearer "):
            raise UnauthorizedException("missing bearer token")
        jwt = authorization[7:].strip()
        claims = self.tokens.get_claims(jwt)
        auth = Authentication(claims["sub"], list(claims.get("auth", [])), jwt, None)
        if tenant_required:
            if not tenant_id:
                raise SiteWhereSystemException(ErrorCode.InvalidTenantToken, detail="tenant id header required",
                                               http_status=401)
            sysctx = self.system()
            with security_context(sysctx):
                t = self.channel.proxy("TenantManagement").get_tenant_by_token(tenant_id)
            if t is None:
                raise SiteWhereSystemException(ErrorCode.InvalidTenantToken, detail=tenant_id, http_status=401)
            if tenant_auth != t.authentication_token:
                raise SiteWhereSystemException(ErrorCode.InvalidTenantAuthToken if hasattr(ErrorCode, "InvalidTenantAuthToken")
                                               else ErrorCode.NotAuthorized, detail="invalid tenant authentication token",
                                               http_status=401)
            if auth.username not in t.authorized_user_ids and not auth.has(SiteWhereAuthority.AdminTenants):
                raise SiteWhereSystemException(ErrorCode.NotAuthorized, detail="user not authorized for tenant",
                                               http_status=403)
            auth.tenant = tenant_id
        return Ctx(self, auth)


def _dep(tenant_required: bool):
    def dep(request: Request, authorization: str | None = Header(None),
            x_sitewhere_tenant_id: str | None = Header(None), x_sitewhere_tenant_auth: str | None = Header(None)) -> Ctx:
        return request.app.state.web.authenticate_jwt(authorization, x_sitewhere_tenant_id, x_sitewhere_tenant_auth,
                                                      tenant_required)
    return dep


TENANT = Depends(_dep(True))
GLOBAL = Depends(_dep(False))


def _nf(v, what: str):
    if v is None:
        raise NotFoundException(ErrorCode.Error, f"{what} not found")
    return v


def png(label) -> Response:
    return Response(content=label.content, media_type=label.content_type or "image/png")


# ------------------------------------------------------------------------------ generic CRUD routers
FAMILIES = [
    # path, service, noun, plural, label kind, update/delete keyed by token
    ("areatypes", "DeviceManagement", "area_type", "area_types", "area_type", False),
    ("areas", "DeviceManagement", "area", "areas", "area", False),
    ("assettypes", "AssetManagement", "asset_type", "asset_types", "asset_type", False),
    ("assets", "AssetManagement", "asset", "assets", "asset", False),
    ("customertypes", "DeviceManagement", "customer_type", "customer_types", "customer_type", False),
    ("customers", "DeviceManagement", "customer", "customers", "customer", False),
    ("commands", "DeviceManagement", "device_command", "device_commands", None, False),
    ("statuses", "DeviceManagement", "device_status", "device_statuses", None, False),
    ("devicetypes", "DeviceManagement", "device_type", "device_types", "device_type", False),
    ("devicegroups", "DeviceManagement", "device_group", "device_groups", "device_group", False),
    ("zones", "DeviceManagement", "zone", "zones", None, False),
    ("schedules", "ScheduleManagement", "schedule", "schedules", None, True),
    ("jobs", "ScheduleManagement", "scheduled_job", "scheduled_jobs", None, True),
]


def _one(field, getter, service="DeviceManagement"):
    def resolve(c, e):
        v = getattr(e, field, None)
        return getattr(c.svc(service), getter)(v) if v else None
    return resolve


def _many(field, getter, service="DeviceManagement"):
    def resolve(c, e):
        fn = getattr(c.svc(service), getter)
        return [x for x in (fn(i) for i in (getattr(e, field, None) or [])) if x is not None]
    return resolve


def _asset(c, e):
    if not getattr(e, "asset_id", None):
        return None
    am = c.svc("AssetManagement")
    return am.get_asset(e.asset_id) or am.get_asset_by_token(e.asset_id)


def _state_events(c, s):
    """DeviceStateMarshalHelper includeEventDetails: the events behind the state's last-event ids."""
    get = c.em.get_device_event_by_id
    loc = get(s.last_location_event_id) if s.last_location_event_id else None
    return {"lastLocationEvent": out(loc) if loc else None,
            "lastMeasurementEvents": {k: out(get(v)) for k, v in (s.last_measurement_event_ids or {}).items()},
            "lastAlertEvents": {k: out(get(v)) for k, v in (s.last_alert_event_ids or {}).items()}}


# the reference's marshal helpers: query flag -> (JSON key, resolver) per resource
INCLUDES = {
    "areas": {"includeAreaType": ("areaType", _one("area_type_id", "get_area_type")),
              "includeParentArea": ("parentArea", _one("parent_area_id", "get_area")),
              "includeZones": ("zones", lambda c, e: c.dm.list_zones({"areaId": e.id, "pageSize": 0}).results)},
    "customers": {"includeCustomerType": ("customerType", _one("customer_type_id", "get_customer_type")),
                  "includeParentCustomer": ("parentCustomer", _one("parent_customer_id", "get_customer"))},
    "assets": {"includeAssetType": ("assetType", _one("asset_type_id", "get_asset_type", "AssetManagement"))},
    "areatypes": {"includeContainedAreaTypes": ("containedAreaTypes", _many("contained_area_type_ids",
                                                                             "get_area_type"))},
    "customertypes": {"includeContainedCustomerTypes": ("containedCustomerTypes",
                                                        _many("contained_customer_type_ids", "get_customer_type"))},
    "devicestates": {"includeDevice": ("device", _one("device_id", "get_device")),
                     "includeDeviceType": ("deviceType", _one("device_type_id", "get_device_type")),
                     "includeDeviceAssignment": ("deviceAssignment", _one("device_assignment_id", "get_device_assignment")),
                     "includeCustomer": ("customer", _one("customer_id", "get_customer")),
                     "includeArea": ("area", _one("area_id", "get_area")),
                     "includeAsset": ("asset", _asset),
                     "includeEventDetails": (None, _state_events)},
    "batchelements": {"includeDevice": ("device", _one("device_id", "get_device"))},
    "invocations": {"includeCommand": ("command", _one("device_command_id", "get_device_command"))},
}


def nested(c, kind: str, entity, flags) -> dict:
    """``out(entity)`` plus the related objects the truthy ``include*`` flags ask for."""
    doc = out(entity)
    for flag, (key, resolve) in INCLUDES.get(kind, {}).items():
        v = flags.get(flag)
        if v is True or (isinstance(v, str) and v.lower() == "true"):
            r = resolve(c, entity)
            if key is None:
                doc.update(r)
            else:
                doc[key] = out(r) if r is not None else None
    return doc


def nested_results(c, kind: str, res, flags) -> dict:
    return {"numResults": res.num_results, "results": [nested(c, kind, e, flags) for e in res.results]}


def crud_router(path, service, noun, plural, label, by_token, before=None) -> APIRouter:
    r = APIRouter(prefix=f"{API}/{path}", tags=[path])

    def get(c: Ctx, token: str):
        return _nf(getattr(c.svc(service), f"get_{noun}_by_token")(token), f"{noun} {token}")

    if before:
        before(r)

    @r.post("")
    def create(body: dict = Body(...), c: Ctx = TENANT):
        return out(getattr(c.svc(service), f"create_{noun}")(body))

    @r.get("")
    def list_(request: Request, page: int = 1, pageSize: int = 100, c: Ctx = TENANT):
        crit = query_criteria(request, page, pageSize)
        return nested_results(c, path, getattr(c.svc(service), f"list_{plural}")(crit), crit)

    @r.get("/{token}")
    def read(token: str, request: Request, c: Ctx = TENANT):
        return nested(c, path, get(c, token), request.query_params)

    @r.put("/{token}")
    def update(token: str, body: dict = Body(...), c: Ctx = TENANT):
        key = token if by_token else get(c, token).id
        return out(getattr(c.svc(service), f"update_{noun}")(key, body))

    @r.delete("/{token}")
    def delete(token: str, c: Ctx = TENANT):
        key = token if by_token else get(c, token).id
        return out(getattr(c.svc(service), f"delete_{noun}")(key))

    if label:
        @r.get("/{token}/label/{generatorId}")
        def label_(token: str, generatorId: str, c: Ctx = TENANT):
            return png(getattr(c.svc("LabelGeneration"), f"get_{label}_label")(generatorId, get(c, token).id))

    r.entity_getter = get  # type: ignore[attr-defined]
    return r


EVENT_KINDS = {"measurements": "list_measurements_for_index", "locations": "list_locations_for_index",
               "alerts": "list_alerts_for_index", "invocations": "list_command_invocations_for_index",
               "responses": "list_command_responses_for_index", "statechanges": "list_state_changes_for_index"}


def add_index_event_routes(r: APIRouter, index: str, getter):
    for kind, fn in EVENT_KINDS.items():
        def make(fn=fn):
            def handler(token: str, page: int = 1, pageSize: int = 100, startDate: str | None = None,
                        endDate: str | None = None, c: Ctx = TENANT):
                ent = getter(c, token)
                return out(getattr(c.em, fn)(index, [ent.id], date_paging(page, pageSize, startDate, endDate)))
            return handler
        r.add_api_route(f"/{{token}}/{kind}", make(), methods=["GET"])

    def assignments(token: str, page: int = 1, pageSize: int = 100, status: str | None = None,
                    includeDevice: bool = False, includeCustomer: bool = False, includeArea: bool = False,
                    includeAsset: bool = False, c: Ctx = TENANT):
        ent = getter(c, token)
        crit = {f"{index.lower()}Id": ent.id, **paging(page, pageSize)}
        if status:
            crit["status"] = status
        res = c.dm.list_device_assignments(crit)
        return {"numResults": res.num_results, "results": [
            marshal_assignment(c, a, includeDevice, includeCustomer, includeArea, includeAsset) for a in res.results]}
    r.add_api_route("/{token}/assignments", assignments, methods=["GET"])


# ------------------------------------------------------------------------------ app
ADMIN_UI_BUILTIN = __import__("pathlib").Path(__file__).resolve().parent / "admin"


def mount_admin_ui(app: FastAPI, directory: str | None = None):
    """Serve an admin UI build at ``/admin/`` (``directory``, else ``SITEWHERE_ADMIN_UI_DIR``, else the
    built-in console in ``web/admin``); ``/`` and ``/admin`` redirect to it, as the reference's
    web-rest does for its Vue app (``VueConfiguration``, ``RedirectServlet``)."""
    import os

    from fastapi.responses import RedirectResponse
    from fastapi.staticfiles import StaticFiles
    d = directory or os.environ.get("SITEWHERE_ADMIN_UI_DIR") or str(ADMIN_UI_BUILTIN)
    if not os.path.isdir(d):
        raise SiteWhereException(f"admin UI directory {d!r} does not exist")

    @app.get("/", include_in_schema=False)
    def root():
        return RedirectResponse("/admin/")

    @app.get("/admin", include_in_schema=False)
    def admin():
        return RedirectResponse("/admin/")
    app.mount("/admin", StaticFiles(directory=d, html=True), name="admin")


def create_app(instance, topology=None, cors: bool = True, admin_ui_dir: str | None = None) -> FastAPI:
    app = FastAPI(title="SiteWhere (MI355X) REST API", version=VERSION["versionIdentifier"],
                  docs_url=f"{API}/docs", openapi_url=f"{API}/openapi.json")
    if cors:   # reference RestSecurity/CORS filter: the admin UI is served from another origin
        from fastapi.middleware.cors import CORSMiddleware
        app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_methods=["*"], allow_headers=["*"],
                           expose_headers=[HEADER_JWT, HEADER_ERROR, HEADER_ERROR_CODE])
    web = WebRest(instance, topology)
    app.state.web = web

    @app.exception_handler(SiteWhereSystemException)
    def sw_error(request, e: SiteWhereSystemException):
        return JSONResponse({"error": str(e), "code": e.code.name}, status_code=e.http_status,
                            headers={HEADER_ERROR: str(e)[:200], HEADER_ERROR_CODE: str(e.code.value[0])})

    @app.exception_handler(SiteWhereException)
    def sw_error2(request, e: SiteWhereException):
        return JSONResponse({"error": str(e)}, status_code=500, headers={HEADER_ERROR: str(e)[:200]})

    # ---- auth ------------------------------------------------------------------------
    @app.get("/sitewhere/authapi/jwt")
    def jwt(authorization: str | None = Header(None)):
        if not authorization or not authorization.lower().startswith("basic "):
            raise UnauthorizedException("basic credentials required")
        user, _, pw = base64.b64decode(authorization[6:]).decode().partition(":")
        with security_context(web.system()):
            u = web.channel.proxy("UserManagement").authenticate(user, pw, True)
        token = web.tokens.generate_token(u.username, list(u.authorities))
        return JSONResponse({"username": u.username, "authorities": u.authorities, "token": token},
                            headers={HEADER_JWT: token})

    # ---- token-keyed entity families -------------------------------------------------------
    routers = {}
    for fam in FAMILIES:
        path = fam[0]
        before = None
        if path == "commands":
            def before(r):
                @r.get("/namespaces")
                def namespaces(deviceTypeToken: str | None = None, c: Ctx = TENANT):
                    crit = {"pageSize": 0}
                    if deviceTypeToken:
                        crit["deviceTypeToken"] = deviceTypeToken
                    cmds = c.dm.list_device_commands(crit).results
                    ns: dict = {}
                    for cmd in cmds:
                        ns.setdefault(cmd.namespace or "", []).append(out(cmd))
                    return [{"value": k, "commands": v} for k, v in sorted(ns.items())]
        elif path == "devicetypes":
            def before(r):
                @r.get("/{token}/proto")
                def proto(token: str, c: Ctx = TENANT):
                    return Response(device_type_proto(c, token), media_type="text/plain")

                @r.get("/{token}/spec.proto")
                def spec(token: str, c: Ctx = TENANT):
                    return Response(device_type_proto(c, token), media_type="application/octet-stream",
                                    headers={"Content-Disposition": f"attachment; filename={token}.proto"})
        elif path == "devicegroups":
            def before(r):
                def grp(c, token):
                    return _nf(c.dm.get_device_group_by_token(token), f"group {token}")

                @r.get("/{token}/elements")
                def elements(token: str, page: int = 1, pageSize: int = 100, c: Ctx = TENANT):
                    return out(c.dm.list_device_group_elements(grp(c, token).id, paging(page, pageSize)))

                @r.put("/{token}/elements")
                def add_elements(token: str, body: list = Body(...), c: Ctx = TENANT):
                    return out(c.dm.add_device_group_elements(grp(c, token).id, body))

                @r.delete("/{token}/elements/{elementId}")
                def del_element(token: str, elementId: str, c: Ctx = TENANT):
                    return out(c.dm.remove_device_group_elements([elementId]))

                @r.delete("/{token}/elements")
                def del_elements(token: str, body: list = Body(...), c: Ctx = TENANT):
                    return out(c.dm.remove_device_group_elements(body))
        routers[path] = crud_router(*fam, before=before)
    add_index_event_routes(routers["areas"], "Area", routers["areas"].entity_getter)
    add_index_event_routes(routers["customers"], "Customer", routers["customers"].entity_getter)
    for r in routers.values():
        app.include_router(r)

    app.include_router(devices_router())
    app.include_router(assignments_router())
    app.include_router(misc_router(web))
    app.include_router(admin_router(web))

    # ---- admin UI (reference VueConfiguration: static UI under /admin/, "/" forwards to it) --------
    mount_admin_ui(app, admin_ui_dir)

    @app.get("/metrics")
    def metrics():
        """Prometheus text exposition of every co-located microservice's registry (the reference only
        logs Dropwizard metrics every 20 s, ``Microservice.java:242-250``)."""
        text = []
        for ms in list(web.instance.microservices.values()):
            body = ms.metrics.prometheus(prefix=f"sitewhere_{ms.identifier.replace('-', '_')}_")
            if body:
                text.append(body)
        return Response("\n".join(text) + "\n", media_type="text/plain; version=0.0.4")

    @app.websocket("/sitewhere/ws/topology")
    async def topology_ws(ws: WebSocket):
        await ws.accept()
        last = None
        try:
            while True:
                snap = web.topology.snapshot.to_dict() if web.topology else {}
                if snap != last:
                    await ws.send_text(json.dumps({"type": "topology", "topology": snap}))
                    last = snap
                await asyncio.sleep(0.25)
        except (WebSocketDisconnect, RuntimeError):
            return

    return app


def device_type_proto(c: Ctx, token: str) -> str:
    """Protobuf spec for a device type's commands (reference DeviceTypeProtoBuilder)."""
    dt = _nf(c.dm.get_device_type_by_token(token), f"device type {token}")
    cmds = c.dm.list_device_commands({"deviceTypeToken": token, "pageSize": 0}).results
    types = {"String": "string", "Double": "double", "Float": "float", "Int32": "int32", "Int64": "int64",
             "UInt32": "uint32", "UInt64": "uint64", "SInt32": "sint32", "SInt64": "sint64", "Fixed32": "fixed32",
             "Fixed64": "fixed64", "SFixed32": "sfixed32", "SFixed64": "sfixed64", "Bool": "bool", "Bytes": "bytes"}
    name = "".join(p.title() for p in dt.token.replace("-", " ").replace(".", " ").split())
    lines = ['syntax = "proto3";', "", f"package {name.lower()};", "", f"message {name} {{", "",
             "  enum Command {"]
    lines += [f"    {cmd.name.upper()} = {i};" for i, cmd in enumerate(sorted(cmds, key=lambda x: x.name))]
    lines += ["  }", "", "  message _Header {", "    Command command = 1;", "    string originator = 2;",
              "    string nestedPath = 3;", "    string nestedSpec = 4;", "  }", ""]
    for cmd in sorted(cmds, key=lambda x: x.name):
        lines.append(f"  message {cmd.name} {{")
        for j, p in enumerate(cmd.parameters or [], 1):
            pname = p["name"] if isinstance(p, dict) else p.name
            ptype = p["type"] if isinstance(p, dict) else p.type
            lines.append(f"    {types.get(getattr(ptype, 'value', ptype), 'string')} {pname} = {j};")
        lines += ["  }", ""]
    lines.append("}")
    return "\n".join(lines) + "\n"


def marshal_device(c, d, include_type: bool = False, include_assignment: bool = False) -> dict:
    """Device JSON with the reference's optional nested objects (``DeviceMarshalHelper``:
    ``deviceType``, ``assignment`` -- the assignment with its customer / area / asset)."""
    doc = out(d)
    if include_type and d.device_type_id:
        t = c.dm.get_device_type(d.device_type_id)
        doc["deviceType"] = out(t) if t else None
    if include_assignment and d.device_assignment_id:
        a = c.dm.get_device_assignment(d.device_assignment_id)
        doc["assignment"] = marshal_assignment(c, a, False, True, True, True) if a else None
    return doc


def marshal_assignment(c, a, include_device=False, include_customer=False, include_area=False,
                       include_asset=False) -> dict:
    """Assignment JSON with optional ``device`` / ``customer`` / ``area`` / ``asset`` objects
    (``DeviceAssignmentMarshalHelper``); the asset is looked up by id or token."""
    doc = out(a)
    if include_device and a.device_id:
        d = c.dm.get_device(a.device_id)
        doc["device"] = out(d) if d else None
    if include_customer and a.customer_id:
        cu = c.dm.get_customer(a.customer_id)
        doc["customer"] = out(cu) if cu else None
    if include_area and a.area_id:
        ar = c.dm.get_area(a.area_id)
        doc["area"] = out(ar) if ar else None
    if include_asset and a.asset_id:
        am = c.svc("AssetManagement")
        asset = am.get_asset(a.asset_id) or am.get_asset_by_token(a.asset_id)
        if asset is not None:
            doc["asset"] = out(asset)
            doc["assetName"] = asset.name
            doc["assetImageUrl"] = getattr(asset, "image_url", None)
    return doc


def devices_router() -> APIRouter:
    r = APIRouter(prefix=f"{API}/devices", tags=["devices"])

    def dev(c, token):
        return _nf(c.dm.get_device_by_token(token), f"device {token}")

    @r.post("")
    def create(body: dict = Body(...), c: Ctx = TENANT):
        return out(c.dm.create_device(body))

    @r.get("")
    def list_(request: Request, page: int = 1, pageSize: int = 100, includeDeviceType: bool = False,
              includeAssignment: bool = False, c: Ctx = TENANT):
        crit = query_criteria(request, page, pageSize)
        res = c.dm.list_devices(crit)
        return {"numResults": res.num_results,
                "results": [marshal_device(c, d, includeDeviceType, includeAssignment) for d in res.results]}

    @r.get("/group/{groupToken}")
    def in_group(groupToken: str, role: str | None = None, c: Ctx = TENANT):
        g = _nf(c.dm.get_device_group_by_token(groupToken), f"group {groupToken}")
        ids = c.dm.expand_group_devices(g.id, [role] if role else None)
        devs = [c.dm.get_device(i) for i in ids]
        return out(SearchResults(len(devs), [d for d in devs if d]))

    @r.get("/grouprole/{role}")
    def in_role(role: str, c: Ctx = TENANT):
        ids: list = []
        for g in c.dm.list_device_groups_with_role(role).results:
            ids += [i for i in c.dm.expand_group_devices(g.id, None) if i not in ids]
        devs = [c.dm.get_device(i) for i in ids]
        return out(SearchResults(len(devs), [d for d in devs if d]))

    @r.get("/{token}")
    def read(token: str, includeDeviceType: bool = True, includeAssignment: bool = True, c: Ctx = TENANT):
        return marshal_device(c, dev(c, token), includeDeviceType, includeAssignment)

    @r.put("/{token}")
    def update(token: str, body: dict = Body(...), c: Ctx = TENANT):
        return out(c.dm.update_device(dev(c, token).id, body))

    @r.delete("/{token}")
    def delete(token: str, c: Ctx = TENANT):
        return out(c.dm.delete_device(dev(c, token).id))

    @r.get("/{token}/label/{generatorId}")
    def label(token: str, generatorId: str, c: Ctx = TENANT):
        return png(c.svc("LabelGeneration").get_device_label(generatorId, dev(c, token).id))

    @r.get("/{token}/symbol")
    def symbol(token: str, c: Ctx = TENANT):
        return png(c.svc("LabelGeneration").get_device_label("qrcode", dev(c, token).id))

    @r.get("/{token}/assignment")
    def current_assignment(token: str, c: Ctx = TENANT):
        return out(_nf(c.dm.get_current_assignment_for_device(dev(c, token).id), "active assignment"))

    @r.get("/{token}/assignments")
    def assignments(token: str, page: int = 1, pageSize: int = 100, c: Ctx = TENANT):
        return out(c.dm.list_device_assignments({"deviceId": dev(c, token).id, **paging(page, pageSize)}))

    @r.post("/{token}/mappings")
    def add_mapping(token: str, body: dict = Body(...), c: Ctx = TENANT):
        return out(c.dm.create_device_element_mapping(dev(c, token).id, body))

    @r.delete("/{token}/mappings")
    def del_mapping(token: str, path: str, c: Ctx = TENANT):
        return out(c.dm.delete_device_element_mapping(dev(c, token).id, path))

    @r.post("/{token}/batch")
    def batch(token: str, body: dict = Body(...), c: Ctx = TENANT):
        a = _nf(c.dm.get_current_assignment_for_device(dev(c, token).id), "active assignment")
        return out(c.em.add_device_event_batch(a.id, body))

    return r


def assignments_router() -> APIRouter:
    r = APIRouter(prefix=f"{API}/assignments", tags=["assignments"])

    def asg(c, token):
        return _nf(c.dm.get_device_assignment_by_token(token), f"assignment {token}")

    @r.post("")
    def create(body: dict = Body(...), c: Ctx = TENANT):
        return out(c.dm.create_device_assignment(body))

    @r.get("")
    def list_(request: Request, page: int = 1, pageSize: int = 100, c: Ctx = TENANT):
        crit = query_criteria(request, page, pageSize)
        for k, fn in (("deviceToken", c.dm.get_device_by_token), ("customerToken", c.dm.get_customer_by_token),
                      ("areaToken", c.dm.get_area_by_token)):
            if crit.get(k):
                crit[k.replace("Token", "Id")] = _nf(fn(crit.pop(k)), k).id
        if crit.get("assetToken"):      # assignments reference an asset by id or (cross-service) by token
            tok = crit.pop("assetToken")
            crit["assetIds"] = [_nf(c.svc("AssetManagement").get_asset_by_token(tok), "assetToken").id, tok]
        res = c.dm.list_device_assignments(crit)
        inc = [bool(crit.get(k)) for k in ("includeDevice", "includeCustomer", "includeArea", "includeAsset")]
        return {"numResults": res.num_results, "results": [marshal_assignment(c, a, *inc) for a in res.results]}

    @r.get("/{token}")
    def read(token: str, includeDevice: bool = False, includeCustomer: bool = False, includeArea: bool = False,
             includeAsset: bool = False, c: Ctx = TENANT):
        return marshal_assignment(c, asg(c, token), includeDevice, includeCustomer, includeArea, includeAsset)

    @r.put("/{token}")
    def update(token: str, body: dict = Body(...), c: Ctx = TENANT):
        return out(c.dm.update_device_assignment(asg(c, token).id, body))

    @r.delete("/{token}")
    def delete(token: str, c: Ctx = TENANT):
        return out(c.dm.delete_device_assignment(asg(c, token).id))

    @r.get("/{token}/label/{generatorId}")
    def label(token: str, generatorId: str, c: Ctx = TENANT):
        return png(c.svc("LabelGeneration").get_device_assignment_label(generatorId, asg(c, token).id))

    @r.get("/{token}/symbol")
    def symbol(token: str, c: Ctx = TENANT):
        return png(c.svc("LabelGeneration").get_device_assignment_label("qrcode", asg(c, token).id))

    @r.post("/{token}/end")
    def end(token: str, c: Ctx = TENANT):
        return out(c.dm.end_device_assignment(asg(c, token).id))

    @r.post("/{token}/missing")
    def missing(token: str, c: Ctx = TENANT):
        return out(c.dm.mark_assignment_missing(asg(c, token).id))

    adders = {"measurements": "add_measurements", "locations": "add_locations", "alerts": "add_alerts",
              "statechanges": "add_state_changes", "responses": "add_command_responses"}
    for kind, fn in EVENT_KINDS.items():
        def make_get(fn=fn, kind=kind):
            def h(token: str, request: Request, page: int = 1, pageSize: int = 100, startDate: str | None = None,
                  endDate: str | None = None, c: Ctx = TENANT):
                return nested_results(c, kind, getattr(c.em, fn)("Assignment", [asg(c, token).id],
                                                                 date_paging(page, pageSize, startDate, endDate)),
                                      request.query_params)
            return h
        r.add_api_route(f"/{{token}}/{kind}", make_get(), methods=["GET"])
        if kind in adders:
            def make_post(add=adders[kind]):
                def h(token: str, body: dict = Body(...), c: Ctx = TENANT):
                    return out(getattr(c.em, add)(asg(c, token).id, body)[0])
                return h
            r.add_api_route(f"/{{token}}/{kind}", make_post(), methods=["POST"])

    @r.get("/{token}/measurements/series")
    def series(token: str, page: int = 1, pageSize: int = 0, startDate: str | None = None, endDate: str | None = None,
               measurementIds: str | None = None, c: Ctx = TENANT):
        ms = c.em.list_measurements_for_index("Assignment", [asg(c, token).id],
                                              date_paging(page, pageSize, startDate, endDate)).results
        want = set(measurementIds.split(",")) if measurementIds else None
        by: dict = {}
        for m in sorted(ms, key=lambda m: m.event_date or 0):
            if want is None or m.name in want:
                by.setdefault(m.name, []).append({"value": m.value, "measurementDate": m.event_date})
        return [{"measurementId": k, "entries": v} for k, v in sorted(by.items())]

    def _invocation_request(c, a, body):
        req = dict(body)
        tok = req.get("commandToken")
        if tok and not req.get("deviceCommandId"):
            cmd = _nf(c.dm.get_device_command_by_token(tok), f"command {tok}")
            req["deviceCommandId"] = cmd.id
        req.setdefault("target", "Assignment")
        req.setdefault("targetId", a.id)
        req.setdefault("initiator", "REST")
        req.setdefault("initiatorId", c.auth.username)
        return req

    @r.post("/{token}/invocations")
    def invoke(token: str, body: dict = Body(...), c: Ctx = TENANT):
        a = asg(c, token)
        return out(c.em.add_command_invocations(a.id, _invocation_request(c, a, body))[0])

    @r.post("/{token}/invocations/schedules/{scheduleToken}")
    def schedule_invocation(token: str, scheduleToken: str, body: dict = Body(...), c: Ctx = TENANT):
        a = asg(c, token)
        return out(c.svc("ScheduleManagement").create_scheduled_job({
            "scheduleToken": scheduleToken, "jobType": "CommandInvocation",
            "jobConfiguration": {"assignmentToken": a.token, "commandToken": body["commandToken"],
                                 "parameterValues": body.get("parameterValues", {})}}))

    @r.post("/{token}/streams")
    def create_stream(token: str, body: dict = Body(...), c: Ctx = TENANT):
        return out(c.dm.create_device_stream(asg(c, token).id, body))

    @r.get("/{token}/streams")
    def list_streams(token: str, page: int = 1, pageSize: int = 100, c: Ctx = TENANT):
        return out(c.dm.list_device_streams(asg(c, token).id, paging(page, pageSize)))

    @r.get("/{token}/streams/{streamId}")
    def get_stream(token: str, streamId: str, c: Ctx = TENANT):
        return out(_nf(c.dm.get_device_stream_by_stream_id(asg(c, token).id, streamId), f"stream {streamId}"))

    # stream chunks as the reference client sends / reads them (``SiteWhereClient.addDeviceStreamData``:
    # binary POST with ?sequenceNumber, ``getDeviceStreamData`` / ``listDeviceStreamData``)
    @r.post("/{token}/streams/{streamId}")
    async def add_stream_data(token: str, streamId: str, sequenceNumber: int, request: Request, c: Ctx = TENANT):
        data = await request.body()
        a = asg(c, token)
        _nf(c.dm.get_device_stream_by_stream_id(a.id, streamId), f"stream {streamId}")
        return out(c.svc("StreamingMedia").add_device_stream_data(a.id, streamId, sequenceNumber, data))

    @r.get("/{token}/streams/{streamId}/data/{sequenceNumber}")
    def get_stream_data(token: str, streamId: str, sequenceNumber: int, c: Ctx = TENANT):
        d = _nf(c.svc("StreamingMedia").get_device_stream_data(asg(c, token).id, streamId, sequenceNumber),
                f"stream {streamId} chunk {sequenceNumber}")
        return Response(d.data, media_type="application/octet-stream")

    @r.get("/{token}/streams/{streamId}/data")
    def list_stream_data(token: str, streamId: str, c: Ctx = TENANT):
        return Response(c.svc("StreamingMedia").get_stream_content(asg(c, token).id, streamId),
                        media_type="application/octet-stream")

    return r


def misc_router(web: WebRest) -> APIRouter:
    r = APIRouter(prefix=API)

    # events / invocations ------------------------------------------------------------
    @r.get("/events/id/{eventId}")
    def event_by_id(eventId: str, c: Ctx = TENANT):
        return out(_nf(c.em.get_device_event_by_id(eventId), f"event {eventId}"))

    @r.get("/events/alternate/{alternateId}")
    def event_by_alt(alternateId: str, c: Ctx = TENANT):
        return out(_nf(c.em.get_device_event_by_alternate_id(alternateId), f"event {alternateId}"))

    @r.get("/invocations/id/{id}")
    def invocation(id: str, c: Ctx = TENANT):
        return out(_nf(c.em.get_device_event_by_id(id), f"invocation {id}"))

    @r.get("/invocations/id/{id}/responses")
    def invocation_responses(id: str, c: Ctx = TENANT):
        return out(c.em.list_command_responses_for_invocation(id))

    @r.get("/invocations/id/{id}/summary")
    def invocation_summary(id: str, c: Ctx = TENANT):
        inv = _nf(c.em.get_device_event_by_id(id), f"invocation {id}")
        cmd = c.dm.get_device_command(inv.device_command_id) if inv.device_command_id else \
            c.dm.get_device_command_by_token(inv.command_token)
        resp = c.em.list_command_responses_for_invocation(id).results
        return {"name": cmd.name if cmd else inv.command_token, "namespace": cmd.namespace if cmd else None,
                "invocationDate": inv.event_date, "parameters": [{"name": k, "value": v} for k, v in
                                                                 (inv.parameter_values or {}).items()],
                "responses": out(resp)}

    # device states ----------------------------------------------------------------------
    @r.post("/devicestates/search")
    def states(request: Request, body: dict = Body({}), c: Ctx = TENANT):
        return nested_results(c, "devicestates", c.svc("DeviceStateManagement").search_device_states(body),
                              request.query_params)

    # batch operations ----------------------------------------------------------------------
    @r.get("/batch")
    def batch_list(page: int = 1, pageSize: int = 100, c: Ctx = TENANT):
        return out(c.svc("BatchManagement").list_batch_operations(paging(page, pageSize)))

    @r.get("/batch/{token}")
    def batch_get(token: str, c: Ctx = TENANT):
        return out(_nf(c.svc("BatchManagement").get_batch_operation_by_token(token), f"batch {token}"))

    @r.get("/batch/{token}/elements")
    def batch_elements(token: str, request: Request, page: int = 1, pageSize: int = 100, c: Ctx = TENANT):
        op = _nf(c.svc("BatchManagement").get_batch_operation_by_token(token), f"batch {token}")
        return nested_results(c, "batchelements", c.svc("BatchManagement").list_batch_operation_elements(
            op.id, paging(page, pageSize)), request.query_params)

    def _device_ids(c, tokens):
        return [_nf(c.dm.get_device_by_token(t), f"device {t}").id for t in tokens]

    @r.post("/batch/command")
    def batch_command(body: dict = Body(...), c: Ctx = TENANT):
        ids = body.get("deviceIds") or _device_ids(c, body.get("deviceTokens", []))
        return out(c.svc("BatchManagement").create_batch_command_invocation({**body, "deviceIds": ids}))

    @r.post("/batch/command/criteria")
    def batch_command_criteria(body: dict = Body(...), c: Ctx = TENANT):
        crit = {k: v for k, v in body.items() if k in ("deviceTypeToken", "excludeAssigned")} | {"pageSize": 0}
        ids = [d.id for d in c.dm.list_devices(crit).results]
        if body.get("groupToken"):
            g = _nf(c.dm.get_device_group_by_token(body["groupToken"]), "group")
            ids = [i for i in ids if i in set(c.dm.expand_group_devices(g.id, None))]
        return out(c.svc("BatchManagement").create_batch_command_invocation({
            "token": body.get("token"), "commandToken": body["commandToken"],
            "parameterValues": body.get("parameterValues", {}), "deviceIds": ids}))

    # external search ----------------------------------------------------------------------
    @r.get("/search")
    def providers(c: Ctx = TENANT):
        return c.svc("EventSearch").list_search_providers()

    @r.get("/search/{providerId}/events")
    def search_events(providerId: str, query: str = "", rows: int = 100, c: Ctx = TENANT):
        return c.svc("EventSearch").search(providerId, query, rows)

    @r.post("/search/{providerId}/raw")
    def search_raw(providerId: str, body: str = Body(...), c: Ctx = TENANT):
        return c.svc("EventSearch").search(providerId, body)

    # system -----------------------------------------------------------------------------
    @r.get("/system/version")
    def version(c: Ctx = GLOBAL):
        return VERSION

    return r


def admin_router(web: WebRest) -> APIRouter:
    r = APIRouter(prefix=API)

    # users ---------------------------------------------------------------------------------
    def um(c):
        return c.svc("UserManagement")

    @r.post("/users")
    def create_user(body: dict = Body(...), c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminUsers)
        return out(um(c).create_user(body))

    @r.get("/users")
    def list_users(page: int = 1, pageSize: int = 100, includeDeleted: bool = False, c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminUsers)
        from ..models.domain import SearchCriteria
        return out(um(c).list_users(SearchCriteria(page, pageSize), includeDeleted))

    @r.get("/users/{username}")
    def get_user(username: str, c: Ctx = GLOBAL):
        if username != c.auth.username:
            c.require(SiteWhereAuthority.AdminUsers)
        return out(_nf(um(c).get_user_by_username(username), f"user {username}"))

    @r.put("/users/{username}")
    def update_user(username: str, body: dict = Body(...), c: Ctx = GLOBAL):
        if username != c.auth.username:
            c.require(SiteWhereAuthority.AdminUsers)
        return out(um(c).update_user(username, body))

    @r.delete("/users/{username}")
    def delete_user(username: str, c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminUsers)
        return out(um(c).delete_user(username))

    @r.get("/users/{username}/authorities")
    def user_authorities(username: str, c: Ctx = GLOBAL):
        return out(SearchResults(*(lambda a: (len(a), a))(um(c).get_granted_authorities_for_user(username))))

    # authorities ---------------------------------------------------------------------------
    @r.post("/authorities")
    def create_authority(body: dict = Body(...), c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminUsers)
        return out(um(c).create_granted_authority(body))

    @r.get("/authorities")
    def list_authorities(c: Ctx = GLOBAL):
        return out(um(c).list_granted_authorities())

    @r.get("/authorities/hierarchy")
    def hierarchy(c: Ctx = GLOBAL):
        auths = um(c).list_granted_authorities().results
        groups: dict = {}
        for a in auths:
            if a.group:
                groups.setdefault(a.parent or a.authority, []).append(out(a))
        roots = [a for a in auths if not a.parent]
        return [{"id": a.authority, "text": a.description, "group": a.group,
                 "items": [x for x in (out(b) for b in auths if b.parent == a.authority)]} for a in roots]

    @r.get("/authorities/{name}")
    def get_authority(name: str, c: Ctx = GLOBAL):
        return out(_nf(um(c).get_granted_authority_by_name(name), f"authority {name}"))

    # tenants -------------------------------------------------------------------------------
    def tm(c):
        return c.svc("TenantManagement")

    def tenant(c, token):
        t = _nf(tm(c).get_tenant_by_token(token), f"tenant {token}")
        if c.auth.username not in t.authorized_user_ids:
            c.require(SiteWhereAuthority.AdminTenants)
        return t

    @r.post("/tenants")
    def create_tenant(body: dict = Body(...), c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminTenants)
        return out(tm(c).create_tenant(body))

    @r.get("/tenants/templates")
    def templates(c: Ctx = GLOBAL):
        return tm(c).get_tenant_templates()

    @r.get("/tenants/datasets")
    def datasets(c: Ctx = GLOBAL):
        return tm(c).get_dataset_templates()

    @r.get("/tenants")
    def list_tenants(page: int = 1, pageSize: int = 100, textSearch: str | None = None, authUserId: str | None = None,
                     c: Ctx = GLOBAL):
        from ..models.domain import SearchCriteria
        user = authUserId if c.auth.has(SiteWhereAuthority.AdminTenants) else c.auth.username
        return out(tm(c).list_tenants(SearchCriteria(page, pageSize), textSearch, user))

    @r.get("/tenants/{token}")
    def get_tenant(token: str, c: Ctx = GLOBAL):
        return out(tenant(c, token))

    @r.put("/tenants/{token}")
    def update_tenant(token: str, body: dict = Body(...), c: Ctx = GLOBAL):
        return out(tm(c).update_tenant(tenant(c, token).id, body))

    @r.delete("/tenants/{token}")
    def delete_tenant(token: str, c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminTenants)
        return out(tm(c).delete_tenant(tenant(c, token).id))

    # instance ------------------------------------------------------------------------------
    def topo():
        return web.topology.snapshot.to_dict() if web.topology else {}

    def mgmt(c, ident):
        return c.svc(f"MicroserviceManagement.{ident}")

    @r.get("/instance/topology")
    def topology(c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.ViewServerInfo)
        return [{"identifier": k, "hosts": v} for k, v in sorted(topo().items())]

    def _split(multitenant: bool):
        from ..assembly import SERVICES_BY_ID
        return [{"identifier": k, "hosts": v} for k, v in sorted(topo().items())
                if getattr(SERVICES_BY_ID.get(k), "multitenant", False) == multitenant]

    @r.get("/instance/topology/global")
    def topology_global(c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.ViewServerInfo)
        return _split(False)

    @r.get("/instance/topology/tenant")
    def topology_tenant(c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.ViewServerInfo)
        return _split(True)

    @r.get("/instance/microservice/{ident}/tenants/{tenantToken}/state")
    def tenant_engine_state(ident: str, tenantToken: str, c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.ViewServerInfo)
        hosts = topo().get(ident, {})
        return {h: {"tenant": tenantToken, "status": s["tenantEngines"].get(tenantToken)} for h, s in hosts.items()}

    @r.get("/instance/microservice/{ident}/configuration/model")
    def config_model(ident: str, c: Ctx = GLOBAL):
        return mgmt(c, ident).get_configuration_model()

    @r.get("/instance/microservice/{ident}/configuration")
    def get_config(ident: str, c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminServer)
        return mgmt(c, ident).get_global_configuration()

    @r.post("/instance/microservice/{ident}/configuration")
    def set_config(ident: str, body: dict = Body(...), c: Ctx = GLOBAL):
        c.require(SiteWhereAuthority.AdminServer)
        return mgmt(c, ident).update_global_configuration(body)

    @r.get("/instance/microservice/{ident}/tenants/{tenantToken}/configuration")
    def get_tenant_config(ident: str, tenantToken: str, c: Ctx = GLOBAL):
        tenant(c, tenantToken)
        return mgmt(c, ident).get_tenant_configuration(tenantToken)

    @r.post("/instance/microservice/{ident}/tenants/{tenantToken}/configuration")
    def set_tenant_config(ident: str, tenantToken: str, body: dict = Body(...), c: Ctx = GLOBAL):
        tenant(c, tenantToken)
        return mgmt(c, ident).update_tenant_configuration(tenantToken, body)

    @r.get("/instance/microservice/{ident}/scripting/templates")
    def script_templates(ident: str, c: Ctx = GLOBAL):
        return [{"id": t, "name": t} for t in mgmt(c, ident).get_script_templates()]

    @r.get("/instance/microservice/{ident}/scripting/templates/{templateId}")
    def script_template(ident: str, templateId: str, c: Ctx = GLOBAL):
        return Response(mgmt(c, ident).get_script_template_content(templateId), media_type="text/plain")

    scripts = web.instance.scripts
    for scope_path, scope_of in (("/instance/microservice/{ident}/scripting/scripts", lambda c, kw: "global"),
                                 ("/instance/microservice/{ident}/tenants/{tenantToken}/scripting/scripts",
                                  lambda c, kw: tenant(c, kw["tenantToken"]).token)):
        add_script_routes(r, scope_path, scope_of, scripts)
    return r


def add_script_routes(r: APIRouter, base: str, scope_of, scripts):
    def ident_scope(c, ident, tenantToken=None):
        c.require(SiteWhereAuthority.AdminServer) if tenantToken is None else None
        return scope_of(c, {"tenantToken": tenantToken}), ident

    def list_scripts(ident: str, tenantToken: str | None = None, c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        return out(scripts.list_scripts(s, i))

    def get_script(ident: str, scriptId: str, tenantToken: str | None = None, c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        return out(scripts.get_script(s, i, scriptId))

    def create_script(ident: str, body: dict = Body(...), tenantToken: str | None = None, c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        content = body.get("content", "")
        if body.get("contentBase64"):
            content = base64.b64decode(body["contentBase64"]).decode()
        return out(scripts.create_script(s, i, body["id"], body.get("name", body["id"]), content,
                                         body.get("description", ""), body.get("interpreterType", "python")))

    def content(ident: str, scriptId: str, versionId: str, tenantToken: str | None = None, c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        return Response(scripts.get_content(s, i, scriptId, versionId), media_type="text/plain")

    def update(ident: str, scriptId: str, versionId: str, body: dict = Body(...), tenantToken: str | None = None,
               c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        content_ = body.get("content")
        if body.get("contentBase64"):
            content_ = base64.b64decode(body["contentBase64"]).decode()
        return out(scripts.update_script(s, i, scriptId, versionId, content_ or "", body.get("name"),
                                         body.get("description")))

    def clone(ident: str, scriptId: str, versionId: str, body: dict = Body({}), tenantToken: str | None = None,
              c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        return out(scripts.clone_script(s, i, scriptId, versionId, body.get("comment", "")))

    def activate(ident: str, scriptId: str, versionId: str, tenantToken: str | None = None, c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        return out(scripts.activate_script(s, i, scriptId, versionId))

    def delete(ident: str, scriptId: str, tenantToken: str | None = None, c: Ctx = GLOBAL):
        s, i = ident_scope(c, ident, tenantToken)
        return out(scripts.delete_script(s, i, scriptId))

    r.add_api_route(base, list_scripts, methods=["GET"])
    r.add_api_route(base, create_script, methods=["POST"])
    r.add_api_route(base + "/{scriptId}", get_script, methods=["GET"])
    r.add_api_route(base + "/{scriptId}", delete, methods=["DELETE"])
    r.add_api_route(base + "/{scriptId}/versions/{versionId}/content", content, methods=["GET"])
    r.add_api_route(base + "/{scriptId}/versions/{versionId}", update, methods=["POST"])
    r.add_api_route(base + "/{scriptId}/versions/{versionId}/clone", clone, methods=["POST"])
    r.add_api_route(base + "/{scriptId}/versions/{versionId}/activate", activate, methods=["POST"])


# ------------------------------------------------------------------------------ microservice
class WebRestMicroservice(GlobalMicroservice):
    """Hosts the REST API (uvicorn on a background thread when ``port`` > 0)."""

    identifier = "web-rest"
    name = "Web/REST"

    def __init__(self, instance, hostname=None, port: int | None = None, host: str = "127.0.0.1"):
        super().__init__(instance, hostname)
        self.port_override, self.host = port, host
        self.app = None
        self._server = None
        self._thread = None

    def default_configuration(self) -> dict:
        return {"port": 8080}

    def microservice_initialize(self, monitor):
        self.app = create_app(self.instance, self.topology, bool(self.config.get("cors", True)),
                              self.config.get("adminUiDir"))

    def microservice_start(self, monitor):
        port = self.port_override if self.port_override is not None else int(self.config.get("port", 8080))
        if port <= 0:
            return
        import uvicorn
        self._server = uvicorn.Server(uvicorn.Config(self.app, host=self.host, port=port, log_level="warning"))
        self._thread = threading.Thread(target=self._server.run, daemon=True, name="web-rest")
        self._thread.start()

    def microservice_stop(self, monitor):
        if self._server is not None:
            self._server.should_exit = True
            self._thread.join(timeout=5)
            self._server = None

    def configuration_updated(self, doc):
        pass
