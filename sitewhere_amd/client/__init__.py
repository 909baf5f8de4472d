"""Python REST client SDK (reference ``sitewhere-client``: ``ISiteWhereClient.java`` / ``SiteWhereClient.java``).

Every ``ISiteWhereClient`` method has a snake_case counterpart here.  The reference SDK predates
parts of the 2.0 REST API, so its names map onto 2.0 resources: *site* -> area, *hardware id* ->
device token, asset *module* -> asset type.

Obtains a JWT from ``/sitewhere/authapi/jwt`` with basic credentials, then sends it as a bearer
token together with the tenant id / tenant auth headers.  ``transport`` may be any object with a
``request(method, url, headers=, json=, params=)`` returning an httpx-like response -- an
``httpx.Client`` for a live server or FastAPI's ``TestClient`` in-process.
"""
from __future__ import annotations

import base64

API = "/sitewhere/api"


class SiteWhereClientError(Exception):
    def __init__(self, status: int, message: str, code: str | None = None):
        super().__init__(f"{status}: {message}")
        self.status, self.message, self.code = status, message, code


class SiteWhereClient:
    def __init__(self, base_url: str = "http://127.0.0.1:8080", username: str = "admin", password: str = "password",
                 tenant_id: str | None = "default", tenant_auth: str | None = "sitewhere1234567890", transport=None):
        self.base = base_url.rstrip("/")
        if transport is None:
            import httpx
            transport = httpx.Client(timeout=30.0)
        self.http = transport
        self.username, self.password = username, password
        self.tenant_id, self.tenant_auth = tenant_id, tenant_auth
        self.jwt: str | None = None

    # ---- plumbing ---------------------------------------------------------------------------
    def authenticate(self) -> str:
        basic = base64.b64encode(f"{self.username}:{self.password}".encode()).decode()
        r = self.http.request("GET", f"{self.base}/sitewhere/authapi/jwt", headers={"Authorization": f"Basic {basic}"})
        self._check(r)
        self.jwt = r.headers["X-Sitewhere-JWT"]
        return self.jwt

    def _headers(self, tenant: bool = True) -> dict:
        if self.jwt is None:
            self.authenticate()
        h = {"Authorization": f"Bearer {self.jwt}"}
        if tenant and self.tenant_id:
            h["X-SiteWhere-Tenant-Id"] = self.tenant_id
            h["X-SiteWhere-Tenant-Auth"] = self.tenant_auth or ""
        return h

    @staticmethod
    def _check(r):
        if r.status_code >= 400:
            raise SiteWhereClientError(r.status_code, r.headers.get("X-SiteWhere-Error", r.text),
                                       r.headers.get("X-SiteWhere-Error-Code"))

    def _call(self, method: str, path: str, body=None, params=None, tenant: bool = True, raw: bool = False):
        r = self.http.request(method, f"{self.base}{API}{path}", headers=self._headers(tenant), json=body,
                              params={k: v for k, v in (params or {}).items() if v is not None})
        self._check(r)
        if raw:
            return r.content
        return r.json() if r.content else None

    def get(self, path, **params):
        return self._call("GET", path, params=params)

    def post(self, path, body=None):
        return self._call("POST", path, body)

    def put(self, path, body=None):
        return self._call("PUT", path, body)

    def delete(self, path):
        return self._call("DELETE", path)

    # ---- system / users / tenants --------------------------------------------------------------
    def get_version(self):
        return self._call("GET", "/system/version", tenant=False)

    def get_site_where_version(self):
        return self.get_version()

    def list_users(self, page: int = 1, page_size: int = 100):
        return self._call("GET", "/users", params={"page": page, "pageSize": page_size}, tenant=False)

    def create_user(self, request: dict):
        return self._call("POST", "/users", request, tenant=False)

    def get_user(self, username: str):
        return self._call("GET", f"/users/{username}", tenant=False)

    def list_tenants(self):
        return self._call("GET", "/tenants", tenant=False)

    def create_tenant(self, request: dict):
        return self._call("POST", "/tenants", request, tenant=False)

    def get_tenant(self, token: str):
        return self._call("GET", f"/tenants/{token}", tenant=False)

    # ---- device model ------------------------------------------------------------------------------
    def create_device_type(self, request: dict):
        return self.post("/devicetypes", request)

    def get_device_type(self, token: str):
        return self.get(f"/devicetypes/{token}")

    def list_device_types(self, **crit):
        return self.get("/devicetypes", **crit)

    def create_device_command(self, request: dict):
        return self.post("/commands", request)

    def list_device_commands(self, device_type_token: str | None = None):
        return self.get("/commands", deviceTypeToken=device_type_token)

    def create_device(self, request: dict):
        return self.post("/devices", request)

    def get_device(self, token: str):
        return self.get(f"/devices/{token}")

    def update_device(self, token: str, request: dict):
        return self.put(f"/devices/{token}", request)

    def delete_device(self, token: str):
        return self.delete(f"/devices/{token}")

    def list_devices(self, **crit):
        return self.get("/devices", **crit)

    def get_current_assignment(self, device_token: str):
        return self.get(f"/devices/{device_token}/assignment")

    def create_device_assignment(self, request: dict):
        return self.post("/assignments", request)

    def get_device_assignment(self, token: str):
        return self.get(f"/assignments/{token}")

    def end_device_assignment(self, token: str):
        return self.post(f"/assignments/{token}/end")

    def create_area(self, request: dict):
        return self.post("/areas", request)

    def create_customer(self, request: dict):
        return self.post("/customers", request)

    def create_zone(self, request: dict):
        return self.post("/zones", request)

    def create_device_group(self, request: dict):
        return self.post("/devicegroups", request)

    def add_device_group_elements(self, group_token: str, elements: list):
        return self.put(f"/devicegroups/{group_token}/elements", elements)

    def create_asset_type(self, request: dict):
        return self.post("/assettypes", request)

    def create_asset(self, request: dict):
        return self.post("/assets", request)

    def get_device_type_by_token(self, token: str):
        return self.get_device_type(token)

    def update_device_type(self, token: str, request: dict):
        return self.put(f"/devicetypes/{token}", request)

    def delete_device_type(self, token: str):
        return self.delete(f"/devicetypes/{token}")

    def get_device_by_hardware_id(self, token: str):
        return self.get_device(token)

    def get_current_assignment_for_device(self, device_token: str):
        return self.get_current_assignment(device_token)

    def list_device_assignment_history(self, device_token: str, **crit):
        return self.get(f"/devices/{device_token}/assignments", **crit)

    def get_device_assignment_by_token(self, token: str):
        return self.get_device_assignment(token)

    def update_device_assignment(self, token: str, request: dict):
        return self.put(f"/assignments/{token}", request)

    def update_device_assignment_metadata(self, token: str, metadata: dict):
        return self.update_device_assignment(token, {"metadata": metadata})

    def delete_device_assignment(self, token: str):
        return self.delete(f"/assignments/{token}")

    def get_area_by_token(self, token: str):
        return self.get(f"/areas/{token}")

    def list_areas(self, **crit):
        return self.get("/areas", **crit)

    def list_assignments_for_site(self, area_token: str, **crit):
        return self.get(f"/areas/{area_token}/assignments", **crit)

    def list_zones_for_site(self, area_token: str, **crit):
        return self.get("/zones", areaToken=area_token, **crit)

    def get_device_group_by_token(self, token: str):
        return self.get(f"/devicegroups/{token}")

    def list_device_groups(self, **crit):
        return self.get("/devicegroups", **crit)

    def delete_device_group(self, token: str):
        return self.delete(f"/devicegroups/{token}")

    def list_device_group_elements(self, group_token: str, **crit):
        return self.get(f"/devicegroups/{group_token}/elements", **crit)

    def delete_device_group_elements(self, group_token: str, element_ids: list):
        return self._call("DELETE", f"/devicegroups/{group_token}/elements", element_ids)

    def get_assets_by_module_id(self, asset_type_token: str, **crit):
        return self.get("/assets", assetTypeToken=asset_type_token, **crit)

    def get_assignments_for_asset(self, asset_token: str, **crit):
        return self.get("/assignments", assetToken=asset_token, **crit)

    # ---- events ------------------------------------------------------------------------------------------
    def add_device_event_batch(self, device_token: str, batch: dict):
        """Measurements / locations / alerts for a device's active assignment in one call."""
        return self.post(f"/devices/{device_token}/batch", batch)

    def create_device_measurements(self, assignment_token: str, request: dict):
        return self.post(f"/assignments/{assignment_token}/measurements", request)

    def create_device_location(self, assignment_token: str, request: dict):
        return self.post(f"/assignments/{assignment_token}/locations", request)

    def create_device_alert(self, assignment_token: str, request: dict):
        return self.post(f"/assignments/{assignment_token}/alerts", request)

    def create_device_command_invocation(self, assignment_token: str, request: dict):
        return self.post(f"/assignments/{assignment_token}/invocations", request)

    def list_device_measurements(self, assignment_token: str, **crit):
        return self.list_measurements(assignment_token, **crit)

    def list_device_locations(self, assignment_token: str, **crit):
        return self.list_locations(assignment_token, **crit)

    def list_device_alerts(self, assignment_token: str, **crit):
        return self.list_alerts(assignment_token, **crit)

    def list_device_command_invocations(self, assignment_token: str, **crit):
        return self.get(f"/assignments/{assignment_token}/invocations", **crit)

    def create_device_stream(self, assignment_token: str, request: dict):
        return self.post(f"/assignments/{assignment_token}/streams", request)

    def get_device_stream(self, assignment_token: str, stream_id: str):
        return self.get(f"/assignments/{assignment_token}/streams/{stream_id}")

    def list_device_streams(self, assignment_token: str, **crit):
        return self.get(f"/assignments/{assignment_token}/streams", **crit)

    def add_device_stream_data(self, assignment_token: str, stream_id: str, sequence_number: int, data: bytes):
        r = self.http.request("POST", f"{self.base}{API}/assignments/{assignment_token}/streams/{stream_id}",
                              headers=dict(self._headers(), **{"Content-Type": "application/octet-stream"}),
                              params={"sequenceNumber": int(sequence_number)}, content=bytes(data))
        self._check(r)
        return r.json()

    def get_device_stream_data(self, assignment_token: str, stream_id: str, sequence_number: int) -> bytes:
        return self._call("GET", f"/assignments/{assignment_token}/streams/{stream_id}/data/{int(sequence_number)}",
                          raw=True)

    def list_device_stream_data(self, assignment_token: str, stream_id: str) -> bytes:
        """The stream's chunks in sequence order, concatenated."""
        return self._call("GET", f"/assignments/{assignment_token}/streams/{stream_id}/data", raw=True)

    def add_measurement(self, assignment_token: str, name: str, value: float, event_date: int | None = None, **extra):
        return self.post(f"/assignments/{assignment_token}/measurements",
                         {"name": name, "value": value, "eventDate": event_date, **extra})

    def add_location(self, assignment_token: str, latitude: float, longitude: float, elevation=None, **extra):
        return self.post(f"/assignments/{assignment_token}/locations",
                         {"latitude": latitude, "longitude": longitude, "elevation": elevation, **extra})

    def add_alert(self, assignment_token: str, type_: str, message: str, level: str = "Info", **extra):
        return self.post(f"/assignments/{assignment_token}/alerts",
                         {"type": type_, "message": message, "level": level, **extra})

    def list_measurements(self, assignment_token: str, **crit):
        return self.get(f"/assignments/{assignment_token}/measurements", **crit)

    def list_locations(self, assignment_token: str, **crit):
        return self.get(f"/assignments/{assignment_token}/locations", **crit)

    def list_alerts(self, assignment_token: str, **crit):
        return self.get(f"/assignments/{assignment_token}/alerts", **crit)

    def measurement_series(self, assignment_token: str, **crit):
        return self.get(f"/assignments/{assignment_token}/measurements/series", **crit)

    def invoke_command(self, assignment_token: str, command_token: str, parameters: dict | None = None):
        return self.post(f"/assignments/{assignment_token}/invocations",
                         {"commandToken": command_token, "parameterValues": parameters or {}})

    def get_event(self, event_id: str):
        return self.get(f"/events/id/{event_id}")

    def get_event_by_alternate_id(self, alternate_id: str):
        return self.get(f"/events/alternate/{alternate_id}")

    # ---- batch / schedules / labels / states -------------------------------------------------------------
    def create_batch_command_invocation(self, token: str, command_token: str, device_tokens: list, params=None):
        return self.post("/batch/command", {"token": token, "commandToken": command_token,
                                            "deviceTokens": device_tokens, "parameterValues": params or {}})

    def get_batch_operation(self, token: str):
        return self.get(f"/batch/{token}")

    def create_schedule(self, request: dict):
        return self.post("/schedules", request)

    def create_scheduled_job(self, request: dict):
        return self.post("/jobs", request)

    def get_device_label(self, device_token: str, generator: str = "qrcode") -> bytes:
        return self._call("GET", f"/devices/{device_token}/label/{generator}", raw=True)

    def search_device_states(self, criteria: dict | None = None):
        return self.post("/devicestates/search", criteria or {})
