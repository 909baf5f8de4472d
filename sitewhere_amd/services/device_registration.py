"""service-device-registration: auto-registration of devices (multitenant).

Reference: ``DefaultRegistrationManager.java:40-115`` -- get-or-create the device (``allowNewDevices``,
default device type / customer / area), assign it if unassigned, acknowledge to the device;
``DeviceRegistrationEventsConsumer`` (registration topic) and ``UnregisteredEventsConsumer``
(events from unknown devices: optionally auto-register, then re-inject into ``inbound-reprocess-events``).
"""
from __future__ import annotations


from ..core.errors import SiteWhereException
from ..runtime.consumers import BusConsumer
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from ..bus import payloads

NEW_REGISTRATION, ALREADY_REGISTERED, REGISTRATION_ERROR = "NEW_REGISTRATION", "ALREADY_REGISTERED", "REGISTRATION_ERROR"


class RegistrationManager:
    def __init__(self, engine, cfg: dict):
        self.engine = engine
        self.allow_new = bool(cfg.get("allowNewDevices", True))
        self.default_type = cfg.get("defaultDeviceTypeToken")
        self.default_customer = cfg.get("defaultCustomerToken")
        self.default_area = cfg.get("defaultAreaToken")
        self.auto_assign = bool(cfg.get("autoAssign", True))
        self.acks: list[dict] = []

    def _dm(self):
        return self.engine.ms.api("DeviceManagement", self.engine.tenant.token)

    def handle_device_registration(self, token: str, req: dict) -> dict:
        dm = self._dm()
        device = dm.get_device_by_token(token)
        state = ALREADY_REGISTERED
        if device is None:
            if not self.allow_new:
                return self._ack(token, REGISTRATION_ERROR, "NEW_DEVICES_NOT_ALLOWED")
            dtype = req.get("deviceTypeToken") or self.default_type
            if not dtype or dm.get_device_type_by_token(dtype) is None:
                return self._ack(token, REGISTRATION_ERROR, "INVALID_SPECIFICATION")
            device = dm.create_device({"token": token, "deviceTypeToken": dtype, "metadata": req.get("metadata", {})})
            state = NEW_REGISTRATION
        if self.auto_assign and not device.device_assignment_id:
            dm.create_device_assignment({"deviceToken": token,
                                         "customerToken": req.get("customerToken") or self.default_customer,
                                         "areaToken": req.get("areaToken") or self.default_area})
        return self._ack(token, state)

    def _ack(self, token, state, error=None) -> dict:
        ack = {"deviceToken": token, "state": state, "errorType": error}
        self.acks.append(ack)
        try:
            cmd = self.engine.ms.api("CommandDelivery", self.engine.tenant.token)
            cmd.deliver_system_command(token, {"type": "RegistrationAck", "state": state, "errorType": error})
        except Exception:
            pass  # command delivery not deployed / device unreachable: the ack stays recorded
        return ack

    def handle_unregistered_event(self, payload: dict) -> bool:
        """Auto-register with the default device type, then reprocess the event."""
        if not (self.allow_new and self.default_type):
            return False
        ack = self.handle_device_registration(payload["deviceToken"], {})
        if ack["state"] == REGISTRATION_ERROR:
            return False
        n = self.engine.ms.instance.naming
        self.engine.ms.producer.send(n.inbound_reprocess_events(self.engine.tenant.token), payload["deviceToken"],
                                     payloads.encode_inbound(payload))
        return True


class DeviceRegistrationTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        self.manager = RegistrationManager(self, self.config)
        n, t = self.ms.instance.naming, self.tenant.token
        # registration is control plane: a failing registration is retried, never dead-lettered
        self.reg_consumer = BusConsumer(self, "registration-events", [n.device_registration_events(t)], self._on_reg,
                                        max_attempts=None)
        self.unreg_consumer = BusConsumer(self, "unregistered-events", [n.unregistered_device_events(t)], self._on_unreg)
        self.api = {"DeviceRegistration": RegistrationApi(self)}

    def _on_reg(self, recs):
        for r in recs:
            p = payloads.decode_inbound(r.value, registration=True)
            try:
                self.manager.handle_device_registration(p["deviceToken"], p["eventCreateRequest"]["request"])
            except SiteWhereException:
                self.logger.exception("registration failed")

    def _on_unreg(self, recs):
        """Events of unknown devices.  Without auto-registration (no default device type) they are
        only acknowledged -- nothing is decoded.  With it, each device of the poll is registered once
        (records are keyed by device token) and its events go to the reprocess topic unchanged (the
        value already is the ``GInboundEventPayload`` that topic carries)."""
        m = self.manager
        if not (m.allow_new and m.default_type):
            return
        by_token: dict[str, list] = {}
        for r in recs:
            tok = bytes(r.key).decode() if r.key else payloads.decode_inbound(r.value)["deviceToken"]
            by_token.setdefault(tok, []).append(r)
        topic = self.ms.instance.naming.inbound_reprocess_events(self.tenant.token)
        for tok, rs in by_token.items():
            if m.handle_device_registration(tok, {})["state"] == REGISTRATION_ERROR:
                continue
            self.ms.producer.send_batch(topic, [(tok, bytes(r.value)) for r in rs])

    def tenant_start(self, monitor):
        self.start_nested_component(self.reg_consumer, monitor, require=True)
        m = self.manager
        if m.allow_new and m.default_type:
            # without auto-registration nothing is done with those events: no consumer reads them
            # (at 1% unknown devices that is 10^4 records per 10^6-event batch of pure overhead)
            self.start_nested_component(self.unreg_consumer, monitor, require=True)

    def tenant_stop(self, monitor):
        self.reg_consumer.lifecycle_stop(monitor)
        if self.unreg_consumer.status.value == "Started":
            self.unreg_consumer.lifecycle_stop(monitor)


class RegistrationApi:
    def __init__(self, e):
        self._e = e

    def register_device(self, token: str, request: dict) -> dict:
        return self._e.manager.handle_device_registration(token, request)

    def list_acknowledgements(self) -> list:
        return list(self._e.manager.acks)


class DeviceRegistrationMicroservice(MultitenantMicroservice):
    identifier = "device-registration"
    name = "Device Registration"

    def service_names(self):
        return ["DeviceRegistration"]

    def create_tenant_engine(self, tenant):
        return DeviceRegistrationTenantEngine(self, tenant)
