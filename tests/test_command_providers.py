"""Command delivery providers beyond MQTT: Twilio SMS over its REST API and CoAP to the device,
routed per device type (reference ``twilio/TwilioCommandDeliveryProvider``,
``destination/coap/CoapCommandDeliveryProvider`` + ``MetadataCoapParameterExtractor``,
``destination/sms/SmsParameterExtractor``, ``DeviceTypeMappingCommandRouter``).

The Twilio API is a local stand-in speaking the same endpoint (no network here); the CoAP device
is this framework's CoAP server in ``paths="any"`` mode.
"""
from __future__ import annotations

import base64
import json
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from sitewhere_amd.assembly import SiteWhereInstance
from sitewhere_amd.edges.receivers import CoapReceiver
from sitewhere_amd.runtime.config import dump_document


class _Twilio(BaseHTTPRequestHandler):
    sent: list = []
    fail = False

    def do_POST(self):  # noqa: N802
        body = self.rfile.read(int(self.headers.get("Content-Length", 0)))
        form = dict(urllib.parse.parse_qsl(body.decode()))
        auth = base64.b64decode(self.headers.get("Authorization", "Basic ")[6:]).decode()
        if auth != "AC123:tok" or self.path != "/2010-04-01/Accounts/AC123/Messages.json":
            self._reply(401, {"code": 20003, "message": "Authenticate"})
        elif _Twilio.fail:
            self._reply(400, {"code": 21211, "message": "The 'To' number is not a valid phone number."})
        else:
            _Twilio.sent.append(form)
            self._reply(201, {"sid": f"SM{len(_Twilio.sent):032d}", "status": "queued"})

    def _reply(self, code, doc):
        b = json.dumps(doc).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(b)))
        self.end_headers()
        self.wfile.write(b)

    def log_message(self, *a):
        pass


def wait(cond, t=20.0):
    end = time.time() + t
    while time.time() < end and not cond():
        time.sleep(0.05)
    return cond()


def test_sms_and_coap_destinations_routed_by_device_type():
    api = ThreadingHTTPServer(("127.0.0.1", 0), _Twilio)
    threading.Thread(target=api.serve_forever, daemon=True).start()
    got = []

    class Src:
        def on_encoded_event_received(self, recv, payload, md):
            got.append((bytes(payload), md["path"]))
    device = CoapReceiver(paths="any")
    device.source = Src()
    device.start(None)
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "default"), sw.api("DeviceEventManagement", "default")
        tab = run(lambda: dm.get_device_by_token("galaxytab-000"))
        hab = run(lambda: dm.get_device_by_token("openhab-000"))
        tab_type = run(lambda: dm.get_device_type(tab.device_type_id)).token
        hab_type = run(lambda: dm.get_device_type(hab.device_type_id)).token
        run(lambda: dm.update_device(tab.id, {"metadata": {"sms_phone": "+15550100"}}))
        run(lambda: dm.update_device(hab.id, {"metadata": {"coap_hostname": "127.0.0.1",
                                                           "coap_port": str(device.port), "coap_url": "cmd/in"}}))
        cd_ms = sw["command-delivery"]
        before = cd_ms.get_tenant_engine("default")
        cfg = json.loads(json.dumps(cd_ms.tenant_configuration("default")))
        cfg["destinations"] = [
            {"id": "sms", "encoder": "json", "provider": "sms", "accountSid": "AC123", "authToken": "tok",
             "fromPhone": "+15550199", "apiBase": f"http://127.0.0.1:{api.server_port}"},
            {"id": "coap", "encoder": "json", "provider": "coap"}]
        cfg["router"] = {"type": "device-type-mapping", "mappings": {tab_type: "sms", hab_type: "coap"}}
        sw.instance.coord.put(cd_ms.tenant_config_path("default"), dump_document(cfg))
        assert wait(lambda: (e := cd_ms.get_tenant_engine("default")) is not None and e is not before
                    and e.status.value == "Started" and "sms" in e.destinations)
        cd = cd_ms.get_tenant_engine("default")

        def invoke(dev, cmd_token):
            cmd = run(lambda: dm.get_device_command_by_token(cmd_token))
            run(lambda: em.add_command_invocations(dev.device_assignment_id, {
                "initiator": "REST", "initiatorId": "admin", "target": "Assignment", "commandToken": cmd.token,
                "deviceCommandId": cmd.id, "parameterValues": {}}))
        invoke(tab, "galaxytab-ping")
        invoke(hab, "openhab-ping")
        assert wait(lambda: len(_Twilio.sent) == 1 and len(got) == 1)
        sms = _Twilio.sent[0]
        assert sms["To"] == "+15550100" and sms["From"] == "+15550199"
        assert json.loads(sms["Body"])["command"]["token"] == "galaxytab-ping"
        payload, path = got[0]
        assert path == "cmd/in" and json.loads(payload)["command"]["token"] == "openhab-ping"
        # the counters move after the provider returns: wait for them rather than racing the worker
        assert wait(lambda: cd.destinations["sms"].delivered == 1 and cd.destinations["coap"].delivered == 1)
        # an API refusal is an undelivered command (reference: undelivered-command-invocations topic)
        _Twilio.fail = True
        u0 = cd.undelivered
        invoke(tab, "galaxytab-ping")
        assert wait(lambda: cd.undelivered == u0 + 1)
        topic = sw.instance.naming.undelivered_command_invocations("default")
        cons = sw.instance.bus.consumer("undelivered-check", [topic])
        recs = [r for rs in cons.poll(2000).values() for r in rs]
        assert any("not a valid phone number" in json.loads(r.value)["error"] for r in recs)
    finally:
        _Twilio.fail = False
        sw.stop()
        device.stop(None)
        api.shutdown()
