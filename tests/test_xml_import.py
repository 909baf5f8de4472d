"""Reference Spring XML tenant templates -> JSON configuration (runtime/xml_import.py).

Reads the reference's own template files (``service-tenant-management/dockerimage/templates``);
the end-to-end case boots a tenant from the imported ``default`` template -- MongoDB datastores on
the in-process MongoDB server, MQTT event sources on the in-process broker -- and delivers a
protobuf measurement over MQTT to the topic the reference's XML names."""
from __future__ import annotations

import os
import time

import pytest

from sitewhere_amd.runtime.xml_import import convert_service, import_tenant_template, register_reference_templates

REF = "/root/reference/service-tenant-management/dockerimage/templates"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference templates not present")


def test_all_reference_templates_import_cleanly():
    for name in ("default", "mongodb", "influxdb", "cassandra", "stomp"):
        t = import_tenant_template(os.path.join(REF, name))
        assert t["warnings"] == [], (name, t["warnings"])
        assert set(t["services"]) >= {"event-sources", "event-management", "device-management", "inbound-processing"}
    d = import_tenant_template(os.path.join(REF, "default"))["services"]
    srcs = d["event-sources"]["sources"]
    assert [s["id"] for s in srcs] == ["protobuf", "json"]
    assert srcs[0]["decoder"] == "protobuf" and srcs[1]["decoder"] == "json"
    assert srcs[0]["receivers"][0] == {"type": "mqtt", "host": "${mqtt.host:localhost}", "port": "${mqtt.port:1883}",
                                       "topic": "SiteWhere/[[tenant.token]]/input/protobuf", "numThreads": 1}
    assert d["inbound-processing"]["processingThreadCount"] == 25
    assert d["device-state"]["presence"] == {"checkInterval": "PT10M", "missingInterval": "PT8H"}
    assert d["device-registration"]["allowNewDevices"] is False
    assert d["event-management"]["datastore"]["type"] == "mongodb" and d["event-management"]["buffered"] is True
    assert d["command-delivery"]["router"] == {"type": "single-choice", "destination": "default"}
    assert d["command-delivery"]["destinations"][0]["provider"] == "mqtt"
    st = import_tenant_template(os.path.join(REF, "stomp"))["services"]["event-sources"]["sources"]
    assert st == [{"id": "stomp", "decoder": "json-batch", "receivers": [
        {"type": "activemq-broker", "transportUri": "stomp://localhost:2345?trace=true", "queueName": "SITEWHERE.STOMP",
         "numConsumers": 5, "brokerName": None}]}]
    cq = import_tenant_template(os.path.join(REF, "cassandra"))["services"]
    assert cq["event-management"]["datastore"]["type"] == "cassandra"
    # overlays keep the reference default's other services (MQTT sources, MongoDB registries)
    assert cq["event-sources"]["sources"][0]["id"] == "protobuf" and cq["device-management"]["datastore"]["type"] == "mongodb"
    assert import_tenant_template(os.path.join(REF, "influxdb"))["services"]["event-management"]["datastore"]["type"] \
        == "influxdb"


def test_unknown_elements_are_reported():
    xml = b"""<beans xmlns:op="x"><op:outbound-connectors>
        <op:mqtt-connector connectorId="m1" hostname="h" port="1884" outboundTopic="out/${tenant.token}"/>
        <op:mystery-connector connectorId="z"/></op:outbound-connectors></beans>"""
    from sitewhere_amd.runtime.xml_import import _Ctx
    ctx = _Ctx()
    doc = convert_service("outbound-connectors", xml, ctx)
    assert doc == {"connectors": [{"id": "m1", "type": "mqtt", "host": "h", "port": 1884,
                                   "topic": "out/[[tenant.token]]"}]}
    assert ctx.warnings == ["outbound-connectors: <mystery-connector> not imported"]


def test_receiver_attributes_and_script_ids_import():
    """MQTT broker attributes (``connector-common.xsd`` mqtt-broker-attributes), socket interaction
    handler factories, WebSocket client receivers and scripted REST polling come through the import;
    script ids resolve against script management when the tenant engine builds the source."""
    xml = b"""<beans xmlns:es="x"><es:event-sources>
      <es:mqtt-event-source sourceId="m" protocol="tls" hostname="broker" port="8883" username="u" password="p"
          trustStorePath="/etc/ca.pem" clientId="sw-${tenant.token}" cleanSession="false" qos="EXACTLY_ONCE"
          topic="in/${tenant.token}" numThreads="3"><es:json-device-request-decoder/></es:mqtt-event-source>
      <es:socket-event-source sourceId="s" port="9000">
          <es:groovy-interaction-handler-factory scriptId="sock-handler"/>
          <es:groovy-event-decoder scriptId="my-decoder"/></es:socket-event-source>
      <es:web-socket-event-source sourceId="w" webSocketUrl="ws://feed:80/x" payloadType="STRING">
          <es:header name="Authorization" value="Bearer t"/><es:json-device-request-decoder/>
      </es:web-socket-event-source>
      <es:polling-rest-event-source sourceId="r" baseUrl="http://api/v1" pollIntervalMs="5000" scriptId="poller"
          username="a" password="b"><es:json-device-request-decoder/></es:polling-rest-event-source>
    </es:event-sources></beans>"""
    from sitewhere_amd.runtime.xml_import import _Ctx
    ctx = _Ctx()
    srcs = {s["id"]: s for s in convert_service("event-sources", xml, ctx)["sources"]}
    assert ctx.warnings == []
    assert srcs["m"]["receivers"][0] == {
        "type": "mqtt", "host": "broker", "port": 8883, "protocol": "tls", "username": "u", "password": "p",
        "trustStorePath": "/etc/ca.pem", "clientId": "sw-[[tenant.token]]", "cleanSession": "false",
        "qos": "EXACTLY_ONCE", "topic": "in/[[tenant.token]]", "numThreads": 3}
    assert srcs["s"]["receivers"][0] == {"type": "socket", "host": "0.0.0.0", "port": 9000, "numThreads": 4,
                                         "handler": "script", "script": "sock-handler"}
    assert srcs["s"]["decoder"] == "script" and srcs["s"]["script"] == "my-decoder"
    assert srcs["w"]["receivers"][0] == {"type": "websocket", "host": "0.0.0.0", "port": 8585, "payloadType": "string",
                                         "webSocketUrl": "ws://feed:80/x", "headers": {"Authorization": "Bearer t"}}
    assert srcs["r"]["receivers"][0] == {"type": "rest-poll", "baseUrl": "http://api/v1", "interval": 5.0,
                                         "username": "a", "password": "b", "scriptId": "poller"}


def test_composite_and_coap_decoders_import():
    xml = b"""<beans xmlns:es="x"><es:event-sources>
      <es:socket-event-source sourceId="bin" port="9001"><es:composite-decoder>
        <es:groovy-device-metadata-extractor scriptId="extract"/>
        <es:choices>
          <es:device-specification-decoder-choice token="tracker"><es:groovy-event-decoder scriptId="trk"/>
          </es:device-specification-decoder-choice>
          <es:device-specification-decoder-choice token="gw"><es:json-device-request-decoder/>
          </es:device-specification-decoder-choice>
        </es:choices></es:composite-decoder></es:socket-event-source>
      <es:coap-server-event-source sourceId="coap" port="5683"><es:coap-json-decoder/></es:coap-server-event-source>
      <es:activemq-client-event-source sourceId="amq" remoteUri="tcp://broker:61613" queueName="Q" numConsumers="2">
        <es:json-device-request-decoder/></es:activemq-client-event-source>
    </es:event-sources></beans>"""
    from sitewhere_amd.runtime.xml_import import _Ctx
    ctx = _Ctx()
    srcs = {s["id"]: s for s in convert_service("event-sources", xml, ctx)["sources"]}
    assert ctx.warnings == []
    assert srcs["bin"]["decoder"] == {"type": "composite", "extractorScript": "extract",
                                      "choices": {"tracker": {"type": "script", "script": "trk"}, "gw": "json"}}
    assert srcs["coap"]["decoder"] == "coap-json" and srcs["coap"]["receivers"][0]["type"] == "coap"
    assert srcs["amq"]["receivers"][0] == {"type": "activemq", "host": "broker", "port": 61613,
                                           "destination": "/queue/Q", "numThreads": 2}


def test_script_ids_resolve_through_script_management():
    """A source configured with a script id (as imported from the reference) runs the active
    version stored in script management; activating another version changes the next engine."""
    import json

    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.runtime.config import dump_document
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        sm = sw.instance.scripts
        v1 = ("import json\ndef decode(payload, metadata):\n    d = json.loads(payload)\n"
              "    return [{'deviceToken': d['t'], 'type': 'DeviceMeasurement', 'request': {'name': 'v1', 'value': d['v']}}]\n")
        meta = sm.create_script("default", "event-sources", "my-decoder", "My decoder", v1)
        es_ms = sw["event-sources"]
        before = es_ms.get_tenant_engine("default")
        doc = json.loads(json.dumps(es_ms.tenant_configuration("default")))
        doc["sources"].append({"id": "scripted", "decoder": "script", "script": "my-decoder", "receivers": []})
        doc["sources"].append({"id": "inline", "decoder": {"type": "script", "script": v1}, "receivers": []})
        sw.instance.coord.put(es_ms.tenant_config_path("default"), dump_document(doc))
        assert wait_for(lambda: (e := es_ms.get_tenant_engine("default")) is not None and e is not before
                        and e.status.value == "Started" and "scripted" in e.manager.sources)
        eng = es_ms.get_tenant_engine("default")
        assert eng.manager.sources["scripted"].decoder.source == v1 == eng.manager.sources["inline"].decoder.source
        v2 = sm.clone_script("default", "event-sources", "my-decoder", meta.active_version).versions[-1]["versionId"]
        sm.update_script("default", "event-sources", "my-decoder", v2, v1.replace("'v1'", "'v2'"))
        sm.activate_script("default", "event-sources", "my-decoder", v2)
        assert eng.script_source("my-decoder") == v1.replace("'v1'", "'v2'")
        assert eng.script_source({"scriptId": "my-decoder", "version": meta.active_version}) == v1
        with pytest.raises(Exception, match="not found"):
            eng.script_source("no-such-script")
    finally:
        sw.stop()


def wait_for(cond, t=30.0):
    end = time.time() + t
    while time.time() < end and not cond():
        time.sleep(0.05)
    return cond()


def test_tenant_boots_from_imported_reference_default_template(monkeypatch):
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.edges.mqtt import MqttBroker, MqttClient
    from sitewhere_amd.models import wire
    from sitewhere_amd.persistence.mongo_server import MiniMongoServer
    from sitewhere_amd.services.tenant_management import TENANT_TEMPLATES
    mongo = MiniMongoServer(port=0).start()
    broker = MqttBroker().start()
    monkeypatch.setenv("MONGODB_URI", f"mongodb://127.0.0.1:{mongo.port}")
    monkeypatch.setenv("MQTT_HOST", "127.0.0.1")
    monkeypatch.setenv("MQTT_PORT", str(broker.port))
    ids = register_reference_templates(REF)
    sw = None
    try:
        assert {"ref-default", "ref-stomp", "ref-mongodb"} <= set(ids)
        sw = SiteWhereInstance().start()
        sw.wait_for_tenant("default", 60)
        tm = sw.api("TenantManagement")
        sw.instance.system_user.run(lambda: tm.create_tenant({"token": "xr", "name": "xr",
                                                              "configurationTemplateId": "ref-default",
                                                              "datasetTemplateId": "construction"}))
        sw.wait_for_tenant("xr", 120)
        run = lambda f: sw.instance.system_user.run(f, "xr")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "xr"), sw.api("DeviceEventManagement", "xr")
        aid = run(lambda: dm.get_device_by_token("meitrack-002")).device_assignment_id
        c = MqttClient("127.0.0.1", broker.port).connect()
        end, res = time.time() + 30, []
        while not res and time.time() < end:
            c.publish("SiteWhere/xr/input/protobuf", wire.measurements("meitrack-002", {"xml.t": 7.25}), qos=1)
            time.sleep(0.5)
            res = [e for e in run(lambda: em.list_measurements_for_index("Assignment", [aid])).results
                   if e.name == "xml.t"]
        assert res and res[0].value == 7.25
        c.disconnect()
    finally:
        if sw is not None:
            sw.stop()
        for k in ids:
            TENANT_TEMPLATES.pop(k, None)
        broker.stop()
        mongo.stop()
