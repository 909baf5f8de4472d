"""Configuration models (``sitewhere_amd/configuration``): role / element trees per microservice
that describe and validate the JSON configuration documents.

Reference: ``sitewhere-configuration/.../ConfigurationModelProvider.java`` and each service's
``*ModelProvider`` / ``*Roles`` (e.g. ``EventSourcesModelProvider.java``: one element per receiver
protocol and decoder, ``EventSourcesRoles.java``: source -> decoder / deduplicator roles)."""
from __future__ import annotations

import os
from types import SimpleNamespace

import pytest

from sitewhere_amd.configuration import MODELS, model_for
from sitewhere_amd.core.errors import SiteWhereException
from sitewhere_amd.services.tenant_management import TENANT_TEMPLATES

REF = "/root/reference/service-tenant-management/dockerimage/templates"


def test_models_have_reference_shape():
    assert len(MODELS) == 19
    for ident, m in MODELS.items():
        d = m.to_dict()
        assert d["rootRoleId"] in d["rolesById"] and d["elementsByRole"][d["rootRoleId"]]
        for role, els in d["elementsByRole"].items():
            assert role in d["rolesById"]
            for e in els:
                assert {a["group"] for a in e["attributes"]} <= {g["id"] for g in e["attributeGroups"]}
    es = MODELS["event-sources"]
    receivers = {v for e in es.elements_for("event-receiver") for v in e.type_value}
    assert {"mqtt", "socket", "websocket", "coap", "rest-poll", "activemq-broker", "activemq", "rabbitmq", "kafka",
            "eventhub"} <= receivers
    decoders = {v for e in es.elements_for("event-decoder") for v in e.type_value}
    assert {"protobuf", "json", "json-batch", "script", "composite", "json-string", "echo", "coap-json"} <= decoders
    connectors = {v for e in MODELS["outbound-connectors"].elements_for("outbound-connector") for v in e.type_value}
    assert len(connectors) == 12
    mqtt = next(e for e in es.elements_for("event-receiver") if "mqtt" in e.type_value)
    assert {"conn", "auth", "perf"} <= {a.group for a in mqtt.attrs}


def test_every_template_validates():
    for tpl in TENANT_TEMPLATES.values():
        for svc, doc in tpl["services"].items():
            assert model_for(svc).validate(doc) == [], (svc, doc)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference templates not present")
def test_imported_reference_templates_validate():
    from sitewhere_amd.runtime.xml_import import import_tenant_template
    for name in sorted(os.listdir(REF)):
        t = import_tenant_template(os.path.join(REF, name))
        for svc, doc in t["services"].items():
            assert model_for(svc).validate(doc) == [], (name, svc)


def test_validation_reports_paths():
    es = model_for("event-sources")
    errs = es.validate({"sources": [
        {"id": "a", "decoder": "protobuf", "receivers": [{"type": "mqtt", "port": "x1883", "topic": "t"}]},
        {"id": "a", "decoder": {"type": "nope"}},
        {"decoder": "json", "receivers": [{"type": "carrier-pigeon"}], "bogus": 1},
        {"id": "c", "decoder": {"type": "composite", "default": "json", "tokenField": 7}}],
        "rawBatchSize": "many"})
    text = "\n".join(errs)
    assert "$.sources[0].receivers[0]: port must be Integer" in text
    assert "$.sources[1]: duplicate id 'a'" in text
    assert "$.sources[1].decoder: Event Decoder type 'nope'" in text
    assert "$.sources[2]: missing required attribute id" in text
    assert "$.sources[2].receivers[0]: Event Receiver type 'carrier-pigeon'" in text
    assert "$.sources[2]: unknown attribute 'bogus'" in text
    assert "$.sources[3].decoder: tokenField must be String" in text
    assert "$: rawBatchSize must be Integer" in text
    assert "missing required Event Decoder" not in text
    assert model_for("event-sources").validate({"sources": [{"id": "x"}]}) == [
        "$.sources[0]: missing required Event Decoder (decoder)"]
    cd = model_for("command-delivery")
    assert cd.validate({"destinations": [{"id": "d", "provider": "mqtt", "encoder": "xml"}]}) == [
        "$.destinations[0]: encoder='xml' is not one of ['json', 'protobuf', 'script']"]
    assert cd.validate({"destinations": [{"id": "d", "provider": "pager"}]})[0].startswith(
        "$.destinations[0]: Command Destination provider 'pager'")
    rp = model_for("rule-processing")
    assert rp.validate({"processors": [{"id": "t", "type": "threshold", "rules": [{"min": 1}]}]}) == [
        "$.processors[0].rules[0]: missing required attribute measurement"]


def test_management_rejects_invalid_tenant_configuration():
    from sitewhere_amd.runtime.microservice import MicroserviceManagementApi
    put = {}
    ms = SimpleNamespace(identifier="outbound-connectors", multitenant=True,
                         configuration_model=lambda: model_for("outbound-connectors"),
                         tenant_config_path=lambda t: f"/t/{t}", instance=SimpleNamespace(
                             coord=SimpleNamespace(put=lambda p, d: put.__setitem__(p, d))))
    api = MicroserviceManagementApi(ms)
    with pytest.raises(SiteWhereException, match="url"):
        api.update_tenant_configuration("t1", {"connectors": [{"id": "h", "type": "http"}]})
    assert not put
    api.update_tenant_configuration("t1", {"connectors": [{"id": "h", "type": "http", "url": "http://x"}]})
    assert "/t/t1" in put
