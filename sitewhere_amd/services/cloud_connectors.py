"""Cloud outbound connectors speaking the services' HTTP APIs directly (no vendor SDKs in this image).

Reference connectors (``service-outbound-connectors/.../connectors/``): ``SqsOutboundConnector``
(188 LoC, AWS SDK ``sendMessage``), ``EventHubOutboundConnector`` (247, Azure AMQP client),
``DweetIoConnector`` (HTTP POST per event), ``InitialStateEventProcessor`` (HTTP events API).
Here:
  * SQS -- ``SendMessageBatch`` (query API, 10 entries per call) signed with AWS Signature V4
  * Event Hubs -- REST ``POST https://<ns>.servicebus.windows.net/<hub>/messages`` with a
    SharedAccessSignature token (batched JSON array, ``application/vnd.microsoft.servicebus.json``)
  * dweet.io -- ``POST /dweet/for/<thing>`` per event, thing name templated by device token
  * Initial State -- ``POST /api/events`` with access/bucket key headers, one key/value per metric
The endpoint URL is configurable (tests point it at a local HTTP server).  ``post`` may be injected.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import json
import time
import urllib.parse
import urllib.request

from ..models.domain import DeviceEventType
from .outbound_connectors import OutboundConnector, event_json


def _http(method: str, url: str, body: bytes, headers: dict, timeout: float = 10.0):
    req = urllib.request.Request(url, data=body, method=method, headers=headers)
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status, r.read()


class _HttpOut(OutboundConnector):
    def __init__(self, cid, filters=None, post=None):
        super().__init__(cid, filters)
        self._post = post or (lambda url, body, headers: _http("POST", url, body, headers))
        self.requests = 0

    def post(self, url, body: bytes, headers: dict):
        self.requests += 1
        return self._post(url, body, headers)


# ---------------------------------------------------------------------------------------- SQS
def sigv4_headers(method: str, url: str, body: bytes, region: str, service: str, access_key: str, secret_key: str,
                  now: _dt.datetime | None = None, extra: dict | None = None) -> dict:
    """AWS Signature Version 4 for a request with a body (header-based signing)."""
    now = now or _dt.datetime.now(_dt.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    date = now.strftime("%Y%m%d")
    u = urllib.parse.urlsplit(url)
    host = u.netloc
    payload_hash = hashlib.sha256(body).hexdigest()
    headers = {"host": host, "x-amz-date": amz_date, "x-amz-content-sha256": payload_hash}
    headers.update({k.lower(): v for k, v in (extra or {}).items()})
    signed = ";".join(sorted(headers))
    canon_headers = "".join(f"{k}:{str(headers[k]).strip()}\n" for k in sorted(headers))
    canon_query = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                           for k, v in sorted(urllib.parse.parse_qsl(u.query, keep_blank_values=True)))
    canon = "\n".join([method, u.path or "/", canon_query, canon_headers, signed, payload_hash])
    scope = f"{date}/{region}/{service}/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canon.encode()).hexdigest()])

    def _h(k, m):
        return hmac.new(k, m.encode(), hashlib.sha256).digest()
    k = _h(_h(_h(_h(("AWS4" + secret_key).encode(), date), region), service), "aws4_request")
    sig = hmac.new(k, to_sign.encode(), hashlib.sha256).hexdigest()
    out = {k2: v for k2, v in headers.items() if k2 != "host"}
    out["Authorization"] = f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={signed}, Signature={sig}"
    return out


class SqsConnector(_HttpOut):
    def __init__(self, cid, queue_url, region, access_key, secret_key, endpoint=None, filters=None, post=None):
        super().__init__(cid, filters, post)
        self.queue_url, self.region = queue_url, region
        self.access_key, self.secret_key = access_key, secret_key
        self.endpoint = endpoint or queue_url

    def deliver(self, items):
        for i in range(0, len(items), 10):             # SendMessageBatch takes at most 10 entries
            params = {"Action": "SendMessageBatch", "QueueUrl": self.queue_url, "Version": "2012-11-05"}
            for j, (ev, ctx) in enumerate(items[i:i + 10], 1):
                params[f"SendMessageBatchRequestEntry.{j}.Id"] = f"m{j}"
                params[f"SendMessageBatchRequestEntry.{j}.MessageBody"] = json.dumps(event_json(ev, ctx))
            body = urllib.parse.urlencode(params).encode()
            h = sigv4_headers("POST", self.endpoint, body, self.region, "sqs", self.access_key, self.secret_key,
                              extra={"content-type": "application/x-www-form-urlencoded"})
            h["Content-Type"] = "application/x-www-form-urlencoded"
            self.post(self.endpoint, body, h)


# ---------------------------------------------------------------------------------- Event Hubs
def sas_token(resource_uri: str, key_name: str, key: str, ttl_s: int = 3600, now: float | None = None) -> str:
    expiry = int((now or time.time()) + ttl_s)
    res = urllib.parse.quote_plus(resource_uri)
    sig = base64.b64encode(hmac.new(key.encode(), f"{res}\n{expiry}".encode(), hashlib.sha256).digest())
    return (f"SharedAccessSignature sr={res}&sig={urllib.parse.quote_plus(sig.decode())}"
            f"&se={expiry}&skn={key_name}")


class EventHubConnector(_HttpOut):
    def __init__(self, cid, namespace, hub, key_name, key, endpoint=None, filters=None, post=None):
        super().__init__(cid, filters, post)
        self.resource = f"https://{namespace}.servicebus.windows.net/{hub}"
        self.url = (endpoint.rstrip("/") + f"/{hub}/messages") if endpoint else self.resource + "/messages"
        self.key_name, self.key = key_name, key

    def deliver(self, items):
        body = json.dumps([{"Body": json.dumps(event_json(ev, ctx)),
                            "BrokerProperties": {"PartitionKey": ctx.get("deviceToken") or ev.device_id}}
                           for ev, ctx in items]).encode()
        self.post(self.url, body, {"Authorization": sas_token(self.resource, self.key_name, self.key),
                                   "Content-Type": "application/vnd.microsoft.servicebus.json"})


# ------------------------------------------------------------------------------------ dweet.io
class DweetConnector(_HttpOut):
    def __init__(self, cid, thing="{deviceToken}", base_url="https://dweet.io", filters=None, post=None):
        super().__init__(cid, filters, post)
        self.thing, self.base = thing, base_url.rstrip("/")

    def on_event(self, ev, ctx):
        thing = self.thing.format(deviceToken=ctx.get("deviceToken") or ev.device_id, tenant=self.tenant_prefix)
        self.post(f"{self.base}/dweet/for/{urllib.parse.quote(thing)}", json.dumps(ev.to_dict()).encode(),
                  {"Content-Type": "application/json"})


# -------------------------------------------------------------------------------- Initial State
class InitialStateConnector(_HttpOut):
    def __init__(self, cid, access_key, bucket_key="{deviceToken}", base_url="https://groker.init.st",
                 filters=None, post=None):
        super().__init__(cid, filters, post)
        self.access_key, self.bucket_key, self.base = access_key, bucket_key, base_url.rstrip("/")

    @staticmethod
    def _values(ev) -> list[tuple[str, object]]:
        if ev.event_type == DeviceEventType.Measurement:
            return [(ev.name, ev.value)]
        if ev.event_type == DeviceEventType.Location:
            return [("location", f"{ev.latitude},{ev.longitude}")]
        if ev.event_type == DeviceEventType.Alert:
            return [(f"alert.{ev.type}", ev.message)]
        return []

    def deliver(self, items):
        by_bucket: dict = {}
        for ev, ctx in items:
            b = self.bucket_key.format(deviceToken=ctx.get("deviceToken") or ev.device_id)
            for k, v in self._values(ev):
                by_bucket.setdefault(b, []).append({"key": k, "value": v, "epoch": (ev.event_date or 0) / 1000.0})
        for bucket, evs in by_bucket.items():
            self.post(f"{self.base}/api/events", json.dumps(evs).encode(),
                      {"Content-Type": "application/json", "X-IS-AccessKey": self.access_key,
                       "X-IS-BucketKey": bucket, "Accept-Version": "~0"})


# ------------------------------------------------------------------------------------ RabbitMQ
class RabbitMqConnector(OutboundConnector):
    """Publish enriched events as JSON over AMQP 0-9-1 (reference RabbitMqOutboundConnector)."""

    def __init__(self, cid, host="127.0.0.1", port=5672, exchange="", routing_key="sitewhere.{tenant}.events",
                 username="guest", password="guest", vhost="/", filters=None):
        super().__init__(cid, filters)
        self.host, self.port, self.exchange, self.routing_key = host, port, exchange, routing_key
        self.username, self.password, self.vhost = username, password, vhost
        self.client = None

    def start(self, monitor):
        from ..edges.amqp import AmqpClient
        self.client = AmqpClient(self.host, self.port, self.username, self.password, self.vhost).connect()

    def stop(self, monitor):
        if self.client:
            self.client.close()

    def on_event(self, ev, ctx):
        rk = self.routing_key.format(tenant=self.tenant_prefix.rstrip("."),
                                     deviceToken=ctx.get("deviceToken") or ev.device_id)
        self.client.publish(self.exchange, rk, json.dumps(event_json(ev, ctx)).encode(), "application/json")


# ------------------------------------------------------------------------------------ Kafka
class KafkaConnector(OutboundConnector):
    """Publish enriched events as JSON to a Kafka topic keyed by device token (the reference's
    downstream integrations read the enriched stream straight off Kafka); a batch per delivery."""

    def __init__(self, cid, bootstrap="127.0.0.1:9092", topic="sitewhere.{tenant}.enriched", tls=False,
                 sasl_plain=None, filters=None):
        super().__init__(cid, filters)
        self.bootstrap, self.topic, self.tls, self.sasl_plain = bootstrap, topic, tls, sasl_plain
        self.bus = None

    def start(self, monitor):
        from ..bus.kafka_client import KafkaEventBus
        self.bus = KafkaEventBus(self.bootstrap, client_id="sitewhere-connector", tls=self.tls,
                                 sasl_plain=self.sasl_plain)
        self.producer = self.bus.producer()

    def stop(self, monitor):
        if self.bus:
            self.bus.client.close()

    def deliver(self, items):
        topic = self.topic.format(tenant=self.tenant_prefix.rstrip("."))
        self.producer.send_batch(topic, [(ctx.get("deviceToken") or ev.device_id,
                                          json.dumps(event_json(ev, ctx)).encode()) for ev, ctx in items])


def build_cloud_connector(t: str, cid: str, cfg: dict, filters):
    if t == "kafka":
        sasl = (cfg["username"], cfg["password"]) if cfg.get("username") else None
        return KafkaConnector(cid, cfg.get("bootstrap", "127.0.0.1:9092"), cfg.get("topic", "sitewhere.{tenant}.enriched"),
                              bool(cfg.get("tls", False)), sasl, filters)
    if t == "sqs":
        return SqsConnector(cid, cfg["queueUrl"], cfg.get("region", "us-east-1"), cfg["accessKey"], cfg["secretKey"],
                            cfg.get("endpoint"), filters)
    if t == "eventhub":
        return EventHubConnector(cid, cfg["namespace"], cfg["hub"], cfg["sasKeyName"], cfg["sasKey"],
                                 cfg.get("endpoint"), filters)
    if t == "dweet":
        return DweetConnector(cid, cfg.get("thing", "{deviceToken}"), cfg.get("url", "https://dweet.io"), filters)
    if t == "rabbitmq":
        return RabbitMqConnector(cid, cfg.get("host", "127.0.0.1"), int(cfg.get("port", 5672)), cfg.get("exchange", ""),
                                 cfg.get("routingKey", "sitewhere.{tenant}.events"), cfg.get("username", "guest"),
                                 cfg.get("password", "guest"), cfg.get("vhost", "/"), filters)
    if t == "initialstate":
        return InitialStateConnector(cid, cfg["accessKey"], cfg.get("bucketKey", "{deviceToken}"),
                                     cfg.get("url", "https://groker.init.st"), filters)
    return None
