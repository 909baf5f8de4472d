"""Process entry points (the reference's per-service Spring Boot ``*Application`` mains + docker-compose).

  python -m sitewhere_amd.serve infra   --port 9092 [--data DIR] [--kafka-port 9093]
      bus (Kafka role, native commit log) + coordination (ZooKeeper role) server; --kafka-port also
      serves the bus over the Kafka wire protocol (bus/kafka_broker.py) to any Kafka client
  python -m sitewhere_amd.serve service <identifier> [<identifier> ...] --infra HOST:PORT [--kafka BOOTSTRAP]
                                         [--zookeeper HOST:PORT/CHROOT] [--bind 0.0.0.0 --advertise NAME]
      one or more microservices in this process, talking to the shared infra and to other
      processes' services over gRPC (topology-discovered replicas); with --kafka the data plane is
      a Kafka cluster (bus/kafka_client.KafkaEventBus) and with --zookeeper the coordination is a
      ZooKeeper ensemble (coord/zk.py), as in the reference deployment
  python -m sitewhere_amd.serve all [--rest-port 8080] [--mqtt-port 1883] [--data DIR]
      a whole instance in one process (single-node deployment; GPU inbound engine per tenant)

Exit codes follow ``MicroserviceApplication.java:80-202``: 2 on initialize/start failure.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading


def _wait_forever(stop: threading.Event):
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            signal.signal(sig, lambda *_: stop.set())
        except ValueError:
            pass
    while not stop.wait(0.5):
        pass


def cmd_infra(args) -> int:
    from .bus.log import EventBus
    from .coord.store import Coordination
    from .rpc.infra import InfraServer
    bus_dir = os.path.join(args.data, "bus") if args.data else None
    snap = os.path.join(args.data, "coordination.json") if args.data else None
    if args.data:
        os.makedirs(bus_dir, exist_ok=True)
    bus = EventBus(bus_dir, default_partitions=args.partitions)
    srv = InfraServer(bus, Coordination(snap), port=args.port, host=args.host).start()
    print(f"infra listening on {srv.address}", flush=True)
    kafka = None
    if args.kafka_port is not None:
        from .bus.kafka_broker import KafkaBrokerServer
        kafka = KafkaBrokerServer(bus, host=args.host, port=args.kafka_port).start()
        print(f"kafka protocol listening on {kafka.address}", flush=True)
    stop = threading.Event()
    _wait_forever(stop)
    if kafka:
        kafka.stop()
    srv.stop()
    return 0


def build_instance(args, network: bool):
    from .rpc.infra import RemoteCoordination, RemoteEventBus
    from .runtime.config import InstanceSettings
    from .runtime.microservice import Instance
    settings = InstanceSettings.from_env(heartbeat_s=args.heartbeat, grpc_port=getattr(args, "grpc_port", 0))
    if getattr(args, "bind", None):
        settings.grpc_host = args.bind
    if getattr(args, "advertise", None):
        settings.grpc_advertise_host = args.advertise
    kw = {}
    if getattr(args, "infra", None):
        kw["bus"] = RemoteEventBus(args.infra)
        kw["coord"] = RemoteCoordination(args.infra)
    kafka = getattr(args, "kafka", None) or os.environ.get("SITEWHERE_KAFKA_BOOTSTRAP")
    if kafka:
        from .bus.kafka_client import KafkaEventBus
        kw["bus"] = KafkaEventBus(kafka)
    zk = getattr(args, "zookeeper", None) or os.environ.get("SITEWHERE_ZOOKEEPER")
    if zk:
        from .coord.zk import ZooKeeperCoordination
        kw["coord"] = ZooKeeperCoordination(zk if "/" in zk else zk + "/sitewhere")
    secret = os.environ.get("SITEWHERE_JWT_SECRET") or args.jwt_secret
    return Instance(settings, jwt_secret=secret, network_rpc=network, **kw)


def cmd_service(args) -> int:
    from .assembly import SERVICES_BY_ID
    from .runtime.microservice import run_microservice, shutdown_microservice
    inst = build_instance(args, network=True)
    services = []
    for ident in args.identifiers:
        cls = SERVICES_BY_ID.get(ident)
        if cls is None:
            print(f"unknown microservice {ident}; choose from {sorted(SERVICES_BY_ID)}", file=sys.stderr)
            return 2
        kw = {"port": args.rest_port, "host": args.bind or "127.0.0.1"} if ident == "web-rest" else {}
        ms = cls(inst, **kw)
        if run_microservice(ms) != 0:
            print(f"{ident} failed: {ms.lifecycle_error}", file=sys.stderr)
            return 2
        services.append(ms)
        print(f"{ident} started (api {ms.api_address})", flush=True)
    stop = threading.Event()
    _wait_forever(stop)
    for ms in reversed(services):
        shutdown_microservice(ms)
    return 0


def cmd_all(args) -> int:
    from .assembly import SiteWhereInstance
    inst = build_instance(args, network=False)
    if args.data:
        pass
    sw = SiteWhereInstance(instance=inst, rest_port=args.rest_port)
    sw.start()
    broker = None
    if args.mqtt_port:
        from .edges.mqtt import MqttBroker
        broker = MqttBroker(port=args.mqtt_port)
        broker.start()
    print(f"SiteWhere instance up: REST http://127.0.0.1:{args.rest_port}/sitewhere/api"
          + (f", MQTT 127.0.0.1:{args.mqtt_port}" if broker else ""), flush=True)
    stop = threading.Event()
    _wait_forever(stop)
    sw.stop()
    if broker:
        broker.stop()
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="sitewhere_amd.serve")
    ap.add_argument("--log-level", default="INFO")
    ap.add_argument("--heartbeat", type=float, default=5.0)
    ap.add_argument("--jwt-secret", default=None,
                    help="HS512 signing secret (or SITEWHERE_JWT_SECRET); default: a random secret created "
                         "once per instance and shared through the coordination store")
    ap.add_argument("--reference-templates", default=None,
                    help="a SiteWhere 2.x templates directory: its Spring XML tenant templates become ref-<name>")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("infra")
    p.add_argument("--port", type=int, default=9092)
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--data", default=None)
    p.add_argument("--partitions", type=int, default=8)
    p.add_argument("--kafka-port", type=int, default=None, help="also serve the bus over the Kafka protocol")
    p = sub.add_parser("service")
    p.add_argument("identifiers", nargs="+")
    p.add_argument("--infra", required=True)
    p.add_argument("--kafka", default=None, help="Kafka bootstrap servers for the data plane")
    p.add_argument("--zookeeper", default=None, help="ZooKeeper connect string (host:port[,..][/chroot])")
    p.add_argument("--grpc-port", type=int, default=0)
    p.add_argument("--rest-port", type=int, default=0)
    p.add_argument("--bind", default=None,
                   help="bind address of this process's gRPC and REST servers (0.0.0.0 in a container; "
                        "env SITEWHERE_GRPC_HOST); default 127.0.0.1")
    p.add_argument("--advertise", default=None,
                   help="host other processes dial for this process's gRPC services (env "
                        "SITEWHERE_GRPC_ADVERTISE_HOST); default: the bind address, or the host name for 0.0.0.0")
    p = sub.add_parser("all")
    p.add_argument("--rest-port", type=int, default=8080)
    p.add_argument("--mqtt-port", type=int, default=0)
    p.add_argument("--data", default=None)
    return ap


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    if args.reference_templates:                 # read by tenant management when it starts
        os.environ["SITEWHERE_REFERENCE_TEMPLATES"] = args.reference_templates
    from .utils.stack_sampler import maybe_start
    maybe_start()                                # SW_STACK_SAMPLE=<prefix>: where this process's time goes
    return {"infra": cmd_infra, "service": cmd_service, "all": cmd_all}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
