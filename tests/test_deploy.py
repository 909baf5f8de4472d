"""Deployment files (deploy/): the reference ships one container image per microservice plus
orchestration; here one image runs any process role (`sitewhere_amd.serve`).  Checks that the
compose file and the node script start every one of the 19 microservices through commands the
CLI accepts, one inbound-processing replica per GPU, and that a server bound to all interfaces
advertises a dialable address."""
from __future__ import annotations

import os
import re
import socket

import yaml

from sitewhere_amd.assembly import SERVICES_BY_ID
from sitewhere_amd.serve import build_parser

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_compose_starts_every_microservice_once_with_valid_commands():
    doc = yaml.safe_load(open(os.path.join(ROOT, "deploy", "docker-compose.yml")))
    parser = build_parser()
    started, gpus = [], []
    for name, svc in doc["services"].items():
        args = parser.parse_args(svc["command"])
        if args.cmd == "service":
            started += args.identifiers
            assert args.bind == "0.0.0.0" and args.advertise == svc["hostname"] == name
            assert args.infra == "infra:9092"
            if "inbound-processing" in args.identifiers:
                gpus.append(svc["environment"]["SITEWHERE_GPU_DEVICE"])
                assert "/dev/kfd" in svc["devices"]
    assert sorted(set(started)) == sorted(SERVICES_BY_ID)
    assert [s for s in started if s != "inbound-processing"] == sorted(set(started) - {"inbound-processing"},
                                                                        key=started.index)
    assert gpus == [str(i) for i in range(len(gpus))] and len(gpus) >= 2


def test_node_script_starts_every_microservice():
    text = open(os.path.join(ROOT, "deploy", "run_node.sh")).read()
    text = text.replace("\\\n", " ")
    parser = build_parser()
    started = []
    for line in text.splitlines():
        m = re.search(r"python -m sitewhere_amd\.serve (service [^>]*)", line)
        if m:
            args = parser.parse_args(m.group(1).replace("$INFRA", "127.0.0.1:9092").split())
            started += args.identifiers
    assert sorted(set(started)) == sorted(SERVICES_BY_ID)
    assert "SITEWHERE_GPU_DEVICE=$g" in text


def test_rpc_server_bound_to_all_interfaces_advertises_host_name():
    from sitewhere_amd.rpc.transport import RpcServer
    assert RpcServer(None, None, host="0.0.0.0").address.startswith(socket.gethostname() + ":")
    assert RpcServer(None, None, host="0.0.0.0", advertise_host="inbound-gpu0").address.startswith("inbound-gpu0:")
    assert RpcServer(None, None).address.startswith("127.0.0.1:")
