"""RPC plane: gRPC (HTTP/2) server and channels with JWT, tenant and tracing metadata.

Reference: ``sitewhere-microservice/.../grpc/GrpcServer.java:57-117`` and
``MultitenantGrpcServer.java:35-45`` (JWT interceptor + tenant interceptor), the client side
``sitewhere-grpc-client/.../GrpcChannel.java:58-82`` with ``JwtClientInterceptor`` /
``TenantTokenClientInterceptor.java:42-58``, and ``ServerTracingInterceptor`` /
``ClientTracingInterceptor`` (never enabled in the reference; always on here).

Two planes on one server.  The reference services' RPCs are served on their own wire schemas:
``/com.sitewhere.grpc.service.<Service>/<Rpc>`` with the ``G*`` protobuf messages (:mod:`.protoplane`),
so reference clients and services interoperate.  Every public method of every service (the
reference RPCs and this framework's additions) is also served as ``/sitewhere.<Service>/<CamelName>``
(e.g. ``create_device_type`` -> ``CreateDeviceType``) with the JSON model codec of :mod:`.codec`,
the internal plane between this framework's processes.  :class:`LocalChannel` short-circuits the
network when caller and service share a process (same headers, same security semantics).
"""
from __future__ import annotations

import json
import re
import socket
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Callable

import grpc

from ..core.errors import (ErrorCode, ErrorLevel, NotFoundException, SiteWhereException, SiteWhereSystemException,
                           TenantEngineNotAvailableException, UnauthorizedException)
from ..core.lifecycle import LifecycleComponent, LifecycleComponentType
from ..core.security import Authentication, TokenManagement, current_authentication, security_context
from ..core.tracing import HEADER as TRACE_HEADER, global_tracer
from . import codec

JWT_HEADER = "authorization"
TENANT_HEADER = "tenant"


def camel_method(name: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in name.split("_"))


def snake_method(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


def public_methods(obj) -> dict[str, Callable]:
    out = {}
    for n in dir(obj):
        if n.startswith("_"):
            continue
        f = getattr(obj, n, None)
        if callable(f) and not isinstance(f, type):
            out[camel_method(n)] = f
    return out


_STATUS = {404: grpc.StatusCode.NOT_FOUND, 401: grpc.StatusCode.UNAUTHENTICATED, 403: grpc.StatusCode.PERMISSION_DENIED,
           503: grpc.StatusCode.UNAVAILABLE, 400: grpc.StatusCode.INVALID_ARGUMENT}


def _error_payload(e: BaseException) -> str:
    if isinstance(e, SiteWhereSystemException):
        return json.dumps({"code": e.code.name, "level": e.level.value, "message": str(e), "http": e.http_status})
    return json.dumps({"code": "Error", "level": "ERROR", "message": str(e), "http": 500})


def _raise_from_payload(s: str):
    try:
        d = json.loads(s)
    except Exception:
        raise SiteWhereException(s)
    code = ErrorCode[d.get("code", "Error")] if d.get("code") in ErrorCode.__members__ else ErrorCode.Error
    http = d.get("http", 500)
    if http == 404:
        raise NotFoundException(code, d.get("message"))
    if http == 401:
        raise UnauthorizedException(d.get("message"))
    if http == 503:
        raise TenantEngineNotAvailableException(d.get("message"))
    if http == 500 and code == ErrorCode.Error:
        raise SiteWhereException(d.get("message"))
    raise SiteWhereSystemException(code, ErrorLevel(d.get("level", "ERROR")), d.get("message"), http)


class ServiceResolver:
    """Maps (service name, tenant) to the object that implements it.

    Global services register one implementation; multitenant services register a callable that
    returns the tenant engine's implementation (the reference's ``*Router`` classes).
    """

    def __init__(self):
        self._global: dict[str, object] = {}
        self._tenant: dict[str, Callable[[str], object]] = {}

    def add_global(self, name: str, impl):
        self._global[name] = impl

    def add_tenant(self, name: str, resolve: Callable[[str], object]):
        self._tenant[name] = resolve

    def resolve(self, name: str, tenant: str | None):
        if name in self._global:
            return self._global[name]
        if name in self._tenant:
            if not tenant:
                raise SiteWhereSystemException(ErrorCode.InvalidTenantToken, detail="tenant header required")
            return self._tenant[name](tenant)
        raise NotFoundException(ErrorCode.Error, f"unknown service {name}")

    def names(self) -> list[str]:
        return sorted(set(self._global) | set(self._tenant))


_IMMUTABLE = (bytes, str, int, float, bool, type(None))


def _trim_optional_tail(fn, args: list) -> list:
    """Drop trailing ``None`` arguments the method has defaults for (unset proto3 fields)."""
    import inspect
    try:
        params = [p for p in inspect.signature(fn).parameters.values()
                  if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
    except (TypeError, ValueError):
        return args
    required = sum(1 for p in params if p.default is p.empty)
    args = list(args[:len(params)]) if not any(p.kind == p.VAR_POSITIONAL for p in
                                                inspect.signature(fn).parameters.values()) else list(args)
    while len(args) > required and args[-1] is None:
        args.pop()
    return args


def invoke(resolver: ServiceResolver, tokens: TokenManagement, service: str, method: str, body: bytes | None,
           jwt: str | None, tenant: str | None, trace: str | None, require_jwt: bool = True, direct=None,
           trim: bool = False):
    """Common server-side dispatch (network and local): auth -> tenant -> span -> call.

    ``direct=(args, kwargs)`` skips the body codec (in-process calls whose arguments are all
    immutable scalars / bytes -- e.g. columnar batch payloads -- need no isolation copy)."""
    if jwt is None:
        if require_jwt:
            raise UnauthorizedException("No JWT in request metadata")
        auth = None
    else:
        if jwt.lower().startswith("bearer "):
            jwt = jwt[7:]
        claims = tokens.get_claims(jwt)
        auth = Authentication(claims["sub"], list(claims.get("auth", [])), jwt, tenant)
    tracer = global_tracer()
    with security_context(auth):
        with tracer.start_span(f"{service}.{method}", child_of=trace) as span:
            span.set_tag("tenant", tenant or "")
            impl = resolver.resolve(service, tenant)
            fn = getattr(impl, snake_method(method), None)
            if fn is None or not callable(fn) or isinstance(fn, type) or snake_method(method).startswith("_"):
                raise NotFoundException(ErrorCode.Error, f"{service} has no method {method}")
            if direct is not None:
                args = _trim_optional_tail(fn, direct[0]) if trim else direct[0]
                return fn(*args, **direct[1])
            req = codec.loads(body) or {}
            return fn(*req.get("args", []), **req.get("kwargs", {}))


class RpcServer(LifecycleComponent):
    """gRPC server exposing every registered service (one port per process, like the reference's
    API port 9000 / management port 9001)."""

    component_type = LifecycleComponentType.Other

    def __init__(self, resolver: ServiceResolver, tokens: TokenManagement, port: int = 0, host: str = "127.0.0.1",
                 workers: int = 16, advertise_host: str = "", identifier: str | None = None):
        super().__init__("rpc-server")
        self.resolver, self.tokens = resolver, tokens
        self.identifier = identifier          # the microservice serving (its MicroserviceManagement)
        self.host, self.port, self.workers = host, port, workers
        self.advertise_host = advertise_host or (socket.gethostname() if host in ("0.0.0.0", "::") else host)
        self._server = None
        self.calls = 0

    def _handler(self, service: str, method: str):
        def handle(request: bytes, context: grpc.ServicerContext):
            md = dict(context.invocation_metadata())
            self.calls += 1
            try:
                out = invoke(self.resolver, self.tokens, service, method, request, md.get(JWT_HEADER),
                             md.get(TENANT_HEADER), md.get(TRACE_HEADER))
                return codec.dumps(out)
            except SiteWhereSystemException as e:
                context.abort(_STATUS.get(e.http_status, grpc.StatusCode.INVALID_ARGUMENT), _error_payload(e))
            except SiteWhereException as e:
                context.abort(grpc.StatusCode.INTERNAL, _error_payload(e))
            except Exception as e:  # noqa: BLE001
                context.abort(grpc.StatusCode.INTERNAL, _error_payload(e))
        return grpc.unary_unary_rpc_method_handler(handle, request_deserializer=None, response_serializer=None)

    def _proto_handler(self, service: str, rpc: str):
        """Handler of a reference RPC on its protobuf schema (see :mod:`.protoplane`)."""
        from . import protoplane as pp
        md = pp.method(service, rpc)
        if md is None:
            return None
        req_cls, resp_cls = pp.message_class(md.input_type.full_name), pp.message_class(md.output_type.full_name)
        ours = pp.SERVICE_ALIASES.get(service, service)
        if ours == "MicroserviceManagement" and self.identifier:
            ours = f"MicroserviceManagement.{self.identifier}"
        fields = list(md.input_type.fields)

        def handle(request, context: grpc.ServicerContext):
            meta = dict(context.invocation_metadata())
            self.calls += 1
            try:
                args = [pp.arg_of(request, f) for f in fields]
                out = invoke(self.resolver, self.tokens, ours, rpc, None, meta.get(JWT_HEADER), meta.get(TENANT_HEADER),
                             meta.get(TRACE_HEADER), direct=(args, {}), trim=True)
                return pp.set_response(resp_cls(), out)
            except SiteWhereSystemException as e:
                context.abort(_STATUS.get(e.http_status, grpc.StatusCode.INVALID_ARGUMENT), _error_payload(e))
            except SiteWhereException as e:
                context.abort(grpc.StatusCode.INTERNAL, _error_payload(e))
            except (TypeError, ValueError, KeyError) as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, _error_payload(e))
            except Exception as e:  # noqa: BLE001
                context.abort(grpc.StatusCode.INTERNAL, _error_payload(e))
        return grpc.unary_unary_rpc_method_handler(handle, request_deserializer=req_cls.FromString,
                                                   response_serializer=resp_cls.SerializeToString)

    def start(self, monitor):
        srv = self

        class _Generic(grpc.GenericRpcHandler):
            def service(self, details):
                path = details.method  # /sitewhere.<Service>/<Method>
                try:
                    svc, meth = path.lstrip("/").split("/", 1)
                except ValueError:
                    return None
                if svc.startswith("com.sitewhere.grpc.service."):
                    return srv._proto_handler(svc[len("com.sitewhere.grpc.service."):], meth)
                if not svc.startswith("sitewhere."):
                    return None
                return srv._handler(svc[len("sitewhere."):], meth)

        self._server = grpc.server(ThreadPoolExecutor(max_workers=self.workers, thread_name_prefix="grpc"))
        self._server.add_generic_rpc_handlers((_Generic(),))
        self.port = self._server.add_insecure_port(f"{self.host}:{self.port}")
        self._server.start()

    def stop(self, monitor):
        if self._server is not None:
            self._server.stop(grace=0.5)
            self._server = None

    @property
    def address(self) -> str:
        """Where other processes dial this server (advertised in the topology)."""
        return f"{self.advertise_host}:{self.port}"


class ApiChannel:
    """Client channel interface (``call``) + dynamic proxies per service."""

    def call(self, service: str, method: str, *args, tenant: str | None = None, timeout: float = 30.0, **kwargs):
        raise NotImplementedError

    def proxy(self, service: str, tenant: str | None = None) -> "ServiceProxy":
        return ServiceProxy(self, service, tenant)

    def close(self):
        pass


class ServiceProxy:
    def __init__(self, channel: ApiChannel, service: str, tenant: str | None):
        self._ch, self._svc, self._tenant = channel, service, tenant

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)

        def call(*args, **kwargs):
            return self._ch.call(self._svc, camel_method(name), *args, tenant=self._tenant, **kwargs)
        return call


def _jwt_for_call(tokens: TokenManagement | None, system_jwt: str | None) -> str | None:
    a = current_authentication()
    if a is not None and a.jwt:
        return a.jwt
    return system_jwt


def _tenant_for_call(explicit: str | None) -> str | None:
    if explicit:
        return explicit
    a = current_authentication()
    return a.tenant if a else None


class GrpcChannel(ApiChannel):
    def __init__(self, address: str, system_jwt: str | None = None):
        self.address = address
        self.system_jwt = system_jwt
        self._ch = grpc.insecure_channel(address)
        self._stubs: dict[str, Callable] = {}
        self._lock = threading.Lock()

    def _stub(self, path: str):
        with self._lock:
            s = self._stubs.get(path)
            if s is None:
                s = self._ch.unary_unary(path, request_serializer=None, response_deserializer=None)
                self._stubs[path] = s
            return s

    def call(self, service, method, *args, tenant=None, timeout=30.0, **kwargs):
        md = []
        jwt = _jwt_for_call(None, self.system_jwt)
        if jwt:
            md.append((JWT_HEADER, f"Bearer {jwt}"))
        t = _tenant_for_call(tenant)
        if t:
            md.append((TENANT_HEADER, t))
        span = global_tracer().active()
        if span is not None:
            md.append((TRACE_HEADER, span.context_header()))
        body = codec.dumps({"args": list(args), "kwargs": kwargs})
        try:
            out = self._stub(f"/sitewhere.{service}/{camel_method(method) if '_' in method else method}")(
                body, metadata=md, timeout=timeout)
        except grpc.RpcError as e:
            if e.code() == grpc.StatusCode.UNAVAILABLE and not e.details().startswith("{"):
                raise TenantEngineNotAvailableException(f"{self.address}: {e.details()}") from None
            _raise_from_payload(e.details())
        return codec.loads(out)

    def ready(self, timeout: float = 1.0) -> bool:
        try:
            grpc.channel_ready_future(self._ch).result(timeout=timeout)
            return True
        except grpc.FutureTimeoutError:
            return False

    def close(self):
        self._ch.close()


class LocalChannel(ApiChannel):
    """In-process channel with the server-side semantics (auth, tenant, spans) and isolated values.

    ``mode="clone"`` (default) copies non-scalar arguments and results structurally
    (:func:`codec.clone`, same result as a wire round trip, ~10x cheaper); ``mode="codec"`` sends
    them through the JSON wire codec exactly as a network call would (``SITEWHERE_LOCAL_RPC=codec``
    -- useful to shake out values that would not survive the wire)."""

    def __init__(self, resolver: ServiceResolver, tokens: TokenManagement, system_jwt: str | None = None,
                 serialize: bool = True, mode: str = "clone"):
        self.resolver, self.tokens, self.system_jwt = resolver, tokens, system_jwt
        self.serialize = serialize
        if mode not in ("clone", "codec"):
            raise ValueError(f"local rpc mode {mode!r}")
        self.mode = mode

    def call(self, service, method, *args, tenant=None, timeout=30.0, **kwargs):
        jwt = _jwt_for_call(self.tokens, self.system_jwt)
        t = _tenant_for_call(tenant)
        span = global_tracer().active()
        m = camel_method(method) if "_" in method else method
        trace = span.context_header() if span else None
        if all(isinstance(x, _IMMUTABLE) for x in args) and all(isinstance(x, _IMMUTABLE) for x in kwargs.values()):
            out = invoke(self.resolver, self.tokens, service, m, None, jwt, t, trace, direct=(args, kwargs))
        elif self.mode == "clone":
            out = invoke(self.resolver, self.tokens, service, m, None, jwt, t, trace,
                         direct=(codec.clone(list(args)), codec.clone(kwargs)))
        else:
            out = invoke(self.resolver, self.tokens, service, m, codec.dumps({"args": list(args), "kwargs": kwargs}),
                         jwt, t, trace)
        if not self.serialize or isinstance(out, _IMMUTABLE):
            return out
        return codec.clone(out) if self.mode == "clone" else codec.loads(codec.dumps(out))
