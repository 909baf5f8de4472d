"""Security: HS512 JWTs, authorities, authentication context, system-user execution.

Reference: ``sitewhere-microservice/.../security/TokenManagement.java:42-130`` (HS512 JWT with the
``auth`` claim; the reference hard-codes the secret "secret" -- here it is configurable and defaults
to a per-instance random secret), ``SystemUser``/``SystemUserRunnable.java``,
``GrpcUtils.handleServerMethodEntry`` (claims -> SecurityContext; the reference caches claims in a
static non-thread-safe HashMap -- here the context is a :mod:`contextvars` variable, no shared cache),
``sitewhere-core-api/.../spi/user/SiteWhereAuthority`` (granted authority names).
"""
from __future__ import annotations

import base64
import contextvars
import hashlib
import hmac
import json
import os
import secrets
import time
from dataclasses import dataclass, field

from .errors import UnauthorizedException


class SiteWhereAuthority:
    """Authority names used across the REST and RPC APIs."""
    AdminServer = "ADMINISTER_SERVER"
    AdminTenants = "ADMINISTER_TENANTS"
    AdminOwnTenant = "ADMINISTER_TENANT_SELF"
    AdminUsers = "ADMINISTER_USERS"
    AdminOwnUser = "ADMINISTER_USER_SELF"
    AdminSchedules = "ADMINISTER_SCHEDULES"
    REST = "REST"
    ViewServerInfo = "VIEW_SERVER_INFO"

    @classmethod
    def all(cls):
        return [cls.AdminServer, cls.AdminTenants, cls.AdminOwnTenant, cls.AdminUsers, cls.AdminOwnUser,
                cls.AdminSchedules, cls.REST, cls.ViewServerInfo]


def _b64e(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _b64d(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


class TokenManagement:
    """Issue and validate HS512 JWTs carrying the username and granted authorities."""

    def __init__(self, secret: str | bytes | None = None, expiration_minutes: int = 60, issuer: str = "sitewhere"):
        if secret is None:
            secret = os.environ.get("SITEWHERE_JWT_SECRET") or secrets.token_hex(32)
        self.secret = secret.encode() if isinstance(secret, str) else secret
        self.expiration_minutes = expiration_minutes
        self.issuer = issuer

    def generate_token(self, username: str, authorities: list[str], expiration_minutes: int | None = None,
                       tenant: str | None = None) -> str:
        now = int(time.time())
        exp = now + 60 * (self.expiration_minutes if expiration_minutes is None else expiration_minutes)
        payload = {"sub": username, "iss": self.issuer, "iat": now, "exp": exp, "auth": list(authorities)}
        if tenant:
            payload["tenant"] = tenant
        header = {"alg": "HS512", "typ": "JWT"}
        h = _b64e(json.dumps(header, separators=(",", ":")).encode())
        p = _b64e(json.dumps(payload, separators=(",", ":")).encode())
        sig = hmac.new(self.secret, f"{h}.{p}".encode(), hashlib.sha512).digest()
        return f"{h}.{p}.{_b64e(sig)}"

    _CACHE_MAX = 4096

    def get_claims(self, token: str) -> dict:
        """Verified claims of ``token``.  Signature checks are memoised per token (a bounded map
        replaced wholesale when full; reads and writes are single dict operations, so concurrent
        RPC threads cannot corrupt it -- unlike the reference's static HashMap);
        expiry is checked on every call."""
        cache = self.__dict__.setdefault("_verified", {})
        claims = cache.get(token)
        if claims is None:
            claims = self._verify(token)
            if len(cache) >= self._CACHE_MAX:
                self._verified = cache = {}
            cache[token] = claims
        if claims.get("exp", 0) < time.time():
            raise UnauthorizedException("JWT expired")
        return dict(claims)

    def _verify(self, token: str) -> dict:
        try:
            h, p, s = token.split(".")
        except ValueError as e:
            raise UnauthorizedException("Malformed JWT") from e
        header = json.loads(_b64d(h))
        if header.get("alg") != "HS512":
            raise UnauthorizedException("Unsupported JWT algorithm")
        want = hmac.new(self.secret, f"{h}.{p}".encode(), hashlib.sha512).digest()
        if not hmac.compare_digest(want, _b64d(s)):
            raise UnauthorizedException("Invalid JWT signature")
        return json.loads(_b64d(p))

    def get_username(self, token: str) -> str:
        return self.get_claims(token)["sub"]

    def get_granted_authorities(self, token: str) -> list[str]:
        return list(self.get_claims(token).get("auth", []))


@dataclass
class Authentication:
    username: str
    authorities: list[str] = field(default_factory=list)
    jwt: str | None = None
    tenant: str | None = None        # tenant token selected for this call

    def has(self, authority: str) -> bool:
        return authority in self.authorities or SiteWhereAuthority.AdminServer in self.authorities


_auth: contextvars.ContextVar[Authentication | None] = contextvars.ContextVar("sw_auth", default=None)


def current_authentication() -> Authentication | None:
    return _auth.get()


def current_tenant() -> str | None:
    a = _auth.get()
    return a.tenant if a else None


class security_context:
    """``with security_context(auth): ...`` -- scoped, restored on exit (unlike the reference's
    unrestored thread-local in MultitenantApiDemux)."""

    def __init__(self, auth: Authentication | None):
        self.auth = auth
        self._tok = None

    def __enter__(self):
        self._tok = _auth.set(self.auth)
        return self.auth

    def __exit__(self, *a):
        _auth.reset(self._tok)
        return False


def require_authority(authority: str):
    a = _auth.get()
    if a is None or not a.has(authority):
        raise UnauthorizedException(f"Missing authority {authority}")


class SystemUser:
    """Tenant-scoped superuser used by background work (reference SystemUser)."""

    def __init__(self, tokens: TokenManagement, username: str = "system"):
        self.tokens = tokens
        self.username = username

    def authentication(self, tenant: str | None = None) -> Authentication:
        auths = SiteWhereAuthority.all()
        return Authentication(self.username, auths, self.tokens.generate_token(self.username, auths), tenant)

    def run(self, fn, tenant: str | None = None, *args, **kw):
        """SystemUserRunnable / SystemUserCallable equivalent."""
        with security_context(self.authentication(tenant)):
            return fn(*args, **kw)


def hash_password(password: str, salt: bytes | None = None) -> str:
    salt = salt or os.urandom(16)
    dk = hashlib.pbkdf2_hmac("sha256", password.encode(), salt, 100_000)
    return f"pbkdf2${salt.hex()}${dk.hex()}"


def verify_password(password: str, hashed: str) -> bool:
    try:
        _, salt, dk = hashed.split("$")
    except ValueError:
        return False
    cand = hashlib.pbkdf2_hmac("sha256", password.encode(), bytes.fromhex(salt), 100_000)
    return hmac.compare_digest(cand.hex(), dk)
