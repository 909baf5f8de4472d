"""service-user-management: users and granted authorities (global microservice).

Reference: ``service-user-management`` -- ``UserManagementImpl`` over ``MongoUserManagement``;
RPC surface ``sitewhere-grpc-user-management/src/main/proto/user-management.proto`` (15 RPCs:
CreateUser, ImportUser, Authenticate, UpdateUser, GetUserByUsername, ListUsers, DeleteUser,
CreateGrantedAuthority, GetGrantedAuthorityByName, UpdateGrantedAuthority, ListGrantedAuthorities,
DeleteGrantedAuthority, GetGrantedAuthoritiesForUser, AddGrantedAuthoritiesForUser,
RemoveGrantedAuthoritiesForUser).
"""
from __future__ import annotations

from ..core.errors import ErrorCode, NotFoundException, SiteWhereSystemException, UnauthorizedException
from ..core.security import SiteWhereAuthority, hash_password, verify_password
from ..models.domain import (AccountStatus, GrantedAuthority, SearchCriteria, SearchResults, User, now_ms,
                             stamp_created, stamp_updated)
from ..persistence.store import EntityStore, create_store
from ..runtime.microservice import GlobalMicroservice

AUTHORITY_DESCRIPTIONS = {
    SiteWhereAuthority.AdminServer: ("Administer server", None, False),
    SiteWhereAuthority.AdminTenants: ("Administer all tenants", None, False),
    SiteWhereAuthority.AdminOwnTenant: ("Administer own tenant", None, False),
    SiteWhereAuthority.AdminUsers: ("Administer all users", None, False),
    SiteWhereAuthority.AdminOwnUser: ("Administer own user profile", None, False),
    SiteWhereAuthority.AdminSchedules: ("Administer schedules", None, False),
    SiteWhereAuthority.REST: ("REST API access", None, False),
    SiteWhereAuthority.ViewServerInfo: ("View server information", None, False),
}


class UserManagement:
    """IUserManagement over an :class:`EntityStore`."""

    USERS, AUTHS = "users", "authorities"

    def __init__(self, store: EntityStore | None = None):
        self._s = store or create_store("memory")
        self._s.register(self.USERS, User, ("token", "username"))
        self._s.register(self.AUTHS, _AuthorityEntity, ("token",))

    # ---- users -------------------------------------------------------------------
    def create_user(self, request: dict, encode_password: bool = True) -> User:
        username = request.get("username")
        if not username:
            raise SiteWhereSystemException(ErrorCode.IncompleteData, detail="username required")
        if self._s.get_by(self.USERS, "username", username):
            raise SiteWhereSystemException(ErrorCode.DuplicateUser, detail=username)
        pw = request.get("password", "")
        u = User(token=username, username=username,
                 hashed_password=hash_password(pw) if encode_password else pw,
                 first_name=request.get("firstName", ""), last_name=request.get("lastName", ""),
                 email=request.get("email"), status=AccountStatus(request.get("status", "Active")),
                 authorities=list(request.get("authorities", [])), metadata=dict(request.get("metadata", {})))
        stamp_created(u)
        return _public(self._s.put(self.USERS, u))

    def import_user(self, user: User, overwrite: bool = False) -> User:
        if isinstance(user, dict):          # wire form (GImportUserRequest carries a GUser)
            user = User.from_dict(user)
        if not user.username:
            raise SiteWhereSystemException(ErrorCode.InvalidUsername, detail="user without a username")
        existing = self._s.get_by(self.USERS, "username", user.username)
        if existing and not overwrite:
            raise SiteWhereSystemException(ErrorCode.DuplicateUser, detail=user.username)
        if existing:
            user.id = existing.id
        user.token = user.username
        return _public(self._s.put(self.USERS, user))

    def authenticate(self, username: str, password: str, update_last_login: bool = True) -> User:
        u = self._s.get_by(self.USERS, "username", username)
        if u is None or not verify_password(password, u.hashed_password):
            raise UnauthorizedException("Invalid username or password")
        if u.status != AccountStatus.Active:
            raise UnauthorizedException(f"Account is {u.status.value}")
        if update_last_login:
            u.last_login = now_ms()
            self._s.put(self.USERS, u)
        return _public(u)

    def update_user(self, username: str, request: dict, encode_password: bool = True) -> User:
        u = self._require(username)
        for k, f in (("firstName", "first_name"), ("lastName", "last_name"), ("email", "email")):
            if k in request:
                setattr(u, f, request[k])
        if request.get("password"):
            u.hashed_password = hash_password(request["password"]) if encode_password else request["password"]
        if "status" in request:
            u.status = AccountStatus(request["status"])
        if "authorities" in request:
            u.authorities = list(request["authorities"])
        if "metadata" in request:
            u.metadata = dict(request["metadata"])
        stamp_updated(u)
        return _public(self._s.put(self.USERS, u))

    def get_user_by_username(self, username: str) -> User | None:
        u = self._s.get_by(self.USERS, "username", username)
        return _public(u) if u else None

    def list_users(self, criteria: SearchCriteria | None = None, include_deleted: bool = False) -> SearchResults:
        c = criteria or SearchCriteria(page_size=0)
        users = self._s.query(self.USERS, sort_key=lambda u: u.username)
        return SearchResults(len(users), [_public(u) for u in c.slice(users)])

    def delete_user(self, username: str) -> User:
        u = self._require(username)
        self._s.delete(self.USERS, u.id)
        return _public(u)

    def _require(self, username: str) -> User:
        u = self._s.get_by(self.USERS, "username", username)
        if u is None:
            raise NotFoundException(ErrorCode.InvalidUsername, username)
        return u

    # ---- authorities -----------------------------------------------------------
    def create_granted_authority(self, request: dict) -> GrantedAuthority:
        name = request.get("authority")
        if self._s.get_by_token(self.AUTHS, name):
            raise SiteWhereSystemException(ErrorCode.DuplicateAuthority, detail=name)
        e = _AuthorityEntity(token=name, authority=name, description=request.get("description", ""),
                             parent=request.get("parent"), group=bool(request.get("group", False)))
        self._s.put(self.AUTHS, e)
        return e.as_authority()

    def get_granted_authority_by_name(self, name: str) -> GrantedAuthority | None:
        e = self._s.get_by_token(self.AUTHS, name)
        return e.as_authority() if e else None

    def update_granted_authority(self, name: str, request: dict) -> GrantedAuthority:
        e = self._s.get_by_token(self.AUTHS, name)
        if e is None:
            raise NotFoundException(ErrorCode.InvalidAuthority, name)
        e.description = request.get("description", e.description)
        e.parent = request.get("parent", e.parent)
        e.group = bool(request.get("group", e.group))
        self._s.put(self.AUTHS, e)
        return e.as_authority()

    def list_granted_authorities(self, criteria: SearchCriteria | None = None) -> SearchResults:
        c = criteria or SearchCriteria(page_size=0)
        auths = [e.as_authority() for e in self._s.query(self.AUTHS, sort_key=lambda e: e.authority)]
        return SearchResults(len(auths), c.slice(auths))

    def delete_granted_authority(self, name: str) -> GrantedAuthority:
        e = self._s.get_by_token(self.AUTHS, name)
        if e is None:
            raise NotFoundException(ErrorCode.InvalidAuthority, name)
        self._s.delete(self.AUTHS, e.id)
        return e.as_authority()

    def get_granted_authorities_for_user(self, username: str) -> list[GrantedAuthority]:
        u = self._require(username)
        out = []
        for a in u.authorities:
            e = self._s.get_by_token(self.AUTHS, a)
            out.append(e.as_authority() if e else GrantedAuthority(authority=a))
        return out

    def add_granted_authorities_for_user(self, username: str, authorities: list[str]) -> list[GrantedAuthority]:
        u = self._require(username)
        for a in authorities:
            if a not in u.authorities:
                u.authorities.append(a)
        self._s.put(self.USERS, u)
        return self.get_granted_authorities_for_user(username)

    def remove_granted_authorities_for_user(self, username: str, authorities: list[str]) -> list[GrantedAuthority]:
        u = self._require(username)
        u.authorities = [a for a in u.authorities if a not in set(authorities)]
        self._s.put(self.USERS, u)
        return self.get_granted_authorities_for_user(username)


from dataclasses import dataclass  # noqa: E402

from ..models.domain import PersistentEntity  # noqa: E402


@dataclass
class _AuthorityEntity(PersistentEntity):
    authority: str = ""
    description: str = ""
    parent: str | None = None
    group: bool = False

    def as_authority(self) -> GrantedAuthority:
        return GrantedAuthority(self.authority, self.description, self.parent, self.group)


def _public(u: User) -> User:
    u = u.copy()
    u.hashed_password = ""
    return u


def bootstrap_default_users(um: UserManagement):
    """Instance template initializer (reference userModel.groovy): authorities + admin / noadmin."""
    for name, (desc, parent, group) in AUTHORITY_DESCRIPTIONS.items():
        if um.get_granted_authority_by_name(name) is None:
            um.create_granted_authority({"authority": name, "description": desc, "parent": parent, "group": group})
    if um.list_users().num_results == 0:
        all_auths = list(AUTHORITY_DESCRIPTIONS)
        um.create_user({"username": "admin", "password": "password", "firstName": "Admin", "lastName": "User",
                        "authorities": all_auths})
        limited = [a for a in all_auths if a not in (SiteWhereAuthority.AdminServer, SiteWhereAuthority.ViewServerInfo,
                                                     SiteWhereAuthority.AdminTenants, SiteWhereAuthority.AdminUsers)]
        um.create_user({"username": "noadmin", "password": "noadmin", "firstName": "Non-Admin", "lastName": "User",
                        "authorities": limited})


class UserManagementMicroservice(GlobalMicroservice):
    identifier = "user-management"
    name = "User Management"

    def __init__(self, instance, hostname=None, store: EntityStore | None = None):
        super().__init__(instance, hostname)
        self._store = store
        self.users: UserManagement | None = None

    def default_configuration(self) -> dict:
        return {"datastore": {"type": "memory"}}

    def register_services(self, resolver):
        from ..persistence.store import create_store as cs
        ds = self.global_configuration().get("datastore", {"type": "memory"})
        self.users = UserManagement(self._store or cs(ds.get("type", "memory"), **{k: v for k, v in ds.items()
                                                                                    if k != "type"}))
        resolver.add_global("UserManagement", self.users)

    def requires_instance_bootstrap(self) -> bool:
        return True

    def configuration_updated(self, doc):
        pass
