"""Configuration models: roles, elements and attributes of every microservice's configuration.

Reference: ``sitewhere-configuration/.../model/ConfigurationModelProvider.java:37-280`` (elements
registered per role, roles resolved from the root role, dependencies on shared providers),
``ElementNode`` / ``AttributeNode`` builders with attribute groups (General, Connectivity,
Authentication, Performance, Batch), each service's ``*Roles`` enum (role -> permitted child roles
and subtype roles, optional / multiple / reorderable / permanent) and ``*ModelProvider`` (one element
per concrete component, ``specializes`` narrowing a child role).  ``GetConfigurationModel`` returns
``{rootRoleId, rolesById, elementsByRole}`` for the admin editor.

Here configuration documents are JSON, not Spring XML: a role is the key under which its
elements sit in the parent element (one object, or a list when the role is ``multiple``), and
the concrete element is chosen by the ``type`` attribute (``discriminator``).  The same tree
validates documents (``ConfigurationModel.validate``): required attributes, attribute types and
choices, unknown keys, role cardinality and permitted element types, recursively, with JSON paths
in the messages.  Management updates are rejected when they do not validate.
"""
from __future__ import annotations

from dataclasses import dataclass, field

GROUPS = {"genr": "General", "conn": "Connectivity", "auth": "Authentication", "perf": "Performance",
          "btch": "Batch Settings", "stor": "Storage", "engn": "MI355X Engine", "scrp": "Scripting",
          "flt": "Filtering"}


@dataclass
class Attr:
    """One configuration attribute (reference ``AttributeNode``)."""
    name: str
    type: str = "String"          # String | Integer | Decimal | Boolean | Script | StringList | Map | List | Object
    description: str = ""
    required: bool = False
    default: object = None
    choices: tuple = ()
    group: str = "genr"
    index: bool = False           # uniquely identifies the element among its siblings (reference makeIndex)
    label: str = ""

    def to_dict(self) -> dict:
        d = {"localName": self.name, "name": self.label or self.name, "type": self.type,
             "description": self.description, "required": self.required, "group": self.group, "index": self.index}
        if self.default is not None:
            d["defaultValue"] = self.default
        if self.choices:
            d["choices"] = list(self.choices)
        return d

    def check(self, v, path: str) -> str | None:
        t = self.type
        if isinstance(v, str) and "${" in v:
            return None                       # instance-settings substitution happens at load time
        ok = True
        if t == "Integer":
            ok = (isinstance(v, int) and not isinstance(v, bool)) or (isinstance(v, str) and v.lstrip("-").isdigit())
        elif t == "Decimal":
            ok = isinstance(v, (int, float)) and not isinstance(v, bool)
            if isinstance(v, str):
                try:
                    float(v)
                    ok = True
                except ValueError:
                    ok = False
        elif t == "Boolean":
            ok = isinstance(v, bool) or v in ("true", "false")
        elif t == "String":
            ok = isinstance(v, str)
        elif t == "Script":
            ok = isinstance(v, (str, dict))
        elif t == "StringList":
            ok = isinstance(v, list) and all(isinstance(x, str) for x in v)
        elif t == "Map":
            ok = isinstance(v, dict)
        elif t == "List":
            ok = isinstance(v, list)
        elif t == "Object":
            ok = isinstance(v, dict)
        elif t == "StringOrInteger":
            ok = isinstance(v, (str, int)) and not isinstance(v, bool)
        if not ok:
            return f"{path}: {self.name} must be {t}, got {type(v).__name__}"
        if self.choices and v not in self.choices:
            return f"{path}: {self.name}={v!r} is not one of {list(self.choices)}"
        return None


@dataclass
class Role:
    """A position in the configuration tree (reference ``ConfigurationRole``)."""
    id: str
    name: str
    key: str | None = None        # JSON key under the parent element (None: the root)
    optional: bool = True
    multiple: bool = False
    reorderable: bool = False
    permanent: bool = False
    children: tuple = ()          # child role ids every element of this role has
    subtypes: tuple = ()          # roles whose elements may also fill this role
    shorthand: bool = False       # a bare string stands for {"type": <string>}
    discriminator: str = "type"   # attribute that selects the element filling this role

    def to_dict(self) -> dict:
        return {"id": self.id, "name": self.name, "key": self.key, "discriminator": self.discriminator,
                "optional": self.optional,
                "multiple": self.multiple, "reorderable": self.reorderable, "permanent": self.permanent,
                "childRoles": list(self.children), "subtypeRoles": list(self.subtypes), "shorthand": self.shorthand}


@dataclass
class Element:
    """A concrete configurable component (reference ``ElementNode``)."""
    name: str
    role: str
    type_value: tuple = ()        # accepted values of the ``type`` discriminator (empty: the only element)
    description: str = ""
    attrs: list = field(default_factory=list)
    icon: str = "cog"
    children: tuple = ()          # extra child roles of this element (beyond its role's)
    specializes: dict = field(default_factory=dict)     # child role -> narrower role (reference specializes)
    open: bool = False            # accepts keys the model does not list (free-form sub-documents)

    def to_dict(self) -> dict:
        groups = sorted({a.group for a in self.attrs})
        return {"name": self.name, "role": self.role, "localName": self.type_value[0] if self.type_value else self.role,
                "typeValues": list(self.type_value), "description": self.description, "icon": self.icon,
                "attributeGroups": [{"id": g, "name": GROUPS.get(g, g)} for g in groups],
                "attributes": [a.to_dict() for a in self.attrs], "childRoles": list(self.children),
                "specializes": dict(self.specializes)}


class ConfigurationModel:
    """Built model of one microservice (reference ``ConfigurationModel``)."""

    def __init__(self, microservice: str, name: str, root_role: str, roles: dict, elements: dict,
                 description: str = ""):
        self.microservice, self.name, self.description = microservice, name, description
        self.root_role, self.roles, self.elements = root_role, roles, elements

    # ---------------------------------------------------------------- views
    @property
    def root(self) -> Element:
        return self.elements[self.root_role][0]

    def elements_for(self, role_id: str) -> list:
        """Elements that may fill ``role_id`` (its own and its subtype roles', transitively)."""
        out, seen, todo = [], set(), [role_id]
        while todo:
            r = todo.pop()
            if r in seen:
                continue
            seen.add(r)
            out += self.elements.get(r, [])
            role = self.roles.get(r)
            if role is not None:
                todo += list(role.subtypes)
        return out

    def child_roles(self, el: Element) -> list:
        role = self.roles[el.role]
        out = []
        for rid in tuple(role.children) + tuple(el.children):
            rid = el.specializes.get(rid, rid)
            if rid not in out:
                out.append(rid)
        return out

    def to_dict(self) -> dict:
        def tree(el: Element, depth=0):
            d = el.to_dict()
            d["children"] = [] if depth > 8 else [
                {"role": self.roles[r].to_dict(), "elements": [tree(e, depth + 1) for e in self.elements_for(r)]}
                for r in self.child_roles(el)]
            return d
        return {"microservice": self.microservice, "name": self.name, "description": self.description,
                "rootRoleId": self.root_role,
                "rolesById": {k: r.to_dict() for k, r in sorted(self.roles.items())},
                "elementsByRole": {k: [e.to_dict() for e in v] for k, v in sorted(self.elements.items())},
                "root": dict(tree(self.root), role=self.microservice)}

    # ---------------------------------------------------------------- validation
    def validate(self, doc) -> list[str]:
        """All problems of ``doc`` against the model, as ``path: message`` strings (empty: valid)."""
        errs: list[str] = []
        if not isinstance(doc, dict):
            return [f"$: configuration must be an object, got {type(doc).__name__}"]
        self._element(self.root, doc, "$", errs)
        return errs

    def _pick(self, role: Role, item, path: str, errs: list):
        cands = self.elements_for(role.id)
        if not cands:
            errs.append(f"{path}: no element can fill role {role.id}")
            return None, item
        if isinstance(item, str) and role.shorthand:
            item = {role.discriminator: item}
        if not isinstance(item, dict):
            errs.append(f"{path}: {role.name} must be an object, got {type(item).__name__}")
            return None, item
        if len(cands) == 1 and not cands[0].type_value:
            return cands[0], item
        t = item.get(role.discriminator)
        for e in cands:
            if t in e.type_value:
                return e, item
        if t is None and len(cands) == 1:
            return cands[0], item
        allowed = sorted({v for e in cands for v in e.type_value})
        errs.append(f"{path}: {role.name} {role.discriminator} {t!r} is not one of {allowed}")
        return None, item

    def _element(self, el: Element, doc: dict, path: str, errs: list):
        known = {a.name: a for a in el.attrs}
        roles = {self.roles[r].key: self.roles[r] for r in self.child_roles(el)}
        disc = self.roles[el.role].discriminator if el.role in self.roles else "type"
        for a in el.attrs:
            if a.required and doc.get(a.name) is None:
                errs.append(f"{path}: missing required attribute {a.name}")
        for k, v in doc.items():
            if k in roles:
                continue
            a = known.get(k)
            if a is None:
                if k != disc and not el.open:
                    errs.append(f"{path}: unknown attribute {k!r} for {el.name}")
                continue
            if v is None:
                continue
            e = a.check(v, path)
            if e:
                errs.append(e)
        # index attributes unique among siblings are checked by the caller
        for key, role in roles.items():
            v = doc.get(key)
            p = f"{path}.{key}"
            if v is None:
                if not role.optional:
                    errs.append(f"{path}: missing required {role.name} ({key})")
                continue
            items = v if role.multiple else [v]
            if role.multiple and not isinstance(v, list):
                errs.append(f"{p}: {role.name} must be a list")
                continue
            seen = {}
            for i, item in enumerate(items):
                ip = f"{p}[{i}]" if role.multiple else p
                child, item = self._pick(role, item, ip, errs)
                if child is None:
                    continue
                for a in child.attrs:
                    if a.index and isinstance(item, dict) and item.get(a.name) is not None:
                        if item[a.name] in seen:
                            errs.append(f"{ip}: duplicate {a.name} {item[a.name]!r} (also at index {seen[item[a.name]]})")
                        seen.setdefault(item[a.name], i)
                self._element(child, item, ip, errs)


class ModelProvider:
    """Builds one microservice's model from its roles and elements plus shared providers'
    (reference ``ConfigurationModelProvider``: ``initializeDependencies`` / ``initializeElements``
    / ``initializeRoles`` / ``buildModel``)."""

    identifier = ""
    title = ""
    description = ""
    root_role = ""

    def __init__(self):
        self.roles: dict[str, Role] = {}
        self.elements: dict[str, list[Element]] = {}
        self.dependencies: list["ModelProvider"] = []
        self.initialize_dependencies()
        self.initialize_roles()
        self.initialize_elements()

    def initialize_dependencies(self):
        pass

    def initialize_roles(self):
        pass

    def initialize_elements(self):
        pass

    def role(self, r: Role):
        self.roles[r.id] = r

    def element(self, e: Element):
        self.elements.setdefault(e.role, []).append(e)

    def build(self) -> ConfigurationModel:
        roles, elements = {}, {}
        for p in self.dependencies + [self]:
            roles.update(p.roles)
            for k, v in p.elements.items():
                elements.setdefault(k, []).extend(v)
        # keep only what the root role reaches (reference findUsedRoles / findUsedElements)
        used, todo = set(), [self.root_role]
        while todo:
            r = todo.pop()
            if r in used or r not in roles:
                continue
            used.add(r)
            todo += list(roles[r].children) + list(roles[r].subtypes)
            for e in elements.get(r, []):
                todo += list(e.children) + list(e.specializes.values())
        missing = [r for rr in used for r in roles[rr].children if r not in roles]
        if missing:
            raise ValueError(f"{self.identifier}: undefined roles {missing}")
        return ConfigurationModel(self.identifier, self.title, self.root_role,
                                  {k: v for k, v in roles.items() if k in used},
                                  {k: v for k, v in elements.items() if k in used}, self.description)
