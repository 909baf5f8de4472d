"""service-instance-management: bootstraps the instance configuration tree and the user/tenant model.

Reference: ``InstanceManagementMicroservice.java:255-340`` -- ``verifyOrBootstrapConfiguration``
(copy the instance template into the coordination tree, write ``/<instance>/state/bootstrapped``;
every other microservice blocks on that marker) then ``initializeModelFromInstanceTemplate``
(user and tenant initializer scripts run as the system user once those services are up).
"""
from __future__ import annotations

import threading

from ..core.lifecycle import CompositeLifecycleStep, SimpleLifecycleStep
from ..runtime.config import dump_document
from ..runtime.microservice import GlobalMicroservice

INSTANCE_TEMPLATES = {
    "default": {
        "name": "Default",
        "conf": {
            "instance-management.json": {"instanceTemplate": "default"},
            "user-management.json": {"datastore": {"type": "memory"}},
            "tenant-management.json": {"datastore": {"type": "memory"}},
            "web-rest.json": {"port": 8080, "cors": True},
        },
        "initializers": {"userManagement": ["default-users"], "tenantManagement": ["default-tenant"]},
    },
    "empty": {"name": "Empty (no users/tenants)", "conf": {}, "initializers": {}},
}


class InstanceManagementMicroservice(GlobalMicroservice):
    identifier = "instance-management"
    name = "Instance Management"

    def __init__(self, instance, hostname=None, template: str = "default", initialize_model: bool = True):
        super().__init__(instance, hostname)
        self.template = template
        self.initialize_model = initialize_model
        self.model_initialized = threading.Event()

    def requires_instance_bootstrap(self) -> bool:
        return False  # this service creates the marker

    def microservice_initialize(self, monitor):
        CompositeLifecycleStep("Instance bootstrap", [
            SimpleLifecycleStep("Verify instance configured", lambda m: self.verify_or_bootstrap_configuration()),
        ]).execute(monitor)

    def verify_or_bootstrap_configuration(self) -> bool:
        inst = self.instance
        inst.coord.ensure(inst.path("state"))
        if inst.coord.exists(inst.bootstrapped_marker()):
            self.logger.info("found bootstrap marker; skipping instance bootstrap")
            return False
        tpl = INSTANCE_TEMPLATES[self.template]
        for name, doc in tpl["conf"].items():
            inst.coord.put(inst.conf_path(name), dump_document(doc))
        inst.coord.ensure(inst.conf_path("tenants"))
        inst.coord.ensure(inst.bootstrapped_marker())
        return True

    def microservice_start(self, monitor):
        if self.initialize_model:
            threading.Thread(target=self._initialize_model, daemon=True, name="instance-model-init").start()

    def _initialize_model(self):
        """Run the template's user/tenant initializers once (markers make it idempotent)."""
        inst = self.instance
        tpl = INSTANCE_TEMPLATES[self.template]
        try:
            inits = tpl.get("initializers", {})
            if inits.get("userManagement") and not inst.coord.exists(inst.path("state", "users-bootstrapped")):
                self.demux("user-management").wait_for_available(60)
                self._wait_service("UserManagement")
                from .user_management import bootstrap_default_users
                inst.system_user.run(lambda: bootstrap_default_users(self.api("UserManagement")))
                inst.coord.ensure(inst.path("state", "users-bootstrapped"))
            if inits.get("tenantManagement") and not inst.coord.exists(inst.path("state", "tenants-bootstrapped")):
                self._wait_service("TenantManagement")
                from .tenant_management import bootstrap_default_tenant
                inst.system_user.run(lambda: bootstrap_default_tenant(self.api("TenantManagement")))
                inst.coord.ensure(inst.path("state", "tenants-bootstrapped"))
        except Exception:
            self.logger.exception("instance model initialization failed")
        finally:
            self.model_initialized.set()

    def _wait_service(self, name: str, timeout_s: float = 60.0):
        import time
        end = time.time() + timeout_s
        while name not in self.instance.resolver.names():
            if time.time() > end:
                raise TimeoutError(name)
            time.sleep(0.05)
