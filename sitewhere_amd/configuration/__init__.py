"""Configuration models of every microservice (reference ``sitewhere-configuration`` plus each
service's ``*ModelProvider`` / ``*Roles``); see ``model.py``."""
from __future__ import annotations

from .model import Attr, ConfigurationModel, Element, ModelProvider, Role
from .services import (AssetManagementProvider, BatchOperationsProvider, CommandDeliveryProvider,
                       DeviceManagementProvider, DeviceStateProvider, EventManagementProvider, EventSearchProvider,
                       InstanceManagementProvider, LabelGenerationProvider, OutboundConnectorsProvider,
                       RuleProcessingProvider, ScheduleManagementProvider, StreamingMediaProvider,
                       TenantManagementProvider, UserManagementProvider, WebRestProvider)
from .sources import DeviceRegistrationProvider, EventSourcesProvider, InboundProcessingProvider

PROVIDERS = (InstanceManagementProvider, UserManagementProvider, TenantManagementProvider, WebRestProvider,
             EventSourcesProvider, InboundProcessingProvider, DeviceRegistrationProvider, EventManagementProvider,
             DeviceManagementProvider, AssetManagementProvider, BatchOperationsProvider,
             ScheduleManagementProvider, DeviceStateProvider, RuleProcessingProvider, OutboundConnectorsProvider,
             CommandDeliveryProvider, LabelGenerationProvider, StreamingMediaProvider, EventSearchProvider)

MODELS: dict[str, ConfigurationModel] = {p.identifier: p().build() for p in PROVIDERS}


def model_for(identifier: str) -> ConfigurationModel | None:
    return MODELS.get(identifier)


__all__ = ["Attr", "ConfigurationModel", "Element", "ModelProvider", "Role", "MODELS", "PROVIDERS", "model_for"]
