"""service-asset-management: asset types and assets (multitenant).

Reference: ``AssetManagementImpl`` over ``MongoAssetManagement`` + ``CacheAwareAssetManagement``;
RPCs (``asset-management.proto``, 12): Create/Update/GetById/GetByToken/Delete/List for AssetType and Asset.
"""
from __future__ import annotations

from ..core.errors import ErrorCode, SiteWhereSystemException
from ..models.domain import Asset, AssetType
from ..persistence.store import create_store
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from .common import Crud


class AssetManagement:
    def __init__(self, store=None):
        s = store or create_store("memory")
        self.asset_types = Crud(s, "assetTypes", AssetType, ErrorCode.InvalidAssetTypeToken)
        self.assets = Crud(s, "assets", Asset, ErrorCode.InvalidAssetToken)

    def create_asset_type(self, request: dict):
        return self.asset_types.create(request)

    def update_asset_type(self, id: str, request: dict):
        return self.asset_types.update(id, request)

    def get_asset_type(self, id: str):
        return self.asset_types.get(id)

    get_asset_type_by_id = get_asset_type

    def get_asset_type_by_token(self, token: str):
        return self.asset_types.get_by_token(token)

    def delete_asset_type(self, id: str):
        if self.assets.query(lambda a: a.asset_type_id == id):
            raise SiteWhereSystemException(ErrorCode.DeviceTypeInUse, detail="asset type has assets")
        return self.asset_types.delete(id)

    def list_asset_types(self, criteria=None):
        return self.asset_types.list(criteria, sort=lambda e: e.name)

    def create_asset(self, request: dict):
        at = self.asset_types.require_token(request["assetTypeToken"]).id if request.get("assetTypeToken") \
            else self.asset_types.require(request["assetTypeId"]).id
        return self.assets.create(request, asset_type_id=at)

    def update_asset(self, id: str, request: dict):
        fixed = {}
        if request.get("assetTypeToken"):
            fixed["asset_type_id"] = self.asset_types.require_token(request["assetTypeToken"]).id
        return self.assets.update(id, request, **fixed)

    def get_asset(self, id: str):
        return self.assets.get(id)

    get_asset_by_id = get_asset

    def get_asset_by_token(self, token: str):
        return self.assets.get_by_token(token)

    def delete_asset(self, id: str):
        return self.assets.delete(id)

    def list_assets(self, criteria=None):
        c = criteria or {}
        at = c.get("assetTypeId") if isinstance(c, dict) else None
        if isinstance(c, dict) and c.get("assetTypeToken"):
            at = self.asset_types.require_token(c["assetTypeToken"]).id
        return self.assets.list(c, (lambda a: a.asset_type_id == at) if at else None, sort=lambda e: e.name)


class AssetManagementTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ds = self.config.get("datastore", {"type": "memory"})
        self.management = AssetManagement(create_store(ds.get("type", "memory"),
                                                       **{k: v for k, v in ds.items() if k != "type"}))
        self.api = {"AssetManagement": self.management}

    def tenant_bootstrap(self, dataset_template, monitor):
        from .builders import AssetBuilder
        from .dataset_runner import run_initializers
        run_initializers(self, "assetManagement", dataset_template, {"asset_builder": AssetBuilder(self.management)})


class AssetManagementMicroservice(MultitenantMicroservice):
    identifier = "asset-management"
    name = "Asset Management"

    def service_names(self):
        return ["AssetManagement"]

    def create_tenant_engine(self, tenant):
        return AssetManagementTenantEngine(self, tenant)
