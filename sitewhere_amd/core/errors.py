"""Exceptions and error codes (reference: sitewhere-core-api/.../spi/error/ErrorCode.java, ErrorLevel.java,
SiteWhereException.java, SiteWhereSystemException.java, ServerStartupException.java)."""
from __future__ import annotations

from enum import Enum


class ErrorLevel(str, Enum):
    INFO = "INFO"
    WARNING = "WARNING"
    ERROR = "ERROR"
    CRITICAL = "CRITICAL"


class ErrorCode(Enum):
    """Subset-compatible error codes; values mirror the reference numbering where it exists."""
    Error = (0, "Unknown error.")
    InvalidDeviceTypeToken = (1, "Device type token not found.")
    InvalidDeviceToken = (2, "Device token not found.")
    DuplicateDeviceToken = (3, "Device token already exists.")
    InvalidDeviceAssignmentToken = (4, "Device assignment token not found.")
    DeviceAlreadyAssigned = (5, "Device is already assigned.")
    DeviceNotAssigned = (6, "Device is not assigned.")
    InvalidCustomerTypeToken = (7, "Customer type token not found.")
    InvalidCustomerToken = (8, "Customer token not found.")
    InvalidAreaTypeToken = (9, "Area type token not found.")
    InvalidAreaToken = (10, "Area token not found.")
    InvalidZoneToken = (11, "Zone token not found.")
    InvalidDeviceCommandToken = (12, "Device command token not found.")
    InvalidDeviceStatusCode = (13, "Device status code not found.")
    InvalidDeviceGroupToken = (14, "Device group token not found.")
    InvalidAssetTypeToken = (15, "Asset type token not found.")
    InvalidAssetToken = (16, "Asset token not found.")
    InvalidBatchOperationToken = (17, "Batch operation token not found.")
    InvalidScheduleToken = (18, "Schedule token not found.")
    InvalidScheduledJobToken = (19, "Scheduled job token not found.")
    InvalidUsername = (20, "Username not found.")
    DuplicateUser = (21, "Username already exists.")
    InvalidPassword = (22, "Invalid password.")
    InvalidAuthority = (23, "Granted authority not found.")
    DuplicateAuthority = (24, "Granted authority already exists.")
    InvalidTenantToken = (25, "Tenant token not found.")
    DuplicateTenantToken = (26, "Tenant token already exists.")
    DuplicateToken = (27, "Token already in use.")
    InvalidStreamId = (28, "Stream id not found.")
    DuplicateStreamId = (29, "Stream id already exists.")
    InvalidDeviceEventId = (30, "Device event id not found.")
    DeviceParentCycle = (31, "Device parent relationship would create a cycle.")
    DeviceElementMappingExists = (32, "Device element mapping already exists for path.")
    InvalidDeviceElementPath = (33, "Invalid device element path.")
    IncompleteData = (34, "Required data was not provided.")
    NotAuthorized = (35, "Not authorized.")
    InvalidAlarmId = (36, "Device alarm not found.")
    InvalidDeviceStateId = (37, "Device state not found.")
    TenantEngineNotAvailable = (38, "Tenant engine not available.")
    InvalidScript = (39, "Script not found.")
    InvalidCommandParameter = (40, "Invalid command parameter value.")
    DeviceTypeInUse = (41, "Device type is in use by existing devices.")
    AssignmentNotActive = (42, "Assignment is not active.")
    InvalidTemplate = (43, "Template not found.")

    @property
    def code(self) -> int:
        return self.value[0]

    @property
    def message(self) -> str:
        return self.value[1]


class SiteWhereException(Exception):
    """Base framework exception."""


class SiteWhereSystemException(SiteWhereException):
    def __init__(self, code: ErrorCode, level: ErrorLevel = ErrorLevel.ERROR, detail: str | None = None,
                 http_status: int = 400):
        self.code = code
        self.level = level
        self.http_status = http_status
        super().__init__(detail or code.message)

    def to_dict(self):
        return {"errorCode": self.code.code, "errorName": self.code.name, "errorLevel": self.level.value,
                "message": str(self)}


class NotFoundException(SiteWhereSystemException):
    def __init__(self, code: ErrorCode, detail: str | None = None):
        super().__init__(code, ErrorLevel.ERROR, detail, http_status=404)


class UnauthorizedException(SiteWhereSystemException):
    def __init__(self, detail: str | None = None):
        super().__init__(ErrorCode.NotAuthorized, ErrorLevel.ERROR, detail, http_status=401)


class ServerStartupException(SiteWhereException):
    """Raised when a *required* nested component fails (LifecycleComponent.java:218-232)."""

    def __init__(self, component, message: str, cause: BaseException | None = None):
        self.component = component
        self.cause = cause
        super().__init__(f"{message}: {cause}" if cause else message)


class EventDecodeException(SiteWhereException):
    pass


class TenantEngineNotAvailableException(SiteWhereSystemException):
    def __init__(self, detail: str | None = None):
        super().__init__(ErrorCode.TenantEngineNotAvailable, ErrorLevel.ERROR, detail, http_status=503)
