"""service-batch-operations: batch command invocations with throttling, pause and resume.

Reference: ``BatchOperationManager.java:49-262`` (10 threads; only ``Unprocessed`` elements are
processed -- the restart/resume semantics; each element Processing -> Succeeded/Failed; throttle
delay between elements) and ``BatchCommandInvocationHandler``; RPCs (``batch-management.proto``, 9):
CreateBatchOperation, CreateBatchCommandInvocation, UpdateBatchOperation, GetBatchOperation,
GetBatchOperationByToken, ListBatchOperations, DeleteBatchOperation, ListBatchOperationElements,
UpdateBatchOperationElement.
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import ThreadPoolExecutor

from ..core.errors import ErrorCode, NotFoundException
from ..models.domain import (BatchElement, BatchOperation, BatchOperationStatus, CommandInitiator,
                             ElementProcessingStatus, SearchResults, now_ms)
from ..persistence.store import create_store
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from .common import Crud, criteria_of

INVOKE_COMMAND = "InvokeCommand"


class BatchManagement:
    def __init__(self, store=None, on_created=None):
        s = self._s = store or create_store("memory")
        self.ops = Crud(s, "batchOperations", BatchOperation, ErrorCode.InvalidBatchOperationToken)
        s.register("batchElements", BatchElement, ())
        self._on_created = on_created or (lambda op: None)

    def create_batch_operation(self, request: dict, device_ids: list[str] | None = None) -> BatchOperation:
        op = self.ops.create(request, processing_status=BatchOperationStatus.Unprocessed)
        for d in device_ids or request.get("deviceIds", []) or []:
            self._s.put("batchElements", BatchElement(batch_operation_id=op.id, device_id=d))
        self._on_created(op)
        return op

    def create_batch_command_invocation(self, request: dict) -> BatchOperation:
        """{token?, commandToken, parameterValues, deviceTokens | deviceIds} -> InvokeCommand batch."""
        params = {"commandToken": request["commandToken"], "parameterValues": request.get("parameterValues", {})}
        return self.create_batch_operation({"token": request.get("token"), "operationType": INVOKE_COMMAND,
                                            "parameters": params, "metadata": request.get("metadata", {})},
                                           request.get("deviceIds", []))

    def update_batch_operation(self, id: str, request: dict):
        return self.ops.update(id, request)

    def get_batch_operation(self, id: str):
        return self.ops.get(id)

    def get_batch_operation_by_token(self, token: str):
        return self.ops.get_by_token(token)

    def list_batch_operations(self, criteria=None):
        return self.ops.list(criteria, sort=lambda o: o.created_date or 0, reverse=True)

    def delete_batch_operation(self, id: str):
        op = self.ops.delete(id)
        for e in self._elements(id):
            self._s.delete("batchElements", e.id)
        return op

    def _elements(self, op_id: str) -> list[BatchElement]:
        return self._s.query("batchElements", lambda e: e.batch_operation_id == op_id, sort_key=lambda e: e.id)

    def list_batch_operation_elements(self, op_id: str, criteria=None) -> SearchResults:
        c = criteria or {}
        st = c.get("processingStatus") if isinstance(c, dict) else None
        els = [e for e in self._elements(op_id) if not st or e.processing_status.value == st]
        cc = criteria_of(c if isinstance(c, dict) and "pageSize" in c else None)
        return SearchResults(len(els), cc.slice(els))

    def update_batch_operation_element(self, element_id: str, request: dict) -> BatchElement:
        e = self._s.get("batchElements", element_id)
        if e is None:
            raise NotFoundException(ErrorCode.InvalidBatchOperationToken, element_id)
        if "processingStatus" in request:
            e.processing_status = ElementProcessingStatus(request["processingStatus"])
        if "processedDate" in request:
            e.processed_date = request["processedDate"]
        if "metadata" in request:
            e.metadata = dict(request["metadata"])
        return self._s.put("batchElements", e)


class BatchOperationManager:
    """Processes operations on a pool; throttling, pause/resume; restarts skip finished elements."""

    def __init__(self, engine, threads: int = 10, throttle_ms: int = 0):
        self.engine = engine
        self.pool = ThreadPoolExecutor(max_workers=threads, thread_name_prefix="batch-op")
        self.throttle_ms = throttle_ms
        self._paused = threading.Event()
        self._paused.set()
        self.futures = {}

    def pause(self):
        self._paused.clear()

    def resume(self):
        self._paused.set()

    def submit(self, op: BatchOperation):
        self.futures[op.id] = self.pool.submit(self.process, op.id)
        return self.futures[op.id]

    def process(self, op_id: str):
        bm: BatchManagement = self.engine.management
        op = bm.get_batch_operation(op_id)
        bm.update_batch_operation(op_id, {"processingStatus": BatchOperationStatus.Processing.value,
                                          "processingStartedDate": now_ms()})
        failed = 0
        for el in bm._elements(op_id):
            if el.processing_status != ElementProcessingStatus.Unprocessed:
                continue      # resume semantics (BatchOperationManager.java:215)
            self._paused.wait()
            bm.update_batch_operation_element(el.id, {"processingStatus": "Processing"})
            try:
                self.handle_element(op, el)
                st = ElementProcessingStatus.Succeeded
            except Exception as e:  # noqa: BLE001
                st = ElementProcessingStatus.Failed
                failed += 1
                self.engine.logger.warning("batch element %s failed: %s", el.id, e)
            bm.update_batch_operation_element(el.id, {"processingStatus": st.value, "processedDate": now_ms()})
            if self.throttle_ms:
                time.sleep(self.throttle_ms / 1000.0)
        bm.update_batch_operation(op_id, {
            "processingStatus": (BatchOperationStatus.FinishedWithErrors if failed else
                                 BatchOperationStatus.FinishedSuccessfully).value, "processingEndedDate": now_ms()})
        return failed

    def handle_element(self, op: BatchOperation, el: BatchElement):
        """BatchCommandInvocationHandler: create a command invocation on the device's assignment."""
        if op.operation_type != INVOKE_COMMAND:
            raise ValueError(f"unsupported batch operation {op.operation_type}")
        t = self.engine.tenant.token
        dm = self.engine.ms.api("DeviceManagement", t)
        dev = dm.get_device(el.device_id)
        if dev is None or not dev.device_assignment_id:
            raise ValueError("device not assigned")
        cmd = dm.get_device_command_by_token(op.parameters["commandToken"])
        self.engine.ms.api("DeviceEventManagement", t).add_command_invocations(dev.device_assignment_id, {
            "initiator": CommandInitiator.BatchOperation.value, "initiatorId": op.id, "target": "Assignment",
            "targetId": dev.device_assignment_id, "commandToken": op.parameters["commandToken"],
            "deviceCommandId": cmd.id if cmd else None, "parameterValues": op.parameters.get("parameterValues", {})})


class BatchOperationsTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ds = self.config.get("datastore", {"type": "memory"})
        self.manager = BatchOperationManager(self, int(self.config.get("threads", 10)),
                                             int(self.config.get("throttleDelayMs", 0)))
        self.management = BatchManagement(create_store(ds.get("type", "memory"),
                                                       **{k: v for k, v in ds.items() if k != "type"}),
                                          on_created=self.manager.submit)
        self.api = {"BatchManagement": self.management}

    def tenant_start(self, monitor):
        # resume operations interrupted by a restart
        for op in self.management.ops.query():
            if op.processing_status in (BatchOperationStatus.Unprocessed, BatchOperationStatus.Processing):
                self.manager.submit(op)


class BatchOperationsMicroservice(MultitenantMicroservice):
    identifier = "batch-operations"
    name = "Batch Operations"

    def service_names(self):
        return ["BatchManagement"]

    def create_tenant_engine(self, tenant):
        return BatchOperationsTenantEngine(self, tenant)
