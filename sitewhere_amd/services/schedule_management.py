"""service-schedule-management: schedules and scheduled jobs that fire command invocations.

Reference: ``QuartzScheduleManager.java:41-180`` (simple + cron triggers), ``CommandInvocationJob``,
``BatchCommandInvocationJob``; RPCs (``schedule-management.proto``, 10): Create/Update/GetByToken/List/
Delete for Schedule and ScheduledJob.  Quartz is replaced by a small timer wheel with a 5-field cron
parser.
"""
from __future__ import annotations

import datetime as _dt
import threading

from ..core.errors import ErrorCode
from ..models.domain import (CommandInitiator, Schedule, ScheduledJob, ScheduledJobState, ScheduledJobType,
                             TriggerType, now_ms)
from ..persistence.store import create_store
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from .common import Crud


class CronExpression:
    """5-field cron: minute hour day-of-month month day-of-week (``*``, ``*/n``, ``a-b``, ``a,b``)."""

    RANGES = [(0, 59), (0, 23), (1, 31), (1, 12), (0, 6)]

    def __init__(self, expr: str):
        parts = expr.split()
        if len(parts) == 6:         # Quartz style with seconds: drop seconds
            parts = parts[1:]
        if len(parts) != 5:
            raise ValueError(f"bad cron expression {expr!r}")
        self.sets = [self._field(p.replace("?", "*"), lo, hi) for p, (lo, hi) in zip(parts, self.RANGES)]

    @staticmethod
    def _field(s, lo, hi):
        out = set()
        for part in s.split(","):
            step = 1
            if "/" in part:
                part, st = part.split("/")
                step = int(st)
            if part in ("*", ""):
                a, b = lo, hi
            elif "-" in part:
                a, b = map(int, part.split("-"))
            else:
                a = b = int(part)
            out.update(range(a, b + 1, step))
        return out

    def matches(self, t: _dt.datetime) -> bool:
        dow = (t.weekday() + 1) % 7
        return (t.minute in self.sets[0] and t.hour in self.sets[1] and t.day in self.sets[2] and
                t.month in self.sets[3] and dow in self.sets[4])

    def next_after(self, ms: int) -> int:
        t = _dt.datetime.fromtimestamp(ms / 1000.0).replace(second=0, microsecond=0) + _dt.timedelta(minutes=1)
        for _ in range(366 * 24 * 60):
            if self.matches(t):
                return int(t.timestamp() * 1000)
            t += _dt.timedelta(minutes=1)
        raise ValueError("cron expression never fires")


def next_fire(schedule: Schedule, after_ms: int, fired: int) -> int | None:
    if schedule.end_date and after_ms > schedule.end_date:
        return None
    start = schedule.start_date or 0
    cfg = schedule.trigger_configuration or {}
    if schedule.trigger_type == TriggerType.CronTrigger:
        n = CronExpression(cfg["cronExpression"]).next_after(max(after_ms, start))
    else:
        interval = int(cfg.get("repeatInterval", 60000))
        count = int(cfg.get("repeatCount", -1))
        if count >= 0 and fired > count:
            return None
        n = max(start, after_ms) if fired == 0 else after_ms + interval
    return None if (schedule.end_date and n > schedule.end_date) else n


class ScheduleManagement:
    def __init__(self, store=None, on_change=None):
        s = store or create_store("memory")
        self.schedules = Crud(s, "schedules", Schedule, ErrorCode.InvalidScheduleToken)
        self.jobs = Crud(s, "scheduledJobs", ScheduledJob, ErrorCode.InvalidScheduledJobToken)
        self._on_change = on_change or (lambda: None)

    def create_schedule(self, request: dict):
        s = self.schedules.create(request)
        self._on_change()
        return s

    def update_schedule(self, token: str, request: dict):
        s = self.schedules.update(self.schedules.require_token(token).id, request)
        self._on_change()
        return s

    def get_schedule_by_token(self, token: str):
        return self.schedules.get_by_token(token)

    def list_schedules(self, criteria=None):
        return self.schedules.list(criteria, sort=lambda e: e.name)

    def delete_schedule(self, token: str):
        s = self.schedules.delete(self.schedules.require_token(token).id)
        self._on_change()
        return s

    def create_scheduled_job(self, request: dict):
        sched = self.schedules.require_token(request["scheduleToken"])
        j = self.jobs.create(request, schedule_id=sched.id, job_state=ScheduledJobState.Active)
        self._on_change()
        return j

    def update_scheduled_job(self, token: str, request: dict):
        j = self.jobs.update(self.jobs.require_token(token).id, request)
        self._on_change()
        return j

    def get_scheduled_job_by_token(self, token: str):
        return self.jobs.get_by_token(token)

    def list_scheduled_jobs(self, criteria=None):
        return self.jobs.list(criteria)

    def delete_scheduled_job(self, token: str):
        j = self.jobs.delete(self.jobs.require_token(token).id)
        self._on_change()
        return j


class ScheduleManager(threading.Thread):
    """Fires due jobs: ``CommandInvocation`` -> invocation on an assignment; ``BatchCommandInvocation``
    -> a batch operation over a device group / device list."""

    def __init__(self, engine, tick_s: float = 1.0):
        super().__init__(daemon=True, name=f"scheduler-{engine.tenant.token}")
        self.engine, self.tick = engine, tick_s
        self._stop = threading.Event()
        self._next: dict[str, int] = {}
        self._fired: dict[str, int] = {}
        self.executions = []

    def reschedule(self):
        self._next.clear()

    def run(self):
        while not self._stop.wait(self.tick):
            try:
                self.run_due(now_ms())
            except Exception:
                self.engine.logger.exception("scheduler tick failed")

    def run_due(self, now: int) -> int:
        sm: ScheduleManagement = self.engine.management
        n = 0
        for job in sm.jobs.query(lambda j: j.job_state == ScheduledJobState.Active):
            sched = sm.schedules.get(job.schedule_id)
            if sched is None:
                continue
            due = self._next.get(job.id)
            if due is None:
                due = next_fire(sched, now, self._fired.get(job.id, 0))
                if due is None:
                    job.job_state = ScheduledJobState.Complete
                    sm.jobs.put(job)
                    continue
                self._next[job.id] = due
            if due <= now:
                self.execute(job)
                self._fired[job.id] = self._fired.get(job.id, 0) + 1
                nxt = next_fire(sched, now, self._fired[job.id])
                if nxt is None:
                    job.job_state = ScheduledJobState.Complete
                    sm.jobs.put(job)
                    self._next.pop(job.id, None)
                else:
                    self._next[job.id] = nxt
                n += 1
        return n

    def execute(self, job: ScheduledJob):
        t = self.engine.tenant.token
        cfg = job.job_configuration or {}
        if job.job_type == ScheduledJobType.CommandInvocation:
            dm = self.engine.ms.api("DeviceManagement", t)
            a = dm.get_device_assignment_by_token(cfg["assignmentToken"])
            cmd = dm.get_device_command_by_token(cfg["commandToken"])
            self.engine.ms.api("DeviceEventManagement", t).add_command_invocations(a.id, {
                "initiator": CommandInitiator.Scheduler.value, "initiatorId": job.token, "target": "Assignment",
                "targetId": a.id, "commandToken": cfg["commandToken"], "deviceCommandId": cmd.id if cmd else None,
                "parameterValues": cfg.get("parameterValues", {})})
        else:
            dm = self.engine.ms.api("DeviceManagement", t)
            ids = list(cfg.get("deviceIds", []))
            if cfg.get("groupToken"):
                g = dm.get_device_group_by_token(cfg["groupToken"])
                ids += dm.expand_group_devices(g.id, cfg.get("groupRoles"))
            self.engine.ms.api("BatchManagement", t).create_batch_command_invocation({
                "commandToken": cfg["commandToken"], "parameterValues": cfg.get("parameterValues", {}), "deviceIds": ids})
        self.executions.append((job.token, now_ms()))

    def stop(self):
        self._stop.set()


class ScheduleManagementTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ds = self.config.get("datastore", {"type": "memory"})
        self.scheduler = ScheduleManager(self, float(self.config.get("tickSeconds", 1.0)))
        self.management = ScheduleManagement(create_store(ds.get("type", "memory"),
                                                          **{k: v for k, v in ds.items() if k != "type"}),
                                             on_change=self.scheduler.reschedule)
        self.api = {"ScheduleManagement": self.management}

    def tenant_start(self, monitor):
        self.scheduler.start()

    def tenant_stop(self, monitor):
        self.scheduler.stop()

    def tenant_bootstrap(self, dataset_template, monitor):
        from .builders import ScheduleBuilder
        from .dataset_runner import run_initializers
        run_initializers(self, "scheduleManagement", dataset_template,
                         {"schedule_builder": ScheduleBuilder(self.management)})


class ScheduleManagementMicroservice(MultitenantMicroservice):
    identifier = "schedule-management"
    name = "Schedule Management"

    def service_names(self):
        return ["ScheduleManagement"]

    def create_tenant_engine(self, tenant):
        return ScheduleManagementTenantEngine(self, tenant)
