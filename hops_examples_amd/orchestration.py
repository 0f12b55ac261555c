"""A small DAG runner with the Hopsworks Airflow operators.

Reference: airflow/launch_jobs.py:67-130 (job-0 >> [job-1, job-2] >> sensor(job-2) >> job-3,
``wait_for_completion=False`` launches) and airflow/feature_group_validation.py:194-223
(launch the validation job, then ``HopsworksFeatureValidationResult`` fails the DAG when the
feature group's latest validation failed).  Airflow itself is not part of the image, so the
operators run on this runner: ``dag.run()`` executes tasks in dependency order, each task
starting as soon as all its upstream tasks succeeded; a failed task marks every downstream
task ``upstream_failed``.
"""
from __future__ import annotations

import time

from . import jobs


class TaskFailed(RuntimeError):
    pass


class BaseOperator:
    def __init__(self, dag: "DAG", task_id: str, **_):
        self.dag, self.task_id = dag, task_id
        self.upstream: list[BaseOperator] = []
        self.downstream: list[BaseOperator] = []
        dag._add(self)

    def __rshift__(self, other):
        others = other if isinstance(other, (list, tuple)) else [other]
        for o in others:
            self.downstream.append(o)
            o.upstream.append(self)
        return other

    def __rrshift__(self, other):  # [a, b] >> c
        for o in (other if isinstance(other, (list, tuple)) else [other]):
            o >> self
        return self

    def set_downstream(self, other):
        return self >> other

    def set_upstream(self, other):
        other >> self
        return self

    def execute(self, context: dict):
        raise NotImplementedError


class PythonOperator(BaseOperator):
    def __init__(self, dag, task_id, python_callable, op_kwargs=None, **kw):
        super().__init__(dag, task_id, **kw)
        self.fn, self.kw = python_callable, op_kwargs or {}

    def execute(self, context):
        return self.fn(**self.kw)


class HopsworksLaunchOperator(BaseOperator):
    def __init__(self, dag, task_id, job_name, project_name=None, job_arguments="", wait_for_completion=True,
                 poke_interval=0.2, timeout=None, **kw):
        super().__init__(dag, task_id, **kw)
        self.job_name, self.args, self.wait = job_name, job_arguments, wait_for_completion
        self.poke, self.timeout = poke_interval, timeout

    def execute(self, context):
        ex = jobs.start_job(self.job_name, self.args)
        if self.wait:
            s = jobs.wait_for_execution(self.job_name, ex["id"], self.timeout, self.poke)
            if s.get("finalStatus") != "SUCCEEDED":
                raise TaskFailed(f"job {self.job_name} execution {ex['id']} ended {s.get('finalStatus')}")
        return ex["id"]


class HopsworksJobSuccessSensor(BaseOperator):
    """Waits for the latest execution of ``job_name`` to finish; fails if it did not succeed."""

    def __init__(self, dag, task_id, job_name, project_name=None, poke_interval=0.2, timeout=None, **kw):
        super().__init__(dag, task_id, **kw)
        self.job_name, self.poke, self.timeout = job_name, poke_interval, timeout

    def execute(self, context):
        t0 = time.time()
        while True:
            ex = jobs.get_executions(self.job_name)
            if ex and ex[-1].get("state") in jobs.TERMINAL:
                if ex[-1].get("finalStatus") != "SUCCEEDED":
                    raise TaskFailed(f"job {self.job_name} ended {ex[-1].get('finalStatus')}")
                return ex[-1]["id"]
            if self.timeout is not None and time.time() - t0 > self.timeout:
                raise TaskFailed(f"sensor timed out waiting for {self.job_name}")
            time.sleep(self.poke)


class HopsworksFeatureValidationResult(BaseOperator):
    """Fails when the latest validation of the feature group has status FAILURE
    (or WARNING too, with ``fail_on_warning``)."""

    def __init__(self, dag, task_id, feature_group_name, feature_group_version=1, project_name=None,
                 ignore_result=False, fail_on_warning=False, **kw):
        super().__init__(dag, task_id, **kw)
        self.fg, self.version = feature_group_name, feature_group_version
        self.ignore, self.fail_on_warning = ignore_result, fail_on_warning

    def execute(self, context):
        from .featurestore import store as S

        fs = S.connection_quiet().get_feature_store()
        vals = fs.get_feature_group(self.fg, self.version).get_validations()
        if not vals:
            raise TaskFailed(f"feature group {self.fg} v{self.version} has no validations")
        last = vals[-1]
        status = last.status if hasattr(last, "status") else last.get("status")
        bad = ("FAILURE", "WARNING") if self.fail_on_warning else ("FAILURE",)
        if status in bad and not self.ignore:
            raise TaskFailed(f"feature group {self.fg} v{self.version} validation status {status}")
        return status


LaunchOperator, JobSuccessSensor, FeatureValidationResult = (HopsworksLaunchOperator, HopsworksJobSuccessSensor,
                                                             HopsworksFeatureValidationResult)


class DAG:
    def __init__(self, dag_id: str, default_args: dict | None = None, schedule_interval=None, **_):
        self.dag_id, self.default_args, self.schedule_interval = dag_id, default_args or {}, schedule_interval
        self.tasks: dict[str, BaseOperator] = {}

    def _add(self, t: BaseOperator):
        if t.task_id in self.tasks:
            raise ValueError(f"duplicate task_id {t.task_id}")
        self.tasks[t.task_id] = t

    def topological_order(self) -> list[BaseOperator]:
        indeg = {t.task_id: len(t.upstream) for t in self.tasks.values()}
        ready = [t for t in self.tasks.values() if indeg[t.task_id] == 0]
        order = []
        while ready:
            t = ready.pop(0)
            order.append(t)
            for d in t.downstream:
                indeg[d.task_id] -= 1
                if indeg[d.task_id] == 0:
                    ready.append(d)
        if len(order) != len(self.tasks):
            raise ValueError("DAG has a cycle")
        return order

    def run(self, raise_on_failure: bool = False) -> dict:
        """Execute once; returns {task_id: 'success' | 'failed' | 'upstream_failed'}."""
        state: dict[str, str] = {}
        errors = {}
        for t in self.topological_order():
            if any(state.get(u.task_id) != "success" for u in t.upstream):
                state[t.task_id] = "upstream_failed"
                continue
            try:
                t.execute({"dag": self, "task": t})
                state[t.task_id] = "success"
            except Exception as e:  # a failing task fails its downstream, not the runner
                state[t.task_id] = "failed"
                errors[t.task_id] = e
        if raise_on_failure and errors:
            k = next(iter(errors))
            raise TaskFailed(f"task {k} failed: {errors[k]}")
        self.errors = errors
        return state
