"""lagom: the asynchronous trial driver (random/grid search + median early stopping,
or LOCO ablation)."""
from __future__ import annotations

import hashlib
import json
import os
import random
import socket
import statistics
import threading
import time
from pathlib import Path

from .. import hdfs
from ..experiment import _runner as R
from .reporter import EarlyStopException, Reporter
from .searchspace import Searchspace


def _trial_id(params: dict) -> str:
    return hashlib.sha1(json.dumps(params, sort_keys=True, default=str).encode()).hexdigest()[:16]


class _Driver:
    def __init__(self):
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(64)
        self.port = self.srv.getsockname()[1]
        self.hist: dict[str, list] = {}
        self.conns: dict[str, socket.socket] = {}
        self.lock = threading.Lock()
        self.stopped: set = set()
        self._alive = True
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        while self._alive:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._reader, args=(c,), daemon=True).start()

    def _reader(self, c):
        f = c.makefile("r")
        for line in f:
            try:
                m = json.loads(line)
            except ValueError:
                continue
            t = m.get("trial")
            with self.lock:
                if m["type"] == "REG":
                    self.conns[t] = c
                    self.hist.setdefault(t, [])
                elif m["type"] == "METRIC":
                    self.hist.setdefault(t, []).append((m["step"], m["value"]))

    def stop_trial(self, t):
        with self.lock:
            c = self.conns.get(t)
            self.stopped.add(t)
        if c is not None:
            try:
                c.sendall(b'{"type": "STOP"}\n')
            except OSError:
                pass

    def close(self):
        self._alive = False
        self.srv.close()


def _median_rule(driver: _Driver, running: list, finished: list, direction: str, es_min: int):
    """Stop running trials whose latest metric is worse than the median of the finished
    trials' metrics at the same step (maggy's median early-stopping policy)."""
    if len(finished) < es_min:
        return
    for t in running:
        h = driver.hist.get(t) or []
        if not h or t in driver.stopped:
            continue
        step, val = h[-1]
        ref = []
        for f in finished:
            fh = [v for s, v in driver.hist.get(f, []) if s <= step]
            if fh:
                ref.append(fh[-1])
        if len(ref) < es_min:
            continue
        med = statistics.median(ref)
        if (direction == "max" and val < med) or (direction == "min" and val > med):
            driver.stop_trial(t)


def _wrap(train_fn, params: dict, hb_interval: float):
    def _trial():
        rep = Reporter(hb_interval=hb_interval)
        try:
            res = train_fn(**params, reporter=rep)
        except EarlyStopException as e:
            res = e.metric
            rep.log("early stopped")
        metric = res.get("metric", next(iter(res.values()))) if isinstance(res, dict) else res
        rep.close(final=metric)
        return {"metric": metric, "early_stopped": rep.stop, "history": rep.history}

    return _trial


def lagom(train_fn, searchspace: Searchspace | None = None, optimizer: str = "randomsearch",
          direction: str = "max", num_trials: int = 1, name: str = "no-name", hb_interval: float = 1,
          es_policy: str = "median", es_interval: float = 300, es_min: int = 10, description: str = "",
          experiment_type: str = "optimization", ablation_study=None, ablator: str = "loco",
          seed: int | None = None, timeout: float | None = None):
    """Run an asynchronous search (``experiment_type='optimization'``) or an ablation study
    (``experiment_type='ablation'``).  Returns a summary dict (best/worst trial, average)."""
    direction = direction.lower()
    if experiment_type == "ablation":
        if ablation_study is None:
            raise ValueError("ablation experiments need ablation_study=")
        from .ablation import trial_generators

        trials = trial_generators(ablation_study, ablator)  # [(trial_name, kwargs-for-train_fn)]
        return _run_ablation(train_fn, trials, name, direction, timeout)
    if searchspace is None:
        raise ValueError("optimization experiments need a searchspace")
    rng = random.Random(seed)
    if optimizer.lower() == "gridsearch":
        configs = searchspace.grid()[:num_trials] if num_trials else searchspace.grid()
    elif optimizer.lower() in ("randomsearch", "random"):
        configs, seen = [], set()
        tries = 0
        while len(configs) < num_trials and tries < 100 * num_trials:
            c = searchspace.sample(rng)
            k = _trial_id(c)
            tries += 1
            if k not in seen:
                seen.add(k)
                configs.append(c)
    else:
        raise ValueError(f"unsupported optimizer {optimizer!r} (randomsearch | gridsearch)")

    app_id = R.next_app_id()
    root = Path(hdfs.project_path()) / "Experiments" / app_id
    root.mkdir(parents=True, exist_ok=True)
    R.write_meta(root, name=name, description=description, type="maggy_" + optimizer, app_id=app_id,
                 start=time.time(), status="RUNNING", searchspace=searchspace.to_dict(), direction=direction)
    driver = _Driver()
    ngpu = R.num_gpus()
    slots = ngpu if ngpu else max(1, min(4, (os.cpu_count() or 2) // 2))
    pending = list(configs)
    running: dict[str, tuple] = {}
    finished: list[str] = []
    results: dict[str, dict] = {}
    params_of: dict[str, dict] = {}
    free = list(range(slots))
    last_es = time.time()
    t0 = time.time()
    try:
        while pending or running:
            while pending and free:
                slot = free.pop(0)
                p = pending.pop(0)
                tid = _trial_id(p)
                params_of[tid] = p
                env = {"HOPSX_TRIAL_ID": tid, "HOPSX_MAGGY_HOST": "127.0.0.1", "HOPSX_MAGGY_PORT": driver.port,
                       "HOPSX_MAGGY_HB": hb_interval}
                w = R.spawn(_wrap(train_fn, p, hb_interval), {}, root / "trials" / tid, env=env,
                            gpu=slot if ngpu else None)
                running[tid] = (slot, w)
            done = [t for t, (_, w) in running.items() if w.proc.poll() is not None]
            for t in done:
                slot, w = running.pop(t)
                free.append(slot)
                try:
                    results[t] = R.collect(w, timeout)
                except Exception as e:
                    results[t] = {"metric": None, "error": str(e)[-500:]}
                finished.append(t)
            if time.time() - last_es >= es_interval and es_policy == "median":
                _median_rule(driver, list(running), [f for f in finished if results[f].get("metric") is not None],
                             direction, es_min)
                last_es = time.time()
            if not done:
                time.sleep(0.05)
    finally:
        driver.close()
    ok = {t: r for t, r in results.items() if r.get("metric") is not None}
    if not ok:
        raise R.TrialError("all trials failed: " + json.dumps(results, default=str)[:2000])
    key = (lambda t: ok[t]["metric"])
    best = max(ok, key=key) if direction == "max" else min(ok, key=key)
    worst = min(ok, key=key) if direction == "max" else max(ok, key=key)
    summary = {
        "best_id": best, "best_config": params_of[best], "best_hp": params_of[best], "best_val": ok[best]["metric"],
        "worst_id": worst, "worst_config": params_of[worst], "worst_val": ok[worst]["metric"],
        "avg": sum(r["metric"] for r in ok.values()) / len(ok), "metric_list": [ok[t]["metric"] for t in ok],
        "num_trials": len(results), "early_stopped": sum(1 for r in ok.values() if r.get("early_stopped")),
        "duration_s": time.time() - t0,
    }
    (root / "result.json").write_text(json.dumps({"summary": summary, "trials": {
        t: {"params": params_of[t], **{k: v for k, v in r.items() if k != "history"}} for t, r in results.items()}},
        indent=2, default=str))
    R.write_meta(root, status="FINISHED", end=time.time(), result=summary)
    print(f"Finished experiment. Best metric {summary['best_val']} with {summary['best_hp']} "
          f"({summary['early_stopped']} of {summary['num_trials']} trials early-stopped)")
    return summary


def _run_ablation(train_fn, trials, name, direction, timeout):
    app_id = R.next_app_id()
    root = Path(hdfs.project_path()) / "Experiments" / app_id
    root.mkdir(parents=True, exist_ok=True)
    R.write_meta(root, name=name, type="maggy_ablation", app_id=app_id, start=time.time(), status="RUNNING",
                 trials=[t for t, _ in trials])
    ngpu = R.num_gpus()
    slots = ngpu if ngpu else max(1, min(4, (os.cpu_count() or 2) // 2))
    from ..experiment import _TrialPool

    pool = _TrialPool(slots)
    specs = [(kw, root / "trials" / tname) for tname, kw in trials]

    def runner(**kw):
        res = train_fn(**kw)
        return res

    vals = pool.run(specs, runner, False, timeout)
    out = {}
    for (tname, _), v in zip(trials, vals):
        out[tname] = None if isinstance(v, Exception) else (v.get("metric") if isinstance(v, dict) else v)
    valid = {k: v for k, v in out.items() if v is not None}
    best = (max if direction == "max" else min)(valid, key=valid.get) if valid else None
    summary = {"results": out, "best_trial": best, "best_val": valid.get(best) if best else None,
               "base": out.get("base")}
    (root / "result.json").write_text(json.dumps(summary, indent=2, default=str))
    R.write_meta(root, status="FINISHED", end=time.time(), result=summary)
    return summary
