"""``experiment`` — the notebook-facing experiment API of hops-util-py, re-built on
MI355X worker processes (one process per GPU, RCCL over xGMI).

Reference call sites:
  launch                 notebooks/ml/Experiment/Tensorflow/mnist.ipynb:228, …/PyTorch/mnist.ipynb:252
  mirrored               …/mirroredstrategy_mnist_example.ipynb:231, …/multiworkermirroredstrategy_mnist_example.ipynb:237
  collective_allreduce   prose only (…/Experiment/Tensorflow/mnist.ipynb:52)
  parameter_server       prose + jobs-client/spark/job_config.json:13
  grid_search            …/grid_search_fashion_mnist.ipynb:311
  differential_evolution …/PyTorch/differential_evolution/mnist.ipynb:230, …/evolutionary_search_mnist.ipynb:267
  random_search          (hops-util-py API; maggy-style async variant in hops_examples_amd.maggy)

Every call returns the reference's result contract:
``(project_path + 'Experiments/<id>[/…]', {**returned_metrics, 'log': 'Experiments/<id>/…/output.log'})``
"""
from __future__ import annotations

import itertools
import json
import os
import random
import time
from pathlib import Path

from .. import hdfs
from . import _runner as R

__all__ = ["launch", "mirrored", "collective_allreduce", "parameter_server", "grid_search",
           "differential_evolution", "random_search", "get_logdir"]

_INLINE = os.environ.get("HOPSX_INLINE", "0") == "1"


def _exp_dir(app_id: str) -> Path:
    return Path(hdfs.project_path()) / "Experiments" / app_id


def _uri(p: Path) -> str:
    return str(p)


def get_logdir() -> str:
    return os.environ.get("HOPSX_LOGDIR", os.getcwd())


def _run_one(fn, kwargs, run_dir: Path, log_name="output.log", gpu=None, env=None, local_logdir=False,
             timeout=None):
    if _INLINE:
        return R.run_inline(fn, kwargs, run_dir, log_name)
    w = R.spawn(fn, kwargs, run_dir, log_name, env=env, gpu=gpu, local_logdir=local_logdir)
    return R.collect(w, timeout)


# ------------------------------------------------------------------- launch
def launch(train_fn, args_dict: dict | None = None, name: str = "no-name", local_logdir: bool = False,
           description: str | None = None, metric_key: str | None = None, gpu: int | None = None,
           timeout: float | None = None):
    """Run ``train_fn`` once (or once per index of ``args_dict`` lists) in a worker process.

    Returns ``(experiment_dir, result_dict)``.
    """
    app_id = R.next_app_id()
    d = _exp_dir(app_id)
    d.mkdir(parents=True, exist_ok=True)
    t0 = time.time()
    R.write_meta(d, name=name, description=description, type="launch", app_id=app_id, start=t0,
                 status="RUNNING", metric_key=metric_key)
    runs = []
    if args_dict:
        n = len(next(iter(args_dict.values())))
        for i in range(n):
            runs.append({k: v[i] for k, v in args_dict.items()})
    else:
        runs.append({})
    results = []
    try:
        for i, kw in enumerate(runs):
            rd = d if len(runs) == 1 else d / "&".join(f"{k}={v}" for k, v in kw.items())
            val = _run_one(train_fn, kw, rd, gpu=gpu, local_logdir=local_logdir, timeout=timeout)
            results.append(R.finalize_result(val, rd))
    except Exception:
        R.write_meta(d, status="FAILED", end=time.time())
        raise
    res = results[0] if len(results) == 1 else results[-1]
    if metric_key and isinstance(res, dict):
        R.write_meta(d, metric=res.get(metric_key))
    R.write_meta(d, status="FINISHED", end=time.time(), duration_s=time.time() - t0, result=res)
    return _uri(d), res


# ------------------------------------------------------ distributed training
def _distributed(train_fn, name, local_logdir, description, metric_key, num_workers, mode, timeout, extra_env=None,
                 heartbeat_timeout=None, max_restarts=0):
    """One worker process per GPU; the first failing rank tears the job down (runtime.health).
    ``max_restarts`` > 0 relaunches the whole gang after a failure with HOPSX_RESTART=<attempt>
    in the environment; a train_fn that checkpoints into ``tensorboard.logdir()``
    (hops_examples_amd.checkpoint) resumes from its latest checkpoint."""
    app_id = R.next_app_id()
    d = _exp_dir(app_id)
    d.mkdir(parents=True, exist_ok=True)
    ngpu = R.num_gpus()
    if num_workers is None:
        num_workers = max(1, ngpu)
    t0 = time.time()
    R.write_meta(d, name=name, description=description, type=mode, app_id=app_id, start=t0, status="RUNNING",
                 num_workers=num_workers)
    attempt = 0
    while True:
        port = R.free_port()
        workers = []
        for rank in range(num_workers):
            env = {"RANK": rank, "LOCAL_RANK": rank if ngpu else 0, "WORLD_SIZE": num_workers,
                   "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port, "HOPSX_DP_MODE": mode,
                   "HOPSX_RESTART": attempt}
            if extra_env:
                env.update(extra_env)
            log = "chief_0_output.log" if rank == 0 else f"worker_{rank - 1}_output.log"
            # every rank sees all GPUs and pins itself to cuda:LOCAL_RANK (RCCL needs peer visibility)
            workers.append(R.spawn(train_fn, {}, d, log, env=env, gpu=None, local_logdir=local_logdir and rank == 0))
        try:
            values = R.wait_all(workers, timeout=timeout, heartbeat_timeout=heartbeat_timeout)
            break
        except Exception as e:  # first failure aborts the gang
            if attempt >= max_restarts:
                R.write_meta(d, status="FAILED", end=time.time(), attempts=attempt + 1, error=str(e)[:2000])
                raise
            attempt += 1
            R.write_meta(d, status="RESTARTING", attempts=attempt, last_error=str(e)[:2000])
    res = R.finalize_result(values[0], d, "chief_0_output.log")
    if metric_key and isinstance(res, dict):
        R.write_meta(d, metric=res.get(metric_key))
    R.write_meta(d, status="FINISHED", end=time.time(), duration_s=time.time() - t0, result=res,
                 attempts=attempt + 1)
    return _uri(d), res


def mirrored(train_fn, name: str = "no-name", local_logdir: bool = False, description: str | None = None,
             evaluator: bool = False, metric_key: str | None = None, num_workers: int | None = None,
             timeout: float | None = None, heartbeat_timeout: float | None = None, max_restarts: int = 0):
    """Synchronous data parallel training: one worker process per GPU of this node.

    Inside ``train_fn`` the process group is already initialised (RCCL); wrap the
    model in ``hops_examples_amd.parallel.DataParallel`` (bucketed all-reduce) —
    the counterpart of building the Keras model under ``strategy.scope()``.
    ``heartbeat_timeout``: tear the job down when a rank stops making progress;
    ``max_restarts``: relaunch after a failure (resume via hops_examples_amd.checkpoint).
    """
    return _distributed(train_fn, name, local_logdir, description, metric_key, num_workers, "mirrored", timeout,
                        heartbeat_timeout=heartbeat_timeout, max_restarts=max_restarts)


def collective_allreduce(train_fn, name: str = "no-name", local_logdir: bool = False,
                         description: str | None = None, evaluator: bool = False, metric_key: str | None = None,
                         num_workers: int | None = None, timeout: float | None = None,
                         heartbeat_timeout: float | None = None, max_restarts: int = 0):
    """Multi-worker collective all-reduce (TF CollectiveAllReduceStrategy / MultiWorkerMirrored).
    Same engine as :func:`mirrored`; multi-node rendezvous comes from MASTER_ADDR/PORT."""
    return _distributed(train_fn, name, local_logdir, description, metric_key, num_workers, "collective_allreduce",
                        timeout, heartbeat_timeout=heartbeat_timeout, max_restarts=max_restarts)


def parameter_server(train_fn, name: str = "no-name", local_logdir: bool = False, description: str | None = None,
                     evaluator: bool = False, metric_key: str | None = None, num_workers: int | None = None,
                     num_ps: int | None = None, timeout: float | None = None):
    """Parameter-server training: parameters are sharded over ``num_ps`` shard owners,
    gradients are reduce-scattered to the owners, owners apply the optimizer and the
    updated shards are all-gathered (``hops_examples_amd.parallel.ps.ParameterServer``)."""
    from .. import config

    nps = num_ps if num_ps is not None else config.get().num_ps
    return _distributed(train_fn, name, local_logdir, description, metric_key, num_workers, "parameter_server",
                        timeout, extra_env={"HOPSX_NUM_PS": nps})


# --------------------------------------------------------------- HPO: common
def _metric_of(value, key):
    if isinstance(value, dict):
        if key in value:
            return value[key]
        if "metric" in value:
            return value["metric"]
        raise KeyError(f"optimization_key {key!r} not in returned dict {list(value)}")
    return value


def _param_dir(kw: dict) -> str:
    return "&".join(f"{k}={v}" for k, v in kw.items())


class _TrialPool:
    """Runs trials in parallel, one per GPU (or per CPU slot on a GPU-less host)."""

    def __init__(self, slots: int | None = None):
        ngpu = R.num_gpus()
        self.gpus = list(range(ngpu)) if ngpu else []
        self.slots = slots or (len(self.gpus) if self.gpus else max(1, min(4, (os.cpu_count() or 2) // 2)))

    def run(self, trials: list[tuple[dict, Path]], fn, local_logdir=False, timeout=None):
        """trials: [(kwargs, run_dir)] -> list of (value | Exception)."""
        if _INLINE:
            out = []
            for kw, rd in trials:
                try:
                    out.append(R.run_inline(fn, kw, rd))
                except Exception as e:
                    out.append(e)
            return out
        results: list = [None] * len(trials)
        pending = list(enumerate(trials))
        running: dict = {}
        free = list(range(self.slots))
        while pending or running:
            while pending and free:
                slot = free.pop(0)
                i, (kw, rd) = pending.pop(0)
                gpu = self.gpus[slot % len(self.gpus)] if self.gpus else None
                running[i] = (slot, R.spawn(fn, kw, rd, gpu=gpu, local_logdir=local_logdir))
            done = [i for i, (_, w) in running.items() if w.proc.poll() is not None]
            if not done:
                time.sleep(0.05)
                continue
            for i in done:
                slot, w = running.pop(i)
                try:
                    results[i] = R.collect(w, timeout)
                except Exception as e:
                    results[i] = e
                free.append(slot)
        return results


def _better(a, b, direction):
    if b is None:
        return True
    return a > b if direction == "max" else a < b


# -------------------------------------------------------------- grid search
def grid_search(train_fn, args_dict: dict, direction: str = "max", optimization_key: str = "metric",
                name: str = "no-name", local_logdir: bool = False, description: str | None = None,
                timeout: float | None = None):
    """Cartesian product of ``args_dict``; one trial per combination, in parallel, one per GPU.

    Returns ``(best_trial_dir, best_params, best_metrics)``.
    """
    direction = direction.lower()
    keys = list(args_dict)
    combos = [dict(zip(keys, vals)) for vals in itertools.product(*[args_dict[k] for k in keys])]
    app_id = R.next_app_id()
    d = _exp_dir(app_id) / "grid_search"
    d.mkdir(parents=True, exist_ok=True)
    R.write_meta(d.parent, name=name, description=description, type="grid_search", app_id=app_id,
                 start=time.time(), status="RUNNING", optimization_key=optimization_key, direction=direction)
    trials = [(kw, d / _param_dir(kw)) for kw in combos]
    vals = _TrialPool().run(trials, train_fn, local_logdir, timeout)
    best, summary = None, []
    for (kw, rd), v in zip(trials, vals):
        if isinstance(v, Exception):
            summary.append({"params": kw, "error": str(v)[-500:]})
            continue
        m = _metric_of(v, optimization_key)
        res = R.finalize_result(v, rd)
        summary.append({"params": kw, "metric": m, "result": res})
        if m is not None and _better(m, None if best is None else best[0], direction):
            best = (m, kw, rd, res)
    (d / "summary.json").write_text(json.dumps(summary, indent=2, default=str))
    if best is None:
        R.write_meta(d.parent, status="FAILED")
        raise R.TrialError("all grid-search trials failed: " + json.dumps(summary, default=str)[:2000])
    R.write_meta(d.parent, status="FINISHED", end=time.time(), best_params=best[1], best_metric=best[0])
    print("Finished Experiment \n")
    return _uri(best[2]), best[1], best[3]


# --------------------------------------------------------- random search
def random_search(train_fn, boundary_dict: dict, direction: str = "max", samples: int = 10,
                  optimization_key: str = "metric", name: str = "no-name", local_logdir: bool = False,
                  description: str | None = None, seed: int | None = None, timeout: float | None = None):
    """Sample ``samples`` points uniformly inside ``{name: [low, high]}`` (ints stay ints)."""
    rng = random.Random(seed)
    combos = [{k: _sample(rng, lo, hi) for k, (lo, hi) in boundary_dict.items()} for _ in range(samples)]
    return _run_points(train_fn, combos, "random_search", direction, optimization_key, name, local_logdir,
                       description, timeout)


def _sample(rng, lo, hi):
    if isinstance(lo, int) and isinstance(hi, int):
        return rng.randint(lo, hi)
    return rng.uniform(float(lo), float(hi))


def _run_points(train_fn, combos, kind, direction, optimization_key, name, local_logdir, description, timeout):
    app_id = R.next_app_id()
    d = _exp_dir(app_id) / kind
    d.mkdir(parents=True, exist_ok=True)
    R.write_meta(d.parent, name=name, description=description, type=kind, app_id=app_id, start=time.time(),
                 status="RUNNING")
    trials = [(kw, d / _param_dir(kw)) for kw in combos]
    vals = _TrialPool().run(trials, train_fn, local_logdir, timeout)
    best = None
    for (kw, rd), v in zip(trials, vals):
        if isinstance(v, Exception):
            continue
        m = _metric_of(v, optimization_key)
        if m is not None and _better(m, None if best is None else best[0], direction):
            best = (m, kw, rd, R.finalize_result(v, rd))
    if best is None:
        raise R.TrialError(f"all {kind} trials failed")
    R.write_meta(d.parent, status="FINISHED", end=time.time(), best_params=best[1], best_metric=best[0])
    return _uri(best[2]), best[1], best[3]


# --------------------------------------------------- differential evolution
def differential_evolution(objective_function, boundary_dict: dict, direction: str = "max", generations: int = 4,
                           population: int = 6, mutation: float = 0.5, crossover: float = 0.7,
                           cleanup_generations: bool = False, name: str = "no-name", local_logdir: bool = False,
                           description: str | None = None, optimization_key: str = "metric",
                           seed: int | None = None, timeout: float | None = None):
    """DE/rand/1/bin over ``{name: [low, high]}`` bounds (int bounds -> int params).

    Prints, per generation, the reference's progress line
    ``Generation g || average metric: …, best metric: …, best parameter combination: ['k=v', …]``
    and returns ``(best_trial_dir, best_params, best_metrics)``; trial dirs are
    ``Experiments/<id>/generation.<g>/<k=v&…>`` (…/evolutionary_search_mnist.ipynb:248-258).
    """
    direction = direction.lower()
    rng = random.Random(seed)
    keys = list(boundary_dict)
    bounds = [boundary_dict[k] for k in keys]
    is_int = [isinstance(lo, int) and isinstance(hi, int) for lo, hi in bounds]
    population = max(4, population)

    def clip(v, i):
        lo, hi = bounds[i]
        v = min(max(v, lo), hi)
        return int(round(v)) if is_int[i] else float(v)

    def to_kw(vec):
        return {k: clip(v, i) for i, (k, v) in enumerate(zip(keys, vec))}

    app_id = R.next_app_id()
    root = _exp_dir(app_id)
    root.mkdir(parents=True, exist_ok=True)
    R.write_meta(root, name=name, description=description, type="differential_evolution", app_id=app_id,
                 start=time.time(), status="RUNNING", generations=generations, population=population)
    pool = _TrialPool()
    cache: dict = {}

    def evaluate(gen: int, vecs):
        todo, dirs = [], []
        for vec in vecs:
            kw = to_kw(vec)
            key = tuple(kw.items())
            rd = root / f"generation.{gen}" / _param_dir(kw)
            dirs.append((kw, key, rd))
            if key not in cache:
                todo.append((kw, rd))
                cache[key] = None
        vals = pool.run(todo, objective_function, local_logdir, timeout)
        for (kw, rd), v in zip(todo, vals):
            key = tuple(kw.items())
            if isinstance(v, Exception):
                cache[key] = (None, rd, {"error": str(v)[-300:]})
            else:
                cache[key] = (_metric_of(v, optimization_key), rd, R.finalize_result(v, rd))
        return [cache[k] for _, k, _ in dirs]

    def fitness(m):
        if m is None:
            return float("-inf") if direction == "max" else float("inf")
        return m

    pop = [[(_sample(rng, lo, hi)) for lo, hi in bounds] for _ in range(population)]
    scores = evaluate(0, pop)
    best_i = None

    def report(g, scores):
        nonlocal best_i
        valid = [s[0] for s in scores if s[0] is not None]
        avg = sum(valid) / len(valid) if valid else float("nan")
        best_i = max(range(len(scores)), key=lambda i: fitness(scores[i][0])) if direction == "max" else \
            min(range(len(scores)), key=lambda i: fitness(scores[i][0]))
        kw = to_kw(pop[best_i])
        print(f"Generation {g} || average metric: {avg}, best metric: {scores[best_i][0]}, "
              f"best parameter combination: {[f'{k}={v}' for k, v in kw.items()]}\n", flush=True)

    report(0, scores)
    for g in range(1, generations + 1):
        trial_vecs = []
        for i in range(population):
            a, b, c = rng.sample([j for j in range(population) if j != i], 3)
            jr = rng.randrange(len(keys))
            vec = []
            for j in range(len(keys)):
                if rng.random() < crossover or j == jr:
                    vec.append(pop[a][j] + mutation * (pop[b][j] - pop[c][j]))
                else:
                    vec.append(pop[i][j])
            trial_vecs.append([clip(v, j) for j, v in enumerate(vec)])
        tscores = evaluate(g, trial_vecs)
        for i in range(population):
            if direction == "max" and fitness(tscores[i][0]) >= fitness(scores[i][0]) or \
                    direction == "min" and fitness(tscores[i][0]) <= fitness(scores[i][0]):
                pop[i], scores[i] = trial_vecs[i], tscores[i]
        report(g, scores)
        if cleanup_generations and g > 1:
            import shutil

            shutil.rmtree(root / f"generation.{g - 1}", ignore_errors=True)
    print("Finished Experiment \n")
    m, rd, res = scores[best_i]
    best_kw = to_kw(pop[best_i])
    R.write_meta(root, status="FINISHED", end=time.time(), best_params=best_kw, best_metric=m)
    return _uri(rd), best_kw, res
