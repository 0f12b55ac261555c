"""Experiment API contracts on CPU: launch result dict +
log path, file-valued returns copied into the run dir, grid search best selection and trial
dirs, differential-evolution progress lines, mirrored with two gloo ranks."""
import json
import re
from pathlib import Path


def test_launch_result_contract(project_root):
    from hops_examples_amd import experiment

    def train():
        import os

        print("training…")
        open("summary.png", "wb").write(b"\x89PNG")
        return {"accuracy": 0.98, "train_summary": "summary.png", "logdir": os.environ["HOPSX_LOGDIR"]}

    d, res = experiment.launch(train, name="keras mnist", local_logdir=True, metric_key="accuracy")
    assert Path(d).parent.name == "Experiments" and re.match(r"application_\d+_\d+_\d+", Path(d).name)
    assert res["accuracy"] == 0.98
    assert res["log"].endswith("output.log") and not res["log"].startswith("/")
    assert "training…" in (project_root / res["log"]).read_text()
    assert (project_root / res["train_summary"]).read_bytes() == b"\x89PNG"
    meta = json.loads((Path(d) / "experiment.json").read_text())
    assert meta["status"] == "FINISHED" and meta["metric"] == 0.98


def test_launch_args_dict_and_failure(project_root):
    import pytest
    from hops_examples_amd import experiment
    from hops_examples_amd.experiment._runner import TrialError

    def train(lr, units):
        return lr * units

    d, res = experiment.launch(train, {"lr": [0.1, 0.2], "units": [10, 20]})
    assert res["metric"] == 0.2 * 20
    assert sorted(p.name for p in Path(d).iterdir() if p.is_dir()) == ["lr=0.1&units=10", "lr=0.2&units=20"]

    def boom():
        raise ValueError("bad hyperparameter")

    with pytest.raises(TrialError, match="bad hyperparameter"):
        experiment.launch(boom)


def test_grid_search(project_root, monkeypatch):
    from hops_examples_amd import experiment

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")

    def wrapper(learning_rate, dropout):
        return {"accuracy": 1.0 - abs(learning_rate - 0.0005) * 100 - dropout / 10}

    args = {"learning_rate": [0.001, 0.0005, 0.0001], "dropout": [0.45, 0.7]}
    d, params, metrics = experiment.grid_search(wrapper, args, direction="max", optimization_key="accuracy")
    assert params == {"learning_rate": 0.0005, "dropout": 0.45}
    assert Path(d).name == "learning_rate=0.0005&dropout=0.45" and Path(d).parent.name == "grid_search"
    assert abs(metrics["accuracy"] - (1 - 0.045)) < 1e-9
    summary = json.loads((Path(d).parent / "summary.json").read_text())
    assert len(summary) == 6


def test_differential_evolution_output(project_root, monkeypatch, capsys):
    from hops_examples_amd import experiment

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")

    def objective(kernel, pool, dropout):
        return -((kernel - 4) ** 2) - (pool - 3) ** 2 - dropout

    d, params, metrics = experiment.differential_evolution(
        objective, {"kernel": [2, 8], "pool": [2, 8], "dropout": [0.01, 0.99]}, direction="max", generations=3,
        population=5, seed=1)
    out = capsys.readouterr().out
    lines = [l for l in out.splitlines() if l.startswith("Generation")]
    assert len(lines) == 4
    m = re.match(r"Generation 3 \|\| average metric: (.+), best metric: (.+), best parameter combination: "
                 r"\['kernel=(\d+)', 'pool=(\d+)', 'dropout=([0-9.]+)'\]", lines[-1])
    assert m, lines[-1]
    assert "Finished Experiment \n" in out
    assert isinstance(params["kernel"], int) and isinstance(params["dropout"], float)
    assert Path(d).parent.name.startswith("generation.")
    assert metrics["metric"] == objective(**params)


def test_mirrored_two_gloo_ranks(project_root, monkeypatch):
    """experiment.mirrored spawns one worker per rank; ranks all-reduce over gloo on CPU."""
    from hops_examples_amd import experiment

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")

    def train():
        import torch
        import torch.distributed as dist

        from hops_examples_amd.parallel import dist as hdist

        rank, _, world = hdist.init(backend="gloo")
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t)
        hdist.barrier()
        return {"sum": t.item(), "world": world, "rank": rank}

    d, res = experiment.mirrored(train, name="mirrored", num_workers=2, metric_key="sum", timeout=120)
    assert res["sum"] == 3.0 and res["world"] == 2 and res["rank"] == 0
    assert res["log"].endswith("chief_0_output.log")
    assert (Path(d) / "worker_0_output.log").exists()
