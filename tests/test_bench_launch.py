"""bench.py / benchmarks/run.py launch their own ranks (parallel/launch.py).

The driver may run ``python bench.py --gpus N`` without torchrun: the script must then start N
ranks itself (never a silent 1-GPU number), refuse when fewer than N GPUs are visible unless
``--rehearse``, and stop every rank when one fails.  CPU: gloo ranks, no GPU.
"""
import json
import os
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        e.pop(k, None)
    e["HIP_VISIBLE_DEVICES"] = e["CUDA_VISIBLE_DEVICES"] = ""  # CPU even on a GPU box
    return e


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--rehearse", "--steps", "3", "--warmup", "1",
                        "--no-taxi"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)  # rank 0 only prints
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 64
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["replicas_identical"] is True
    assert [x["rank"] for x in rec["config"]["ranks"]] == [0, 1]
    assert all(x["world"] == 2 for x in rec["config"]["ranks"])
    assert rec["dtype"] == "fp32" and rec["config"]["hipgraph"] is False  # honest about the CPU run


def test_bench_refuses_more_ranks_than_gpus():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-taxi"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "refusing" in r.stderr and not r.stdout.strip()


def test_benchmarks_run_self_launches(tmp_path):
    r = subprocess.run([sys.executable, "benchmarks/run.py", "mnist_mirrored", "--gpus", "2", "--rehearse",
                        "--steps", "2", "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"


def test_launch_failing_rank_stops_the_others(tmp_path):
    sys.path.insert(0, ROOT)
    from hops_examples_amd.parallel import launch

    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)  # rank 0 'blocked in a collective'
    """))
    env_backup = {k: os.environ.pop(k) for k in ("RANK", "WORLD_SIZE") if k in os.environ}
    try:
        t0 = time.time()
        rc = launch.launch(2, [str(script)], rehearse=True)
        assert rc == 3
        assert time.time() - t0 < 60
    finally:
        os.environ.update(env_backup)


def test_cifar_benchmark_runs_through_collective_allreduce(tmp_path):
    env = _env()
    env["HOPSX_PROJECT_ROOT"] = str(tmp_path / "proj")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "run.py"), "cifar_resnet", "--gpus", "2",
                        "--rehearse", "--steps", "1", "--warmup", "1", "--batch", "4"], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["launcher"] == "experiment.collective_allreduce"
    assert rec["log"].endswith("chief_0_output.log") and rec["replicas_identical"] is True
    assert os.path.isdir(rec["experiment_dir"])


def test_titanic_td_benchmark_four_ranks_row_group_sharded(tmp_path):
    """BASELINE config 4 at 4 ranks (gloo rehearsal): the Titanic TD is written once as Parquet with
    64k-row row groups and every rank of experiment.mirrored reads only its row groups."""
    env = _env()
    env["HOPSX_PROJECT_ROOT"] = str(tmp_path / "proj")
    env["TMPDIR"] = str(tmp_path)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "run.py"), "titanic", "--gpus", "4",
                        "--rehearse", "--steps", "2", "--warmup", "1", "--rows", "262144"], cwd=str(tmp_path),
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 4 and rec["config"]["launcher"] == "experiment.mirrored"
    assert rec["shard_mode"] == "row_groups" and rec["rows_per_rank"] == 65536
    assert [x["rows"] for x in rec["config"]["ranks"]] == [65536] * 4
    assert rec["replicas_identical"] is True


def test_bench_eight_ranks_rehearsal():
    """World size 8 (BASELINE configs 2 and 5 run on 8 GPUs): eight gloo ranks on the CPU."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--rehearse", "--steps", "2", "--warmup", "1",
                        "--no-taxi"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 8 and rec["config"]["global_batch"] == 256 and rec["config"]["parallelism"] == "dp8"
    assert rec["replicas_identical"] is True
    assert [x["rank"] for x in rec["config"]["ranks"]] == list(range(8))


def test_cifar_resnet_eight_workers_rehearsal(tmp_path):
    """BASELINE config 5 at 8 workers through experiment.collective_allreduce (gloo rehearsal)."""
    env = _env()
    env["HOPSX_PROJECT_ROOT"] = str(tmp_path / "proj")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "run.py"), "cifar_resnet", "--gpus", "8",
                        "--rehearse", "--depth", "20", "--batch", "4", "--steps", "1", "--warmup", "1"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 8 and rec["replicas_identical"] is True
