"""Profiling, health checks and metrics on CPU; the HIP non-finite
reduction itself is checked in tests/test_kernels_v2_gpu.py."""
import json

import pytest
import torch


def test_step_profiler_window_writes_trace(tmp_path):
    from hops_examples_amd import profiler

    x = torch.randn(64, 64)
    with profiler.profile("2,3", logdir=str(tmp_path), run_name="r") as p:
        for _ in range(5):
            (x @ x).sum()
            p.step()
    assert p.trace_path is not None and p.trace_path.exists()
    assert p.trace_path.parent == tmp_path / "plugins" / "profile" / "r"
    data = json.loads(p.trace_path.read_text())
    assert any("mm" in e.get("name", "") for e in data["traceEvents"])
    assert p.summary_path.exists()


def test_profile_batch_parsing():
    from hops_examples_amd.profiler import _parse_window

    assert _parse_window("5,10") == (5, 10)
    assert _parse_window(7) == (7, 7)
    assert _parse_window(0) is None
    with pytest.raises(ValueError):
        _parse_window("10,5")


def test_rocprof_command_shapes():
    from hops_examples_amd.profiler import rocprof_command

    c = rocprof_command("python3 bench.py --steps 5", "out")
    assert c.startswith("rocprofv3 --kernel-trace --stats -d out") and c.endswith("-- python3 bench.py --steps 5")
    c = rocprof_command(["python3", "x.py"], "o2", pmc=["SQ_WAVES", "SQ_INSTS_VALU"])
    assert "--pmc SQ_WAVES SQ_INSTS_VALU" in c and "--kernel-trace" not in c and "--sys-trace" not in c


def test_summarize_rocprof(tmp_path):
    from hops_examples_amd.profiler import summarize_rocprof

    p = tmp_path / "s.csv"
    p.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage"\n"a",2,4000,2000,40\n"b",1,6000,6000,60\n')
    rows = summarize_rocprof(p)
    assert [r["name"] for r in rows] == ["b", "a"] and rows[1]["avg_us"] == 2.0


def test_health_check_flags_nonfinite():
    from hops_examples_amd import profiler
    from hops_examples_amd.runtime.arena import ParamArena

    m = torch.nn.Linear(4, 3)
    ParamArena.from_module(m)
    hc = profiler.HealthCheck(m, every=1)
    assert hc.check(1)["grads"] == {"nan": 0, "inf": 0}
    m._hx_arena.grad[3] = float("nan")
    m._hx_arena.grad[5] = float("inf")
    with pytest.raises(profiler.NonFiniteError, match="1 NaN, 1 Inf"):
        hc.check(2)
    assert profiler.nonfinite(torch.tensor([1.0, float("nan"), float("-inf")])) == (1, 1)


def test_metrics_registry_sinks(tmp_path):
    from hops_examples_amd import metrics
    from hops_examples_amd.tensorboard import read_scalars

    r = metrics.Registry(logdir=str(tmp_path), rank=0)
    r.inc("steps", 3)
    r.set("images_per_sec", 1234.5)
    with r.timer("step"):
        sum(range(1000))
    snap = r.flush(step=7, to_tensorboard=True)
    assert snap["counters"]["steps"] == 3 and snap["timers"]["step"]["count"] == 1
    r2 = metrics.Registry(logdir=str(tmp_path), rank=1)
    r2.inc("steps", 1)
    r2.flush(step=7)
    recs = metrics.merge_jsonl(tmp_path)
    assert [x["rank"] for x in recs] == [0, 1]
    txt = r.prometheus_text()
    assert 'hopsx_images_per_sec{rank="0"} 1234.5' in txt and "hopsx_step_seconds_count" in txt
    sc = read_scalars(str(tmp_path / "metrics_rank0"))
    assert any("images_per_sec" in k for k in sc)
