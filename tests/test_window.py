"""Range-window feature aggregates (featurestore.window; reference feature_engineering.ipynb:229-249)
against a brute-force pandas evaluation of Spark's rangeBetween semantics."""
import numpy as np
import pandas as pd
import pytest

from hops_examples_amd.featurestore.window import days, range_sums, with_range_sums


def _frame(n_days=200, seed=0):
    r = np.random.default_rng(seed)
    rows = []
    for s in (1, 2):
        for d in (1, 2, 3):
            dates = np.sort(r.choice(np.arange(n_days), n_days // 3, replace=False))
            for day in dates:
                rows.append((s, d, int(day) * 86400 + 1_600_000_000, float(r.normal(20000, 4000))))
    df = pd.DataFrame(rows, columns=["store", "dept", "ts", "weekly_sales"])
    return df.sample(frac=1.0, random_state=1).reset_index(drop=True)  # unsorted input


def _brute(df, keys, lo, hi):
    out = np.full(len(df), np.nan)
    for i, row in df.iterrows():
        m = np.ones(len(df), bool)
        for k in keys:
            m &= (df[k] == row[k]).to_numpy()
        m &= ((df.ts >= row.ts + lo) & (df.ts <= row.ts + hi)).to_numpy()
        if m.any():
            out[i] = df.weekly_sales[m].sum()
    return out


@pytest.mark.parametrize("keys", [["store", "dept"], ["store"]])
def test_range_sums_match_spark_semantics(keys):
    df = _frame()
    wins = [(days(-30), days(-1)), (days(-90), days(-1)), (0, 0), (days(-365), days(-1))]
    got, cnt = range_sums(df, keys, "ts", "weekly_sales", wins, device="cpu", with_count=True)
    for j, (lo, hi) in enumerate(wins):
        want = _brute(df, keys, lo, hi)
        np.testing.assert_allclose(got[:, j], want, rtol=1e-12, equal_nan=True)
        assert ((cnt[:, j] == 0) == np.isnan(want)).all()


def test_with_range_sums_fills_like_the_reference():
    df = _frame(60)
    out = with_range_sums(df, {"sales_last_month_store_dep": (days(-30), days(-1))}, ["store", "dept"], "ts",
                          "weekly_sales")
    first = out.sort_values("ts").groupby(["store", "dept"]).head(1)
    assert (first.sales_last_month_store_dep == 0.0).all()  # nothing before the first row -> null -> 0
    assert list(out.columns[:4]) == list(df.columns)


def _dp_rank(rank, world, port, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        df = _frame(seed=3)
        wins = [(days(-30), days(-1)), (days(-90), days(-1))]
        s, c = range_sums(df, ["store", "dept"], "ts", "weekly_sales", wins, device="cpu", with_count=True)
        q.put((rank, s, c))
    finally:
        dist.destroy_process_group()


def test_range_sums_data_parallel_gloo():
    """2 ranks each compute their partitions' windows and all-gather: every rank returns exactly the
    single-process result (feature engineering as a data-parallel job)."""
    import socket

    import torch.multiprocessing as mp

    df = _frame(seed=3)
    wins = [(days(-30), days(-1)), (days(-90), days(-1))]
    want, wcnt = range_sums(df, ["store", "dept"], "ts", "weekly_sales", wins, device="cpu", with_count=True,
                            process_group=False)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dp_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, s, c in res:
        np.testing.assert_array_equal(np.isnan(s), np.isnan(want))
        np.testing.assert_allclose(np.nan_to_num(s), np.nan_to_num(want), rtol=1e-12)
        np.testing.assert_array_equal(c, wcnt)
