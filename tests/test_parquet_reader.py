"""Parquet -> device reader (io/parquet.py): values, column order, dtype conversion, row-group
sharding; CPU here, the pinned/side-stream path on the GPU box."""
import numpy as np
import pandas as pd
import pytest
import torch

from hops_examples_amd.io.parquet import ParquetDeviceReader, read_parquet_to_device


def _file(tmp_path, n=10000, rg=1024):
    rng = np.random.default_rng(0)
    df = pd.DataFrame({"a": rng.integers(-5, 5, n), "b": rng.normal(size=n),
                       "c": rng.random(n).astype(np.float32), "d": rng.integers(0, 2, n).astype(bool),
                       "e": rng.integers(0, 100, n).astype(np.int32)})
    p = tmp_path / "t.parquet"
    df.to_parquet(p, index=False, row_group_size=rg)
    return p, df


def _check(dev, tmp_path):
    p, df = _file(tmp_path)
    cols = ["e", "b", "a", "d", "c"]
    t = read_parquet_to_device(p, cols, device=dev)
    want = df[cols].to_numpy(dtype=np.float32)
    assert t.shape == want.shape and t.dtype == torch.float32
    np.testing.assert_array_equal(t.cpu().numpy(), want)
    # shards partition the row groups
    parts = [ParquetDeviceReader(p, cols, device=dev, shard=(3, i)).read().cpu().numpy() for i in range(3)]
    assert sum(len(x) for x in parts) == len(df)
    got = np.concatenate(parts)
    np.testing.assert_array_equal(np.sort(got[:, 1]), np.sort(want[:, 1]))


def test_parquet_reader_cpu(tmp_path):
    _check(torch.device("cpu"), tmp_path)


@pytest.mark.gpu
def test_parquet_reader_gpu(tmp_path):
    _check(torch.device("cuda", 0), tmp_path)


@pytest.mark.gpu
def test_cols_to_f32_all_dtypes():
    """columns.hip: every supported column dtype, a row stride wider than k, a partial last block."""
    from hops_examples_amd.ops import kernels as K

    dev = torch.device("cuda", 0)
    n = 1000 + 37
    g = torch.Generator().manual_seed(0)
    cols = [torch.randn(n, generator=g).to(torch.float64), torch.randn(n, generator=g),
            torch.randint(-2**40, 2**40, (n,), generator=g), torch.randint(-1000, 1000, (n,), generator=g).int(),
            torch.randint(-300, 300, (n,), generator=g).short(), torch.randint(-100, 100, (n,), generator=g).to(torch.int8),
            torch.randint(0, 255, (n,), generator=g).to(torch.uint8), torch.randn(n, generator=g).half()]
    out = torch.full((n, len(cols) + 3), -7.0, device=dev)
    K.cols_to_f32([c.to(dev) for c in cols], out[:, 1:1 + len(cols)])
    want = torch.stack([c.to(torch.float32) for c in cols], 1)
    torch.testing.assert_close(out[:, 1:1 + len(cols)].cpu(), want, rtol=0, atol=0)
    assert (out[:, 0] == -7).all() and (out[:, -2:] == -7).all()
