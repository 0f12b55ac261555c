"""The native Parquet decoder (csrc/io/parquet_core.h via _hopsx_io.ParquetFile) against pyarrow on
every layout it covers — codecs NONE / SNAPPY, dictionary on / off, data pages v1 / v2, nulls in
every physical type — and the reader's use of it (io/parquet.py), including the Arrow fallback for
columns outside its scope."""
import itertools

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest
import torch

from hops_examples_amd import _hopsx_io as io
from hops_examples_amd.io.parquet import ParquetDeviceReader

W = {"i32": 4, "i64": 8, "f32": 4, "f64": 8, "f64n": 8, "b": 1, "bn": 1, "i64n": 8, "cat": 8}


def _table(n=20000, seed=0):
    rng = np.random.default_rng(seed)
    return pa.table({"i32": pa.array(rng.integers(-1000, 1000, n).astype(np.int32)),
                     "i64": pa.array(rng.integers(-2**40, 2**40, n)),
                     "f32": pa.array(rng.random(n).astype(np.float32)),
                     "f64": pa.array(np.where(rng.random(n) < 0.1, np.nan, rng.random(n))),
                     "f64n": pa.array(rng.random(n), mask=rng.random(n) < 0.2),
                     "b": pa.array(rng.random(n) < 0.5), "bn": pa.array(rng.random(n) < 0.5, mask=rng.random(n) < 0.1),
                     "i64n": pa.array(rng.integers(0, 5, n), mask=rng.random(n) < 0.3),
                     "cat": pa.array(rng.integers(0, 7, n).astype(np.int64))})


@pytest.mark.parametrize("comp,dic,dpv", list(itertools.product(["NONE", "SNAPPY"], [False, True], ["1.0", "2.0"])))
def test_native_decode_matches_arrow(tmp_path, comp, dic, dpv):
    tbl = _table()
    path = str(tmp_path / "t.parquet")
    pq.write_table(tbl, path, compression=comp, use_dictionary=dic, data_page_version=dpv, row_group_size=6000)
    f = io.ParquetFile(path)
    md = f.meta()
    names = [c[0] for c in md["columns"]]
    assert names == list(W) and md["num_rows"] == 20000 and len(md["row_groups"]) == 4
    ref = pq.ParquetFile(path)
    for rgi, (rows, _) in enumerate(md["row_groups"]):
        offs, o = [], 0
        for c in names:
            offs.append(o)
            o += -(-rows * W[c] // 256) * 256
        buf = torch.zeros(o, dtype=torch.uint8)
        f.decode(rgi, list(range(len(names))), buf.data_ptr(), offs)
        t = ref.read_row_group(rgi)
        for c, off in zip(names, offs):
            a = t.column(c).combine_chunks()
            if a.null_count:  # the reader's null rule: NaN for floating columns, 0 / False otherwise
                a = a.fill_null(float("nan") if pa.types.is_floating(a.type) else
                                (False if pa.types.is_boolean(a.type) else 0))
            v = a.to_numpy(zero_copy_only=False)
            v = v.view(np.uint8) if v.dtype == np.bool_ else v
            got = buf[off:off + rows * W[c]].numpy().view(v.dtype)
            assert np.array_equal(got, v, equal_nan=True), (c, rgi)


def test_native_rejects_malformed_and_out_of_scope(tmp_path):
    p = tmp_path / "bad.parquet"
    p.write_bytes(b"PAR1" + b"\0" * 40 + b"PAR1")
    with pytest.raises(Exception):
        io.ParquetFile(str(p))
    s = tmp_path / "s.parquet"
    pq.write_table(pa.table({"name": ["a", "b"], "x": [1.0, 2.0]}), s)
    f = io.ParquetFile(str(s))
    buf = torch.zeros(512, dtype=torch.uint8)
    with pytest.raises(io.ParquetUnsupported):
        f.decode(0, [0], buf.data_ptr(), [0])  # a string column: the reader falls back to Arrow


def test_reader_uses_native_and_falls_back(tmp_path):
    tbl = _table(5000)
    p = str(tmp_path / "n.parquet")
    pq.write_table(tbl, p, row_group_size=1000)
    cols = ["f64n", "i32", "bn", "cat"]
    r = ParquetDeviceReader(p, cols, device="cpu")
    assert p in r.native  # natively decodable
    got = r.read()
    assert r.bytes_read > 0
    want = tbl.select(cols).to_pandas().astype(np.float32).fillna(np.nan).to_numpy()
    want[np.isnan(want[:, 2]), 2] = 0  # null booleans -> 0
    np.testing.assert_array_equal(got.numpy(), np.nan_to_num(want, nan=np.nan))
    # a file with a string column among the requested ones -> Arrow path
    s = str(tmp_path / "s.parquet")
    pq.write_table(pa.table({"x": np.arange(10.0), "y": [str(i) for i in range(10)]}), s)
    r2 = ParquetDeviceReader(s, ["x"], device="cpu")
    assert s in r2.native  # only numeric columns requested: native
    np.testing.assert_array_equal(r2.read().numpy()[:, 0], np.arange(10.0, dtype=np.float32))


def test_annotated_columns_take_the_arrow_path(tmp_path):
    """DECIMAL (INT32/INT64 physical, scaled), unsigned, DATE and TIMESTAMP columns carry raw values that
    are not the column's values: the native plan refuses them and Arrow converts (no unscaled decimals,
    no negative uint32); signed small ints (INT_8 / INT_16 annotations) stay native."""
    import decimal

    n = 64
    rng = np.random.default_rng(1)
    dec = [decimal.Decimal(int(v)).scaleb(-2) for v in rng.integers(-10**6, 10**6, n)]
    tbl = pa.table({"d": pa.array(dec, type=pa.decimal128(9, 2)),
                    "u": pa.array(rng.integers(2**31, 2**32 - 1, n, dtype=np.uint32)),
                    "day": pa.array(rng.integers(0, 20000, n).astype("datetime64[D]").astype("datetime64[D]")),
                    "ts": pa.array(rng.integers(0, 10**9, n).astype("datetime64[s]")),
                    "i8": pa.array(rng.integers(-100, 100, n).astype(np.int8)),
                    "x": pa.array(rng.random(n))})
    p = str(tmp_path / "a.parquet")
    pq.write_table(tbl, p, store_decimal_as_integer=True)
    f = io.ParquetFile(p)
    plain = {c[0]: c[3] for c in f.meta()["columns"]}
    assert plain == {"d": False, "u": False, "day": False, "ts": False, "i8": True, "x": True}
    r = ParquetDeviceReader(p, ["i8", "x"], device="cpu")
    assert p in r.native
    np.testing.assert_array_equal(r.read().numpy()[:, 0], tbl.column("i8").to_numpy().astype(np.float32))
    for col in ("d", "u"):
        r = ParquetDeviceReader(p, [col, "x"], device="cpu")
        assert p not in r.native
        got = r.read().numpy()[:, 0]
        want = np.array([float(v) for v in tbl.column(col).to_pylist()], dtype=np.float32)
        np.testing.assert_allclose(got, want, rtol=1e-6)
        assert (got >= 0).all() if col == "u" else True
