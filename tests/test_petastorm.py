"""Petastorm-compatible datasets (notebooks/featurestore/petastorm/PetastormHelloWorld.ipynb):
Unischema + codecs, materialize/write, make_reader with column selection, sharding, predicates,
batch reader over plain Parquet, torch DataLoader, legacy featurestore TD in petastorm format."""
import numpy as np
import pandas as pd
import pytest


def _schema():
    from petastorm.codecs import CompressedImageCodec, NdarrayCodec, ScalarCodec
    from petastorm.types import IntegerType
    from petastorm.unischema import Unischema, UnischemaField

    return Unischema("HelloWorldSchema", [
        UnischemaField("id", np.int32, (), ScalarCodec(IntegerType()), False),
        UnischemaField("image1", np.uint8, (128, 256, 3), CompressedImageCodec("png"), False),
        UnischemaField("array_4d", np.uint8, (None, 128, 30, None), NdarrayCodec(), False),
    ])


def _rows(n=10):
    rng = np.random.default_rng(0)
    return [{"id": x, "image1": rng.integers(0, 255, (128, 256, 3), dtype=np.uint8),
             "array_4d": rng.integers(0, 255, (4, 128, 30, 3), dtype=np.uint8)} for x in range(n)]


def test_hello_world_roundtrip(project_root):
    from hops import hdfs
    from petastorm import make_reader
    from petastorm.etl.dataset_metadata import materialize_dataset, write_rows

    schema = _schema()
    url = hdfs.project_path() + "Resources/hello_world"
    rows = _rows()
    with materialize_dataset(None, url, schema, 256):
        write_rows(url, schema, rows, rows_per_group=2)
    with make_reader(url, shuffle_row_groups=False) as reader:
        got = list(reader)
    assert [r.id for r in got] == list(range(10))
    np.testing.assert_array_equal(got[3].image1, rows[3]["image1"])  # png is lossless
    np.testing.assert_array_equal(got[7].array_4d, rows[7]["array_4d"])
    with make_reader(url, schema_fields=["array_4d", "id"]) as r:
        s = next(r)
        assert s._fields == ("array_4d", "id")
    # sharding by row group: 5 row groups over 2 shards
    ids = []
    for shard in range(2):
        with make_reader(url, shard_count=2, cur_shard=shard) as r:
            ids.append(sorted(x.id for x in r))
    assert sorted(ids[0] + ids[1]) == list(range(10)) and not set(ids[0]) & set(ids[1])
    from petastorm.predicates import in_lambda

    with make_reader(url, predicate=in_lambda(["id"], lambda id: id == 5)) as r:
        assert [x.id for x in r] == [5]
    with make_reader(url, num_epochs=3) as r:
        assert len(list(r)) == 30


def test_schema_validation():
    from petastorm.unischema import dict_to_spark_row

    schema = _schema()
    bad = _rows(1)[0]
    bad["image1"] = np.zeros((10, 10, 3), np.uint8)
    with pytest.raises(ValueError):
        dict_to_spark_row(schema, bad)
    assert str(schema.as_spark_schema().field("image1").type) == "binary"


def test_batch_reader_and_torch_loader(project_root):
    import pyarrow as pa
    import pyarrow.parquet as pq
    import torch
    from hops import hdfs
    from petastorm import make_batch_reader, make_reader
    from petastorm.pytorch import DataLoader

    url = hdfs.project_path() + "Resources/hello_world_external"
    p = hdfs._resolve(url)
    p.mkdir(parents=True)
    df = pd.DataFrame({"id": range(10), "value1": np.arange(10) * 2, "value2": -np.arange(10)})
    pq.write_table(pa.Table.from_pandas(df), str(p / "part-0.parquet"), row_group_size=5)
    with make_batch_reader(url, schema_fields=["id", "value1", "value2"], shuffle_row_groups=False) as reader:
        batches = list(reader)
    assert len(batches) == 2 and list(batches[0].id) == [0, 1, 2, 3, 4]
    with DataLoader(make_batch_reader(url, shuffle_row_groups=False)) as loader:
        b = next(iter(loader))
        assert isinstance(b["id"], torch.Tensor) and b["id"].tolist() == [0, 1, 2, 3, 4]
    schema = _schema()
    from petastorm.etl.dataset_metadata import write_rows

    url2 = hdfs.project_path() + "Resources/hw"
    write_rows(url2, schema, _rows(6), rows_per_group=3)
    with DataLoader(make_reader(url2, shuffle_row_groups=False), batch_size=4) as loader:
        bs = list(loader)
    assert bs[0]["image1"].shape == (4, 128, 256, 3) and bs[1]["id"].tolist() == [4, 5]


def test_legacy_featurestore_petastorm_td(project_root):
    from hops import featurestore
    from petastorm.codecs import ScalarCodec
    from petastorm.types import IntegerType
    from petastorm.unischema import Unischema, UnischemaField

    df = pd.DataFrame(np.random.default_rng(0).integers(0, 100, size=(100, 4)), columns=list("ABCD"))
    schema = Unischema("TestSchema", [UnischemaField(c, np.int32, (), ScalarCodec(IntegerType()), False)
                                      for c in "ABCD"])
    featurestore.create_training_dataset(df, "petastorm_hello_world", data_format="petastorm",
                                         petastorm_args={"schema": schema})
    got = featurestore.get_training_dataset("petastorm_hello_world")
    assert len(got) == 100 and sorted(got.A.tolist()) == sorted(df.A.tolist())
    assert featurestore.get_training_dataset_path("petastorm_hello_world").endswith("petastorm_hello_world_1")
