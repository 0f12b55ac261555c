"""Delta-style versioned tables (notebooks/featurestore/delta/DeltaOnHops.ipynb): bulk insert,
overwrite, versionAsOf time travel, MERGE upsert, history, vacuum."""
import pandas as pd
import pytest


def _df(rows):
    return pd.DataFrame(rows, columns=["id", "date", "value", "country"])


def test_delta_lifecycle(project_root):
    from hops_examples_amd import delta

    path = "Resources/hello_delta"
    v0 = delta.write(_df([(1, "2019-02-30", 0.4151, "Sweden"), (2, "2019-05-01", 1.2151, "Ireland"),
                          (3, "2019-08-06", 0.2151, "Belgium"), (4, "2019-08-06", 0.8151, "Russia")]), path)
    assert v0 == 0
    with pytest.raises(FileExistsError):
        delta.write(_df([]), path)
    v1 = delta.write(_df([(1, "2019-06-30", 0.4151, "Sweden"), (2, "2019-05-01", 1.2151, "Ireland"),
                          (3, "2017-08-06", 0.2151, "Belgium"), (4, "2019-08-06", 0.8151, "Russia")]), path,
                     mode="overwrite")
    assert v1 == 1
    assert delta.read(path, version_as_of=0).date.tolist()[0] == "2019-02-30"
    assert delta.read(path).date.tolist()[0] == "2019-06-30"
    t = delta.DeltaTable.forPath(path)
    up = _df([(5, "2019-02-30", 0.7921, "Northern Ireland"), (1, "2019-05-01", 1.151, "Norway"),
              (3, "2019-08-06", 0.999, "Belgium"), (6, "2019-08-06", 0.0151, "France")])
    cols = {c: f"newData.{c}" for c in ["id", "date", "value", "country"]}
    v2 = (t.alias("oldData").merge(up, "oldData.id = newData.id").whenMatched.update(cols)
          .whenNotMatched.insert(cols).execute())
    assert v2 == 2
    cur = delta.read(path).sort_values("id").reset_index(drop=True)
    assert cur.id.tolist() == [1, 2, 3, 4, 5, 6]
    assert cur.country.tolist() == ["Norway", "Ireland", "Belgium", "Russia", "Northern Ireland", "France"]
    assert abs(cur.value[2] - 0.999) < 1e-9
    assert len(delta.read(path, version_as_of=1)) == 4  # time travel after the merge
    h = delta.history(path)
    assert h.operation.tolist() == ["MERGE", "WRITE", "WRITE"]
    assert t.vacuum(retain_versions=1) == 2 and len(delta.read(path)) == 6
