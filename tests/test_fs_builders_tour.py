"""JVM-style builder API of the feature store and the FS-tour feature job."""
import pandas as pd
import pytest


@pytest.fixture
def fs(project_root):
    import hops_examples_amd.featurestore as hsfs

    return hsfs.HopsworksConnection.builder.build().getFeatureStore()


def test_builder_time_travel_scala_shapes(fs):
    import hops_examples_amd.featurestore as hsfs

    fg = (fs.createFeatureGroup().name("tt_fg").version(1).description("hudi fg")
          .timeTravelFormat(hsfs.TimeTravelFormat.HUDI).primaryKeys(["id"]).partitionKeys(["part"])
          .hudiPrecombineKey("id").statisticsConfig(hsfs.statistics_config(True, True, True)).build())
    fg.save(pd.DataFrame({"id": [1, 2, 3], "part": [0, 0, 1], "v": [1.0, 2.0, 3.0]}))
    fg.insert(pd.DataFrame({"id": [2, 4], "part": [0, 1], "v": [20.0, 4.0]}))
    cd = fg.commitDetails()
    assert len(cd) == 2
    got = fs.getFeatureGroup("tt_fg", 1).selectAll().read().sort_values("id")
    assert got["v"].tolist() == [1.0, 20.0, 3.0, 4.0]
    first = sorted(cd)[0]
    assert sorted(fg.selectAll().asOf(first).read()["id"].tolist()) == [1, 2, 3]


def test_builder_rules_expectations_validation(fs):
    import hops_examples_amd.featurestore as hsfs
    from hops_examples_amd.featurestore import Rule

    r = Rule.createRule(hsfs.RuleName.HAS_MIN).min(0).level(hsfs.Level.WARNING).build()
    assert r.name == "HAS_MIN" and r.min == 0 and r.level == "WARNING"
    r2 = Rule.createRule(hsfs.RuleName.HAS_MAX).max(10).level(hsfs.Level.ERROR).build()
    e = fs.createExpectation().name("range").description("0..10").features(["v"]).rules([r, r2]).build()
    e.save()
    fg = (fs.createFeatureGroup().name("val_fg").version(1).primaryKeys(["id"]).validationType("STRICT")
          .expectations([e]).build())
    fg.save(pd.DataFrame({"id": [1, 2], "v": [1.0, 5.0]}))
    vals = fg.getValidations()
    assert vals and all(x.status == "SUCCESS" for x in vals)
    with pytest.raises(Exception):
        fg.insert(pd.DataFrame({"id": [3], "v": [50.0]}))


def test_featurestore_tour_job(fs, tmp_path):
    from hops_examples_amd.featurestore import tour

    d = tour.generate(tmp_path / "tour", n_teams=12, seed=1)
    out = tour.run(d, fs=fs)
    players = fs.getFeatureGroup(tour.PLAYERS_FEATUREGROUP, 1).read()
    raw = pd.read_csv(d / "players.csv")
    ref = raw.groupby("team_id")["age"].mean()
    got = players.set_index("team_id")["average_player_age"]
    assert (abs(got.sort_index().to_numpy() - ref.sort_index().to_numpy()) < 1e-3).all()
    assert fs.getFeatureGroup(tour.SEASON_SCORES_FEATUREGROUP, 1).online_enabled
    hudi = fs.getFeatureGroup(tour.GAMES_FEATUREGROUP_TOUR_HUDI, 1)
    assert hudi.partition_key == ["score"]
    od = out["season_on_demand"].read()
    assert len(od) > 0 and (od["average_position"] > 3).all()
    td = fs.getTrainingDataset(tour.TOUR_TRAINING_DATASET, 1)
    df = td.read()
    assert set(df.columns) >= {"average_player_age", "team_budget", "average_attendance"} and len(df) == 12
