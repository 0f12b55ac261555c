"""Feature-store tour feature-engineering job.

The reference ships it as a Scala/Spark jar (featurestore_tour/src/main/scala/io/hops/examples/
featurestore_tour/Main.scala:13-52 and featuregroups/ComputeFeatures.scala:19-328): read five CSVs
of football data, aggregate per team, and create six feature groups (games, games HUDI partitioned
by score, season_scores online-enabled, attendances, players, teams), one on-demand feature group
over the online store's JDBC connector and a TFRecord training dataset joining three of them.

Here the same job runs as a Python program (``python -m hops_examples_amd.featurestore.tour
--input DIR``, or as a ``jobs`` service job) against the hopsx feature store through the
builder API of builders.py; the per-team group-bys are pandas over Arrow-backed frames (a few
hundred rows — the GPU path is for the training side).  ``generate`` writes synthetic inputs
with the reference's schemas (RawTeam / RawPlayer / RawAttendance / RawSeasonScore / RawGame,
ComputeFeatures.scala:39-90) because the sample CSVs are not part of the snapshot.
"""
from __future__ import annotations

import argparse
import logging
import sys
from pathlib import Path

import numpy as np
import pandas as pd

from .builders import DataFormat, TimeTravelFormat
from .statistics import StatisticsConfig

TEAMS_FEATUREGROUP = "teams_features"
GAMES_FEATUREGROUP = "games_features"
GAMES_FEATUREGROUP_TOUR_HUDI = "games_features_hudi_tour"
SEASON_FEATUREGROUP_TOUR_ON_DEMAND = "season_features_on_demand"
PLAYERS_FEATUREGROUP = "players_features"
ATTENDANCES_FEATUREGROUP = "attendances_features"
SEASON_SCORES_FEATUREGROUP = "season_scores_features"
TOUR_TRAINING_DATASET = "tour_training_dataset_test"
FEATUREGROUP_VERSION = 1

log = logging.getLogger("hopsx.featurestore_tour")


def generate(out_dir, n_teams: int = 50, seed: int = 0) -> Path:
    """Synthetic teams/players/attendances/season_scores/games CSVs with the reference schemas."""
    rng = np.random.default_rng(seed)
    d = Path(out_dir)
    d.mkdir(parents=True, exist_ok=True)
    teams = np.arange(1, n_teams + 1)
    pd.DataFrame({"team_budget": rng.uniform(1e5, 1e7, n_teams).round(2), "team_id": teams,
                  "team_name": [f"team_{i}" for i in teams], "team_owner": [f"owner_{i}" for i in teams],
                  "team_position": rng.permutation(n_teams) + 1}).to_csv(d / "teams.csv", index=False)
    n_p = n_teams * 20
    pd.DataFrame({"age": rng.integers(17, 38, n_p), "rating": rng.uniform(1, 10, n_p).round(3),
                  "team_id": np.repeat(teams, 20), "worth": rng.uniform(1e4, 1e6, n_p).round(2)}
                 ).to_csv(d / "players.csv", index=False)
    years = np.arange(2000, 2020)
    pd.DataFrame({"attendance": rng.uniform(1e3, 8e4, n_teams * len(years)).round(1),
                  "team_id": np.repeat(teams, len(years)), "year": np.tile(years, n_teams)}
                 ).to_csv(d / "attendances.csv", index=False)
    pd.DataFrame({"position": rng.integers(1, n_teams + 1, n_teams * len(years)),
                  "team_id": np.repeat(teams, len(years)), "year": np.tile(years, n_teams)}
                 ).to_csv(d / "season_scores.csv", index=False)
    n_g = n_teams * 10
    pd.DataFrame({"away_team_id": rng.integers(1, n_teams + 1, n_g), "home_team_id": rng.integers(1, n_teams + 1, n_g),
                  "score": rng.integers(0, 6, n_g)}).to_csv(d / "games.csv", index=False)
    return d


def _stats():
    return StatisticsConfig(True, True, True)


def _per_team(raw: pd.DataFrame, cols: dict) -> pd.DataFrame:
    """sum + count per team_id, averaged (the Spark groupBy().sum() join groupBy().count() of
    ComputeFeatures.scala:148-160)."""
    g = raw.groupby("team_id")
    out = pd.DataFrame({"team_id": g.size().index.astype("int32")})
    cnt = g.size().to_numpy().astype(np.float32)
    for src, (avg_name, sum_name) in cols.items():
        s = g[src].sum().to_numpy().astype(np.float32)
        if avg_name:
            out[avg_name] = s / cnt
        if sum_name:
            out[sum_name] = s
    return out


def compute_games(fs, input_dir):
    raw = pd.read_csv(Path(input_dir) / "games.csv")
    fg = (fs.createFeatureGroup().name(GAMES_FEATUREGROUP).version(FEATUREGROUP_VERSION)
          .description("Features of games").timeTravelFormat(TimeTravelFormat.NONE)
          .primaryKeys(["home_team_id"]).statisticsConfig(_stats()).build())
    fg.save(raw)
    hudi = (fs.createFeatureGroup().name(GAMES_FEATUREGROUP_TOUR_HUDI).version(FEATUREGROUP_VERSION)
            .description("Features of games, HUDI feature group example").timeTravelFormat(TimeTravelFormat.HUDI)
            .primaryKeys(["home_team_id"]).partitionKeys(["score"]).statisticsConfig(_stats()).build())
    hudi.save(raw)
    return fg, hudi


def compute_season_scores(fs, input_dir):
    raw = pd.read_csv(Path(input_dir) / "season_scores.csv")
    feats = _per_team(raw, {"position": ("average_position", "sum_position")})
    fg = (fs.createFeatureGroup().name(SEASON_SCORES_FEATUREGROUP).version(FEATUREGROUP_VERSION)
          .description("Features of average season scores for football teams")
          .timeTravelFormat(TimeTravelFormat.NONE).onlineEnabled(True).primaryKeys(["team_id"])
          .statisticsConfig(_stats()).build())
    fg.save(feats)
    return fg


def compute_season_scores_on_demand(fs):
    sc = fs.getOnlineStorageConnector()
    fg = (fs.createOnDemandFeatureGroup().name(SEASON_FEATUREGROUP_TOUR_ON_DEMAND)
          .description("Features of games, on demand feature group example").version(FEATUREGROUP_VERSION)
          .query(f"SELECT * FROM {SEASON_SCORES_FEATUREGROUP}_{FEATUREGROUP_VERSION} WHERE average_position > 3")
          .storageConnector(sc).build())
    fg.save()
    return fg


def compute_attendances(fs, input_dir):
    raw = pd.read_csv(Path(input_dir) / "attendances.csv")
    feats = _per_team(raw, {"attendance": ("average_attendance", "sum_attendance")})
    fg = (fs.createFeatureGroup().name(ATTENDANCES_FEATUREGROUP).version(FEATUREGROUP_VERSION)
          .description("Features of average attendance of games of football teams")
          .timeTravelFormat(TimeTravelFormat.NONE).primaryKeys(["team_id"]).statisticsConfig(_stats()).build())
    fg.save(feats)
    return fg


def compute_players(fs, input_dir):
    raw = pd.read_csv(Path(input_dir) / "players.csv")
    feats = _per_team(raw, {"rating": ("average_player_rating", "sum_player_rating"),
                            "age": ("average_player_age", "sum_player_age"),
                            "worth": ("average_player_worth", "sum_player_worth")})
    feats = feats[["team_id", "average_player_rating", "average_player_age", "average_player_worth",
                   "sum_player_rating", "sum_player_age", "sum_player_worth"]]
    fg = (fs.createFeatureGroup().name(PLAYERS_FEATUREGROUP).version(FEATUREGROUP_VERSION)
          .description("Aggregate features of players football teams").timeTravelFormat(TimeTravelFormat.NONE)
          .primaryKeys(["team_id"]).statisticsConfig(_stats()).build())
    fg.save(feats)
    return fg


def compute_teams(fs, input_dir):
    raw = pd.read_csv(Path(input_dir) / "teams.csv")
    feats = pd.DataFrame({"team_budget": raw["team_budget"].astype(np.float32), "team_id": raw["team_id"],
                          "team_position": raw["team_position"]})
    fg = (fs.createFeatureGroup().name(TEAMS_FEATUREGROUP).version(FEATUREGROUP_VERSION)
          .description("Features of football teams").timeTravelFormat(TimeTravelFormat.NONE)
          .primaryKeys(["team_id"]).statisticsConfig(_stats()).build())
    fg.save(feats)
    return fg


def create_training_dataset(fs):
    players = fs.getFeatureGroup(PLAYERS_FEATUREGROUP, FEATUREGROUP_VERSION)
    teams = fs.getFeatureGroup(TEAMS_FEATUREGROUP, FEATUREGROUP_VERSION)
    att = fs.getFeatureGroup(ATTENDANCES_FEATUREGROUP, FEATUREGROUP_VERSION)
    query = (players.select(["average_player_age"]).join(teams.select(["team_budget"]))
             .join(att.select(["average_attendance"])))
    td = (fs.createTrainingDataset().name(TOUR_TRAINING_DATASET).version(1)
          .description("Sample Training Dataset for the Feature store Tour").dataFormat(DataFormat.TFRECORD)
          .statisticsConfig(_stats()).build())
    td.save(query)
    return td


def run(input_dir, fs=None):
    """The job body (Main.scala:41-48 order)."""
    if fs is None:
        from .store import connection

        fs = connection().get_feature_store()
    log.info("Starting Sample Feature Engineering Job For Feature Store Examples")
    out = {}
    out["games"], out["games_hudi"] = compute_games(fs, input_dir)
    out["season_scores"] = compute_season_scores(fs, input_dir)
    out["attendances"] = compute_attendances(fs, input_dir)
    out["players"] = compute_players(fs, input_dir)
    out["teams"] = compute_teams(fs, input_dir)
    out["season_on_demand"] = compute_season_scores_on_demand(fs)
    out["training_dataset"] = create_training_dataset(fs)
    log.info("feature store tour job complete")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Sample feature engineering job for the feature store tour")
    ap.add_argument("--input", default=None, help="path to input sample data files (csv files); "
                                                  "synthetic data is generated when omitted")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    inp = a.input
    if inp is None:
        from .. import config

        inp = str(generate(config.get().project_root / "Resources" / "featurestore_tour"))
    run(inp)
    return 0


if __name__ == "__main__":
    sys.exit(main())
