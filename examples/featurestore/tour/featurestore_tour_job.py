# %% [markdown]
# # Feature store tour: feature engineering job
# Mirrors featurestore_tour/src/main/scala/io/hops/examples/featurestore_tour/Main.scala:13-52 and
# featuregroups/ComputeFeatures.scala: five CSVs of football data -> six feature groups (games, games
# HUDI partitioned by score, online season scores, attendances, players, teams), an on-demand feature
# group over the online store, and a TFRecord training dataset joining players, teams and attendances.
# The sample CSVs are not in the reference snapshot: synthetic data with the same schemas is generated.
# %%
import hsfs
from hops_examples_amd import config
from hops_examples_amd.featurestore import tour

data_dir = tour.generate(config.get().project_root / "Resources" / "featurestore_tour", n_teams=50)
fs = hsfs.HopsworksConnection.builder.build().getFeatureStore()
out = tour.run(data_dir, fs=fs)

# %%
for name in ("games", "games_hudi", "season_scores", "attendances", "players", "teams"):
    fg = out[name]
    print(f"{fg.name} v{fg.version}: {len(fg.read())} rows, primary key {fg.primary_key}")
print(out["season_on_demand"].read().head())
td = fs.getTrainingDataset(tour.TOUR_TRAINING_DATASET, 1)
print(td.read().head())
