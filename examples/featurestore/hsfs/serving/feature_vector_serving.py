# %% [markdown]
# # Online feature store and serving vectors
# Mirrors notebooks/featurestore/hsfs/serving/feature_engineering-online-fs.ipynb and
# feature_vector_model_serving.ipynb (online_enabled feature groups, TD from online FGs,
# init_prepared_statement, serving_keys, get_serving_vector).
# %%
import numpy as np
import pandas as pd

import hsfs

fs = hsfs.connection().get_feature_store()
rng = np.random.default_rng(0)
teams = pd.DataFrame({"team_id": np.arange(20), "team_budget": rng.uniform(1e6, 1e7, 20),
                      "team_position": rng.integers(1, 21, 20)})
players = pd.DataFrame({"team_id": np.arange(20), "average_player_age": rng.uniform(20, 32, 20),
                        "sum_player_rating": rng.uniform(500, 900, 20)})
tfg = fs.create_feature_group("teams_features_online", 1, primary_key=["team_id"], online_enabled=True)
tfg.save(teams)
pfg = fs.create_feature_group("players_features_online", 1, primary_key=["team_id"], online_enabled=True)
pfg.save(players)

# %%
td = fs.create_training_dataset("team_position_prediction", version=1, data_format="csv")
td.save(tfg.select(["team_budget", "team_position"]).join(pfg.select(["average_player_age", "sum_player_rating"])))
td.init_prepared_statement()
print(td.serving_keys)
print(td.get_serving_vector({"team_id": 1}))
