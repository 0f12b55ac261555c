# %% [markdown]
# # Heat map over time (folium HeatMapWithTime stand-in)
# Mirrors notebooks/ml/Plotting/folium_heat_map.ipynb:37-111: 100 points around (48, 5) drifting
# for 1000 steps, a time-indexed heat map with a date per frame.  Frames render to SVG (no tile
# server, no browser widget).
# %%
import os
from datetime import datetime, timedelta

import numpy as np

from hops_examples_amd import plotting

FAST = os.environ.get("HOPSX_FAST") == "1"
np.random.seed(3141592)
initial_data = np.random.normal(size=(100, 2)) * np.array([[1, 1]]) + np.array([[48, 5]])
move_data = np.random.normal(size=(100, 2)) * 0.01
steps = 50 if FAST else 1000
data = [(initial_data + move_data * i).tolist() for i in range(steps)]
weight = 1  # default value
for time_entry in data:
    for row in time_entry:
        row.append(weight)

# %%
m = plotting.Map([48., 5.], zoom=5)
hm = plotting.HeatMapWithTime(data, auto_play=True, min_speed=10.0)
hm.add_to(m)
time_index = [(datetime(2021, 1, 1) + k * timedelta(1)).strftime("%Y-%m-%d") for k in range(len(data))]
m2 = plotting.Map([48., 5.], zoom=6)
hm2 = plotting.HeatMapWithTime(data, index=time_index, auto_play=True, max_opacity=0.3)
hm2.add_to(m2)
frames = hm2.frames(m2)
print(len(frames), "frames;", "first", time_index[0], "last", time_index[-1])
c = hm.centroids()
print("cloud centre drift:", np.round(c[-1] - c[0], 4))
plotting.save(frames[-1], "Resources/plots/heatmap_last_frame.svg")
