# %% [markdown]
# # Feature bias with a census-style LinearClassifier (What-If style counterfactuals)
# Mirrors notebooks/featurestore/feature-bias/feature-bias-whatif.ipynb: numeric + vocabulary indicator
# columns, FTRL, 5000 steps of batch 64; instead of the WIT widget, counterfactual predictions for flipped
# sensitive attributes.  Synthetic UCI-adult-shaped data.
# %%
import os

import numpy as np
import pandas as pd

from hops_examples_amd.models.linear import LinearClassifier

FAST = os.environ.get("HOPSX_FAST") == "1"
rng = np.random.default_rng(0)
n = 8000
df = pd.DataFrame({"Age": rng.integers(17, 90, n), "Education-Num": rng.integers(1, 17, n),
                   "Capital-Gain": rng.exponential(1000, n).round(), "Capital-Loss": rng.exponential(90, n).round(),
                   "Hours-per-week": rng.integers(1, 99, n),
                   "Workclass": rng.choice(["Private", "Self-emp", "Gov", "?"], n),
                   "Marital-Status": rng.choice(["Married", "Never-married", "Divorced"], n),
                   "Occupation": rng.choice(["Tech", "Sales", "Craft", "Service"], n),
                   "Relationship": rng.choice(["Husband", "Wife", "Own-child", "Unmarried"], n),
                   "Race": rng.choice(["White", "Black", "Asian", "Other"], n),
                   "Sex": rng.choice(["Male", "Female"], n), "Country": rng.choice(["US", "Other"], n)})
logit = (0.04 * (df.Age - 40) + 0.3 * (df["Education-Num"] - 10) + 0.03 * (df["Hours-per-week"] - 40)
         + np.where(df.Sex == "Male", 0.6, -0.6) + np.where(df["Marital-Status"] == "Married", 0.8, -0.4))
df["Over-50K"] = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(int)
numeric = ["Age", "Education-Num", "Capital-Gain", "Capital-Loss", "Hours-per-week"]
vocab = {c: sorted(df[c].unique()) for c in ["Workclass", "Marital-Status", "Occupation", "Relationship", "Race",
                                             "Sex", "Country"]}
clf = LinearClassifier(numeric, vocab)
clf.fit(df, "Over-50K", steps=300 if FAST else 5000, batch_size=64)
print(clf.evaluate(df, "Over-50K"))

# %%
sample = df.sample(200, random_state=0)
flipped = sample.assign(Sex=np.where(sample.Sex == "Male", "Female", "Male"))
delta = clf.predict_proba(flipped) - clf.predict_proba(sample)
print("mean |change in P(>50K)| when flipping Sex:", float(np.abs(delta).mean()))
