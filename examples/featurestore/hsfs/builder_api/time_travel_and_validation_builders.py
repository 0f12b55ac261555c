# %% [markdown]
# # JVM-style builder API: time travel and data validation
# Mirrors the Scala notebooks notebooks/featurestore/hsfs/time_travel/time_travel_scala.ipynb (builder
# createFeatureGroup().name().version().primaryKeys().partitionKeys().hudiPrecombineKey()
# .timeTravelFormat(HUDI).build(), commitDetails, readChanges, asOf) and
# notebooks/featurestore/hsfs/data_validation/feature_validation_scala.ipynb
# (Rule.createRule(RuleName.HAS_MIN).min(0).level(Level.WARNING).build(), createExpectation(),
# getValidation(ts, ValidationTimeType.COMMIT_TIME)) with the same call shapes in Python.
# %%
import time

import pandas as pd

import hsfs
from hsfs import DataFormat, Level, Rule, RuleName, TimeTravelFormat, ValidationTimeType

fs = hsfs.HopsworksConnection.builder.build().getFeatureStore()
fg = (fs.createFeatureGroup().name("economy_fg_scala").version(1).description("HUDI time travel")
      .timeTravelFormat(TimeTravelFormat.HUDI).primaryKeys(["id"]).partitionKeys(["year"]).hudiPrecombineKey("id")
      .build())
fg.save(pd.DataFrame({"id": [1, 2, 3], "salary": [10.0, 20.0, 30.0], "year": [2020, 2020, 2021]}))
time.sleep(1.1)
fg.insert(pd.DataFrame({"id": [2, 4], "salary": [25.0, 40.0], "year": [2020, 2021]}))
commits = fg.commitDetails()
t0, t1 = [commits[k]["committedOn"] for k in sorted(commits)]
print(fg.readChanges(t0, t1))
print(fg.selectAll().asOf(t0).read())

# %%
rule_min = Rule.createRule(RuleName.HAS_MIN).min(0).level(Level.WARNING).build()
rule_max = Rule.createRule(RuleName.HAS_MAX).max(100).level(Level.ERROR).build()
exp = fs.createExpectation().name("salary_range").description("0 <= salary <= 100").features(["salary"]) \
    .rules([rule_min, rule_max]).build()
exp.save()
vfg = (fs.createFeatureGroup().name("salaries_validated").version(1).primaryKeys(["id"])
       .timeTravelFormat(TimeTravelFormat.HUDI).validationType("ALL").expectations([exp]).build())
vfg.save(pd.DataFrame({"id": [1, 2], "salary": [10.0, 50.0], "year": [2020, 2020]}))
ct = sorted(vfg.commitDetails())[0]
for v in vfg.getValidation(ct, ValidationTimeType.COMMIT_TIME):
    print(v.validation_time, v.status)
td = (fs.createTrainingDataset().name("salaries_td").version(1).dataFormat(DataFormat.CSV).build())
td.save(vfg.selectAll())
print(td.read())
