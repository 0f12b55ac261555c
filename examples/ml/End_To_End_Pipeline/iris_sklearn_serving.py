# %% [markdown]
# # Iris: feature store -> KNN -> model registry -> Python serving -> inference log
# Mirrors notebooks/ml/End_To_End_Pipeline/sklearn/IrisClassification_And_Serving_SKLearn.ipynb and the
# `Predict` contract of iris_flower_classifier.py.
# %%
import json
import os

import joblib
import numpy as np
import pandas as pd
from sklearn.datasets import load_iris
from sklearn.neighbors import KNeighborsClassifier

import hsfs
from hops import hdfs, kafka, model, serving

conn = hsfs.connection()
fs = conn.get_feature_store()
iris = load_iris(as_frame=True)
df = iris.frame.rename(columns=lambda c: c.replace(" (cm)", "").replace(" ", "_"))
df["id"] = np.arange(len(df))
fg = fs.create_feature_group("iris_features", version=1, primary_key=["id"], description="Iris flower features")
fg.save(df)

# %%
data = fg.read()
X, y = data[["sepal_length", "sepal_width", "petal_length", "petal_width"]].to_numpy(), data["target"].to_numpy()
knn = KNeighborsClassifier(n_neighbors=5).fit(X, y)
acc = float(knn.score(X, y))
print("train accuracy", acc)

# %%
os.makedirs("iris_model", exist_ok=True)
joblib.dump(knn, "iris_model/iris_knn.pkl")
with open("iris_model/iris_flower_classifier.py", "w") as f:
    f.write('''import joblib, os
class Predict(object):
    def __init__(self):
        self.model = joblib.load(os.path.join(os.path.dirname(__file__), "iris_knn.pkl"))
    def predict(self, inputs):
        return self.model.predict(inputs).tolist()
    def classify(self, inputs):
        return self.model.predict_proba(inputs).tolist()
    def regress(self, inputs):
        return self.predict(inputs)
''')
path = model.export("iris_model", "IrisFlowerClassifier", metrics={"accuracy": acc})
best = model.get_best_model("IrisFlowerClassifier", "accuracy", model.Metric.MAX)
print(best)

# %%
serving.create_or_update("irisflowerclassifier", path, model_version=best["version"], model_server="FLASK")
serving.start("irisflowerclassifier")
resp = serving.make_inference_request("irisflowerclassifier", {"inputs": X[:5].tolist()})
print(resp)

# %%
consumer = kafka.Consumer({"group.id": "iris", "auto.offset.reset": "earliest"})
consumer.subscribe([serving.get_kafka_topic("irisflowerclassifier")])
msg = consumer.poll(timeout=5.0)
print(json.loads(msg.value())["inferenceResponse"])
serving.stop("irisflowerclassifier")
conn.close()
