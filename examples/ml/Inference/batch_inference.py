# %% [markdown]
# # Batch inference over an image directory, one worker per GPU
# Mirrors notebooks/ml/Inference/Batch_Inference_Imagenet_Spark.ipynb (mapPartitions over ImageNet files,
# 10k-image limit, Parquet labels with top-1..3).  Synthetic images; random-init ResNet-50.
# %%
import functools
import os

import numpy as np
from PIL import Image

from hops import hdfs
from hops_examples_amd import inference
from hops_examples_amd.models.resnet import cifar_resnet, resnet50

FAST = os.environ.get("HOPSX_FAST") == "1"
d = hdfs.project_path() + "Resources/images"
os.makedirs(d, exist_ok=True)
rng = np.random.default_rng(0)
paths = []
for i in range(8 if FAST else 256):
    p = os.path.join(d, f"img_{i}.jpg")
    Image.fromarray(rng.integers(0, 255, (256, 256, 3), dtype=np.uint8)).save(p)
    paths.append(p)

# %%
builder = functools.partial(cifar_resnet, 8, num_classes=10) if FAST else resnet50
labels = inference.batch_predict(builder, paths, "Resources/labels.parquet", batch_size=100, limit=10000)
print(labels.head())
print(labels.iloc[0].top1_label, labels.iloc[0].top2_label, labels.iloc[0].top3_label)
