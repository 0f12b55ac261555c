# %% [markdown]
# # Single-image inference with ResNet-50
# Mirrors notebooks/ml/Inference/Inference_Hello_World.ipynb: build ResNet-50, save it to the project,
# reload, load an image at 224x224, predict, decode the top-3 classes.  No ImageNet weights are
# available offline, so the network is random-init (labels are class_<i>).
# %%
import numpy as np
import torch
from PIL import Image

from hops import hdfs
from hops_examples_amd import inference
from hops_examples_amd.model import load_torch, save_torch
from hops_examples_amd.models.resnet import resnet50

m = resnet50()
save_torch(m, hdfs.project_path() + "Resources/resnet_imagenet", builder="hops_examples_amd.models.resnet:resnet50")
model = load_torch(hdfs.project_path() + "Resources/resnet_imagenet")

# %%
img = Image.fromarray(np.random.default_rng(0).integers(0, 255, (300, 400, 3), dtype=np.uint8))
img.save("sample.jpg")
x = inference.load_img("sample.jpg", target_size=(224, 224))[None]
preds = inference.predict(model, x)
for i, p in enumerate(inference.decode_predictions(preds, top=3)[0], 1):
    print(f"Top {i} Prediction: {p}")
