# %% [markdown]
# # ResNet-50 training benchmark
# Mirrors notebooks/ml/Benchmarks/benchmark.ipynb (ResNet50, synthetic 224x224x3, 1000 classes,
# batch 8 per GPU, RMSprop(0.2)) — which printed no throughput (`{'metric': None}`); this one
# reports images/sec via the benchmark harness (benchmarks/run.py resnet50).
# %%
import os
import subprocess
import sys

root = os.environ.get("HOPSX_REPO", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(
    __file__ if "__file__" in dir() else ".")))))
FAST = os.environ.get("HOPSX_FAST") == "1"
args = [sys.executable, os.path.join(root, "benchmarks", "run.py"), "resnet50", "--steps", "2" if FAST else "50",
        "--warmup", "1" if FAST else "5"] + (["--batch", "2"] if FAST else [])
print(subprocess.run(args, capture_output=True, text=True, check=True).stdout)
