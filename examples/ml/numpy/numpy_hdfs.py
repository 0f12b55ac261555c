# %% [markdown]
# # numpy arrays in the project (`hops.numpy_helper`), mirrors notebooks/ml/numpy/numpy-hdfs.ipynb
# %%
import numpy as np

from hops import numpy_helper as numpy

a = np.arange(12).reshape(3, 4)
numpy.save("Resources/arr.npy", a)
print(numpy.load("Resources/arr.npy"))
