# %% [markdown]
# # Project filesystem operations (`hops.hdfs`)
# Mirrors notebooks/ml/Filesystem/HopsFSOperations.ipynb.
# %%
from hops import hdfs

print(hdfs.project_name(), hdfs.project_path())
hdfs.dump("hello hopsx", "Resources/hello.txt")
print(hdfs.load("Resources/hello.txt"))
print(hdfs.exists("Resources/hello.txt"), hdfs.isfile("Resources/hello.txt"), hdfs.isdir("Resources"))
hdfs.mkdir("Resources/tmp_dir")
hdfs.cp("Resources/hello.txt", "Resources/tmp_dir/hello_copy.txt")
print(hdfs.ls("Resources/tmp_dir"), hdfs.glob(hdfs.project_path() + "Resources/*.txt"))
hdfs.move("Resources/tmp_dir/hello_copy.txt", "Resources/hello_moved.txt")
print(hdfs.lsl("Resources")[:2])
hdfs.chmod("Resources/hello_moved.txt", 0o644)
print(oct(hdfs.stat("Resources/hello_moved.txt").st_mode & 0o777))
local = hdfs.copy_to_local("Resources/hello.txt", "", overwrite=True)
hdfs.copy_to_hdfs("hello.txt", "Resources/uploaded", overwrite=True)
hdfs.rmr("Resources/tmp_dir")
print(hdfs.exists("Resources/tmp_dir"))
