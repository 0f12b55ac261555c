import os, sys, json
sys.path.insert(0, os.getcwd())
sys.argv = ["x"]
import tools.det_check as D
import torch
out = {}
for dis in ("bnstats,bn_dgrad_sums", "bnstats"):
    a = D.resnet_step(dis); b = D.resnet_step(dis)
    out[dis] = bool(torch.equal(a, b))
    out[dis + "_maxdiff"] = float((a - b).abs().max())
print(json.dumps(out))
