"""Taxi wide&deep trainer step only (for rocprofv3 kernel traces): python tools/taxi_only.py [steps]"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.models.widedeep import bench_taxi


def timed(fn, n, dev):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0


steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
print(json.dumps(bench_taxi(torch.device("cuda", 0), 40, steps, 10, timed)))
