# %% [markdown]
# # CIFAR-10 ResNet with `experiment.collective_allreduce`
# The reference names CollectiveAllReduceStrategy / `experiment.collective_allreduce` only in prose
# (notebooks/ml/Experiment/Tensorflow/mnist.ipynb:52) and BASELINE.json config 5 asks for a CIFAR-10
# ResNet trained this way: one worker process per GPU, the gradient exchange over RCCL / the P2P xGMI
# step tail, BatchNorm + residual epilogues in the hopsx conv kernels.  ResNet-20 (He et al. CIFAR
# variant), SGD + momentum 0.9, weight decay 1e-4, per-replica batch 128, synthetic 32x32 images
# with a class-dependent colour cue (no dataset download).  On a GPU-less host: 2 gloo ranks on CPU.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def cifar_training():
    import torch

    from hops_examples_amd import optim
    from hops_examples_amd.models.resnet import cifar_resnet
    from hops_examples_amd.ops import functional as F
    from hops_examples_amd.parallel import dist, ps
    from hops_examples_amd.runtime.arena import ALIGN, ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    rank, _, world = dist.init()
    dev = dist.device()
    B = 16 if dev.type != "cuda" else 128
    steps = 4 if FAST or dev.type != "cuda" else 200
    g = torch.Generator().manual_seed(100 + rank)
    nb = 8
    y = torch.randint(0, 10, (nb, B), generator=g)
    x = torch.randint(0, 160, (nb, B, 32, 32, 3), dtype=torch.uint8, generator=g)
    for c in range(10):  # class cue: one channel brightened in a class-specific band
        x[..., c * 3:c * 3 + 3, :, c % 3][y == c] += 90
    x, y = x.to(dev), y.to(dev)
    torch.manual_seed(0)
    model = cifar_resnet(20).to(dev)
    ParamArena.from_module(model, dev, pad_multiple=world * ALIGN)
    opt = optim.SGD(model, lr=0.05, momentum=0.9, weight_decay=1e-4)
    dp = ps.make(model, opt)
    step = TrainStep(model, opt, "sparse_ce", dp=dp, graph=dev.type == "cuda")
    for i in range(steps):
        r = step.step_resident(x, y)
    model.eval()
    st = {}
    with torch.no_grad():
        F.loss(model(x[0]), y[0], stats=st)
    acc = dist.all_reduce_scalar(float(st["correct"]) / B, "sum") / world
    path = getattr(dp, "path", "none")
    if hasattr(dp, "close"):
        dp.close()
    return {"accuracy": acc, "loss": float(r["loss"]), "allreduce": path, "replicas": world}


# %%
n = None if os.environ.get("HOPSX_NUM_GPUS", "") not in ("", "0") else 2
logdir, result = experiment.collective_allreduce(cifar_training, name="cifar10 resnet20", metric_key="accuracy",
                                                 num_workers=n)
print(result)
