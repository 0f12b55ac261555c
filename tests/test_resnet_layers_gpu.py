"""ResNet-20 training-step numerics checked PER LAYER (runtime/layercheck.py): every conv / BN / GAP /
linear forward against fp64 of the same op on the tensors the kernels read, and every parameter's
gradient against the fp64 backward through the kernels' own forward values (bf16 activation gradients
rounded where the kernels store them).  Both BN-statistics paths (conv-epilogue statistics vs the
separate pass) and both BN-backward-sums paths (consumer dgrad epilogue vs the BN kernel), at batch 16
and 128.

This replaces the whole-step cosine against a free-running fp64 step (0.96, tests/test_bnstats_gpu.py),
which measures the random-init network's sensitivity to any rounding rather than the kernels.
Reference workload: notebooks/ml/Benchmarks/benchmark.ipynb:144; BASELINE config 5.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.runtime import layercheck as LC  # noqa: E402

dev = torch.device("cuda", 0)
VARIANTS = {"fused": "", "bnstats-off": "bnstats", "bnsums-off": "bn_dgrad_sums",
            "both-off": "bnstats,bn_dgrad_sums", "pair-off": "bwd_pair"}


def _check(batch, variant):
    return LC.resnet20_check(batch, VARIANTS[variant])


@pytest.mark.parametrize("batch", [16, 128])
@pytest.mark.parametrize("variant", list(VARIANTS))
def test_resnet20_per_layer_vs_fp64(batch, variant):
    r = _check(batch, variant)
    fw = r["forward"]
    gr = r["grads"]
    worst_f = min(fw, key=lambda t: t[1])
    worst_g = min(gr.items(), key=lambda kv: kv[1][0])
    print(f"\n[B={batch} {variant}] loss {r['loss']:.4f}; {len(fw)} ops, worst forward {worst_f[0]} cos {worst_f[1]:.7f}; "
          f"{len(gr)} parameter tensors, worst gradient {worst_g[0]} cos {worst_g[1][0]:.7f} rel {worst_g[1][1]:.2e}")
    for n, (c, e) in gr.items():
        print(f"  grad {n:28s} cos {c:.7f} rel {e:.2e}")
    bad_f = [(n, c) for n, c, _ in fw if c < 0.9999]
    assert not bad_f, bad_f
    bad_g = [(n, c) for n, (c, _) in gr.items() if c < 0.999]
    assert not bad_g, bad_g
