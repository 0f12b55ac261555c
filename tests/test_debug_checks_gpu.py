"""Device-side bound checks (common.h hx_check / hx_guard).

* Release build: the always-on guards turn a user-supplied index out of range (an embedding id, a class
  label) into a skipped access plus a record that kernels.debug_errors() names, never into an
  out-of-bounds read or write.
* Debug build (``python -m hops_examples_amd._build --debug`` -> _hopsx_ops_dbg, HOPSX_DEBUG=1): the same
  record makes kernels.check() raise right after the launch, naming the kernel source line; the kernel
  suites also run under it once (tools/gpu.sh debug), with conftest's fixture asserting no record.
"""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"
ROOT = Path(__file__).resolve().parents[1]


def test_embedding_id_out_of_range_is_skipped_and_recorded():
    K.debug_errors()  # (clear)
    torch.manual_seed(0)
    table = torch.randn(50, 24, device=dev)
    idx = torch.tensor([3, 7, 50, 12, -1, 49], device=dev)  # 50 and -1 are out of range
    offs = torch.tensor([0, 3, 6], device=dev)[:2]
    out = torch.zeros(2, 24, device=dev)
    if os.environ.get("HOPSX_DEBUG", "0") == "1":
        with pytest.raises(RuntimeError, match="embedding.hip"):
            K.embedding_bag_fwd(table, idx, offs, 0, out)
        return
    K.embedding_bag_fwd(table, idx, offs, 0, out)
    errs = K.debug_errors()
    assert errs and errs[0][0] == "embedding" and errs[0][1] == 2 * 24, errs  # two ids x 24 lanes
    ref = torch.stack([table[3] + table[7], table[12] + table[49]])
    torch.testing.assert_close(out, ref)
    dt = torch.zeros_like(table)
    K.embedding_bag_bwd(torch.ones(2, 24, device=dev), idx, offs, 0, dt, 2)
    assert K.debug_errors()[0][0] == "embedding"
    assert float(dt.sum()) == 4 * 24 and float(dt[3].sum()) == 24  # only the four valid ids got gradient
    assert K.debug_errors() == []  # reading cleared the record


def test_label_out_of_range_is_recorded():
    K.debug_errors()
    logits = torch.randn(8, 10, device=dev)
    target = torch.tensor([1, 2, 3, 10, 4, 5, 6, 7], device=dev)
    ls, cor = torch.zeros(1, device=dev), torch.zeros(1, device=dev, dtype=torch.int32)
    dl = torch.empty_like(logits)
    if os.environ.get("HOPSX_DEBUG", "0") == "1":
        with pytest.raises(RuntimeError, match="loss.hip"):
            K.loss_fwd_bwd(0, logits, target, 1.0, ls, cor, dl)
        return
    K.loss_fwd_bwd(0, logits, target, 1.0, ls, cor, dl)
    errs = K.debug_errors()
    assert errs and errs[0][0] == "loss" and errs[0][1] == 1, errs
    assert torch.isfinite(ls).all() and torch.isfinite(dl).all()


def test_debug_build_raises_at_the_launch():
    so = list((ROOT / "hops_examples_amd").glob("_hopsx_ops_dbg*.so"))
    if not so:
        pytest.skip("debug build not present (python -m hops_examples_amd._build --debug)")
    code = (
        "import torch\n"
        "from hops_examples_amd.ops import kernels as K, _C\n"
        "assert _C.ext().DEBUG == 1\n"
        "t = torch.randn(8, 16, device='cuda'); out = torch.zeros(1, 16, device='cuda')\n"
        "try:\n"
        "    K.embedding_bag_fwd(t, torch.tensor([1, 9], device='cuda'), torch.tensor([0], device='cuda'), 0, out)\n"
        "except RuntimeError as e:\n"
        "    print('RAISED', e)\n"
    )
    env = dict(os.environ, HOPSX_DEBUG="1", PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "RAISED" in r.stdout and "embedding.hip line" in r.stdout, r.stdout
