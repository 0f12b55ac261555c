"""Repeat the noise-relative model-level GPU tests (BN statistics are float-atomic sums, so these
compare against rerun noise) several times in ONE process and report pass / fail counts."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytest  # noqa: E402,F401
import tests.test_bnstats_gpu as tb  # noqa: E402
import tests.test_kernels_v2_gpu as tk  # noqa: E402


class _MP:  # minimal monkeypatch for the test's setenv
    def setenv(self, k, v):
        os.environ[k] = v


res = {}
for name, fn in (("resnet20_bnstats", tb.test_resnet20_step_bnstats_matches_unfused),
                 ("paired_cifar", lambda: tk.test_paired_conv_backward_matches_separate_launches(_MP(), "cifar")),
                 ("convbn_layer", tb.test_convbn_layer_grads_bnstats_matches_unfused)):
    ok = 0
    for i in range(5):
        try:
            fn()
            ok += 1
        except AssertionError:
            print(name, "FAILED", traceback.format_exc().splitlines()[-1], flush=True)
        os.environ["HOPSX_DISABLE"] = ""
    res[name] = f"{ok}/5"
    print(name, res[name], flush=True)
print(res)
