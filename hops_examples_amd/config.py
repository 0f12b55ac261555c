"""Framework configuration: kwargs first, then ``HOPSX_*`` environment overrides.

Mirrors the knobs the reference passes through Spark job configs
(``jobs-client/spark/job_config.json:1-23``: executor gpus, ``spark.tensorflow.num.ps``)
and the implicit Hopsworks project context (project name / user / root).

Environment:
  HOPSX_PROJECT_ROOT   local directory that plays the role of the HopsFS project
                       (default ``~/.hopsx/projects/<name>``)
  HOPSX_PROJECT_NAME   project name (default ``demo``)
  HOPSX_USER           project user (default ``$USER``)
  HOPSX_GPUS_PER_WORKER, HOPSX_NUM_PS, HOPSX_BUCKET_MB, HOPSX_DTYPE (bf16|fp32),
  HOPSX_GRAPH (1 = capture steady-state train steps into hipGraphs)

Performance / communication knobs read where they act:
  HOPSX_STEPS_PER_EXEC  steps per hipGraph replay (runtime/step.py, default 8)
  HOPSX_DIST_BACKEND    process-group backend override, e.g. ``gloo`` to run several ranks on
                        one GPU (parallel/dist.py; default ``nccl`` = RCCL on GPU)
  HOPSX_ONESHOT_AR      1 = gradient buckets on the P2P one-/two-shot all-reduce kernels
                        (parallel/oneshot.py); HOPSX_ONESHOT_MB staging size (default 8),
                        HOPSX_TWOSHOT_MIN_KB two-shot threshold for N > 2 (default 256)
  HOPSX_GRAPH_COLLECTIVES  1 = capture the RCCL all-reduce inside the step graph
  HOPSX_OPT_GRID        optimizer grid cap (default 256 workgroups up to 8 M params, else 512)
  HOPSX_OPT_NT          1 = nontemporal master/state stores in the optimizer kernel
  HOPSX_GEMM_T64_MIN / HOPSX_GEMM_T128_MIN  tile counts below which a non-split GEMM drops to the
                        next smaller tile (csrc/ops/gemm_core.h plan_gemm; defaults 2 x CUs / CUs)
  HOPSX_GEMM_SPLIT_CFG, HOPSX_GEMM_SPLIT_TARGET  split-K GEMM tile (1 = 64x64) / workgroups per CU
  HOPSX_WGRAD_MFMA_MAXK  largest KH*KW*C on the direct MFMA weight gradient (default 640)
  HOPSX_BNSTATS_MAX_1X1_FLOP  1x1 convs above this run as plain GEMMs (gg engine) + a BN statistics
                        pass (default: no limit); HOPSX_PLAIN_MIN_PX fewest output pixels for that path (256)
  HOPSX_WGRAD_MFMA_MAX_MK  short-conv weight gradients from this many pixel-columns on go to the
                        LDS-DMA engine (default 32M)
  HOPSX_BN_DEFER_MAXC, HOPSX_BN_MAXG, HOPSX_BN_APPLY_MAXG, HOPSX_BN_RPT  BN launch geometry (A/B only)
  HOPSX_BN_COOP         1 = one-launch BN backward with a grid barrier (measured slower; off)
  HOPSX_DGRAD_XCD       1 = XCD-aware block order in the direct MFMA dgrad (measured neutral; off)
  HOPSX_DISABLE         comma list of fast paths to turn off for A/B checks, e.g. bnstats, bn_defer,
                        ks5, bwd_pair, conv_mfma, wgrad_mfma, blaslt_1x1, direct_conv
"""
from __future__ import annotations

import dataclasses
import getpass
import os
from pathlib import Path


@dataclasses.dataclass
class Config:
    project_name: str = "demo"
    project_root: Path = Path.home() / ".hopsx" / "projects" / "demo"
    user: str = "hopsx"
    gpus_per_worker: int = 1
    num_ps: int = 1
    bucket_mb: float = 25.0
    dtype: str = "bf16"
    graph: bool = True
    app_id: str = ""

    @property
    def hdfs_prefix(self) -> str:
        return "hopsfs://"


_cfg: Config | None = None


def _user() -> str:
    try:
        return getpass.getuser()
    except Exception:  # pragma: no cover
        return "hopsx"


def get() -> Config:
    global _cfg
    if _cfg is None:
        name = os.environ.get("HOPSX_PROJECT_NAME", "demo")
        root = os.environ.get("HOPSX_PROJECT_ROOT")
        c = Config(
            project_name=name,
            project_root=Path(root) if root else Path.home() / ".hopsx" / "projects" / name,
            user=os.environ.get("HOPSX_USER", _user()),
            gpus_per_worker=int(os.environ.get("HOPSX_GPUS_PER_WORKER", "1")),
            num_ps=int(os.environ.get("HOPSX_NUM_PS", "1")),
            bucket_mb=float(os.environ.get("HOPSX_BUCKET_MB", "25")),
            dtype=os.environ.get("HOPSX_DTYPE", "bf16"),
            graph=os.environ.get("HOPSX_GRAPH", "1") == "1",
        )
        c.project_root.mkdir(parents=True, exist_ok=True)
        _cfg = c
    return _cfg


def reset() -> None:
    global _cfg
    _cfg = None


def set(**kw) -> Config:  # noqa: A001 - mirrors a config setter
    c = get()
    for k, v in kw.items():
        if not hasattr(c, k):
            raise AttributeError(k)
        setattr(c, k, Path(v) if k == "project_root" else v)
    if "project_root" in kw:
        c.project_root.mkdir(parents=True, exist_ok=True)
    return c
