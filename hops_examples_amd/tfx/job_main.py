"""Program of the pipeline's job-backed stages (``jobs`` runs a file): ``python job_main.py
<component> --root DIR [...]`` -> :func:`hops_examples_amd.tfx.pipeline.main`."""
import os
import sys
from pathlib import Path

if __name__ == "__main__":
    sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from hops_examples_amd.tfx.pipeline import main

    sys.exit(main())
