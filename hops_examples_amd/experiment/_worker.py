"""Worker entry point: ``python -m hops_examples_amd.experiment._worker <payload> <result>``.

Loads (fn, kwargs) written by the driver (cloudpickle; files this framework
wrote itself), sets up the process group for distributed runs (WORLD_SIZE > 1),
runs the function, copies a local TensorBoard logdir back into the run
directory and writes (ok, value | traceback).
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile
import traceback


def main() -> int:
    payload, result = sys.argv[1], sys.argv[2]
    import cloudpickle

    ok, value = False, None
    run_dir = os.environ.get("HOPSX_LOGDIR", os.getcwd())
    local_dir = None
    try:
        if os.environ.get("HOPSX_LOCAL_LOGDIR") == "1":
            local_dir = tempfile.mkdtemp(prefix="hopsx_tb_")
            os.environ["HOPSX_TB_LOGDIR"] = local_dir
        else:
            os.environ["HOPSX_TB_LOGDIR"] = run_dir
        with open(payload, "rb") as f:
            fn, kwargs = cloudpickle.loads(f.read())
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            from hops_examples_amd.parallel import dist

            dist.init()
        value = fn(**kwargs)
        ok = True
    except BaseException:
        value = traceback.format_exc()
        print(value, file=sys.stderr, flush=True)
    finally:
        if local_dir is not None:
            for item in os.listdir(local_dir):
                src = os.path.join(local_dir, item)
                dst = os.path.join(run_dir, item)
                if os.path.isdir(src):
                    shutil.copytree(src, dst, dirs_exist_ok=True)
                else:
                    shutil.copy2(src, dst)
            shutil.rmtree(local_dir, ignore_errors=True)
        try:
            from hops_examples_amd.parallel import dist

            dist.shutdown()
        except Exception:
            pass
    try:
        data = cloudpickle.dumps((ok, value))
    except Exception:
        data = cloudpickle.dumps((False, "return value is not picklable:\n" + traceback.format_exc()))
    with open(result, "wb") as f:
        f.write(data)
    sys.stdout.flush()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
