"""Where the fixed per-launch time of the persistent MNIST step goes at bench.py's 20 steps per run.

Prints (median over reps, us): the host cost of issuing run_resident (Python + HIP launch call, no sync),
the host wall of issue + synchronize, the GPU time between events recorded around the launch, and the
same for an empty elementwise kernel (the launch + completion floor of this process).
usage (GPU): python tools/persist_overhead.py [--steps 20] [--reps 30]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.runtime.arena import ParamArena
    from hops_examples_amd.runtime.step import make_step

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    opt = optim.Adadelta(m, lr=1.0)
    st = make_step(m, opt, "sparse_ce", dp="auto", batch=32, graph=True, steps_per_execution=32)
    xs = torch.randint(0, 256, (1920, 32, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (1920, 32), dtype=torch.int64, device=dev)
    for _ in range(3):
        st.run_resident(xs, ys, a.steps)
    st.prepare_resident(xs, ys, n=a.steps)
    torch.cuda.synchronize()
    issue, wall, gpu, e_issue, e_wall = [], [], [], [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    z = torch.zeros(1, device=dev)
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        st.run_resident(xs, ys, a.steps)
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        issue.append((t1 - t0) * 1e6)
        wall.append((t2 - t0) * 1e6)
        gpu.append(e0.elapsed_time(e1) * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        z.add_(1)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        e_issue.append((t1 - t0) * 1e6)
        e_wall.append((t2 - t0) * 1e6)
    med = statistics.median
    print(f"persistent step, {a.steps} steps per launch (us, median of {a.reps}): issue {med(issue):.1f}, "
          f"issue + sync {med(wall):.1f} ({med(wall) / a.steps:.2f} per step), GPU events {med(gpu):.1f} "
          f"({med(gpu) / a.steps:.2f} per step)")
    print(f"empty elementwise kernel: issue {med(e_issue):.1f}, issue + sync {med(e_wall):.1f}")


if __name__ == "__main__":
    main()
