"""One training-step workload for rocprofv3 (run on the GPU box): 2 envs x 10 000 pairs (the
reference batch), 3 warm + 5 profiled steps of Loss -> loss.backward() -> AdamW."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "p-ntfields_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    print(bench.train_extras(torch.device("cuda", 0), sizes=((2, n),), reps=5), flush=True)
