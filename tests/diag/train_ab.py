"""Same-box A/B of the training step (Model.Loss -> backward -> AdamW, 2 x n pairs, eager) on
two package trees: each leg runs in its own subprocess with that tree's p-ntfields_amd first
on sys.path (its own libpntf.so), alternating A B A B.  Diagnostics only.

    python tests/diag/train_ab.py <pkgdir A> <pkgdir B> [n] [rounds]
"""
import json
import subprocess
import sys

CHILD = r'''
import sys, time, json
sys.path.insert(0, sys.argv[1])
import torch
from models import model_res_sigmoid_multi as md
from pntf import synth
from pntf.train import AdamW
n = int(sys.argv[2]); dev = torch.device("cuda", 0); torch.cuda.set_device(0)
net = md.NN(dev, 3)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_weights(0).items()})
net.to(dev)
m = md.Model(".", ".", 3, 2, device=dev); m.network = net
opt = AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
E = 2
pts = torch.from_numpy(synth.make_pairs(E * n, 3, seed=77).reshape(E, n, 6)).to(dev)
yo = torch.from_numpy(synth.make_speeds(E * n, seed=78).reshape(E, n, 2)).to(dev)
Bt = torch.from_numpy(synth.make_B_table(E, 3, first_seed=21)).to(dev)
def step():
    loss, _, _ = m.Loss(pts, yo, Bt, 1.0, 1e-3); loss.backward(); opt.step(); opt.zero_grad()
for _ in range(8): step()
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(30): step()
torch.cuda.synchronize()
print(json.dumps({"pkg": sys.argv[1], "ms": (time.perf_counter() - t0) / 30 * 1e3}))
'''


def main():
    a, b = sys.argv[1], sys.argv[2]
    n = sys.argv[3] if len(sys.argv) > 3 else "10000"
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    for _ in range(rounds):
        for pkg in (a, b):
            r = subprocess.run([sys.executable, "-c", CHILD, pkg, n], capture_output=True,
                               text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print(line[0] if line else json.dumps({"pkg": pkg, "error": r.stderr[-500:]}),
                  flush=True)


if __name__ == "__main__":
    main()
