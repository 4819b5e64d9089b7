"""A/B bit-identity of the block inverse between two builds (not a test):
FIODE_LIB=<lib> python tools/ab_inverse.py out.pt ; python tools/ab_inverse.py --cmp a.pt b.pt"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

if sys.argv[1] == "--cmp":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for k in a:
        print(k, "identical" if torch.equal(a[k], b[k]) else f"DIFFER max {float((a[k] - b[k]).abs().max())}")
    sys.exit(0 if all(torch.equal(a[k], b[k]) for k in a) else 1)

from fiode_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
out = {}
for b, n in ((1, 512), (2, 512), (1, 128), (3, 200), (1, 64)):
    A = torch.randn(b, n, n, generator=g) * 0.05
    M = torch.eye(n) + (A - A.mT) + 0.1 * (A @ A.mT) / n
    inv = ops.block_inverse(M.to(dev)) if b > 1 else ops.block_inverse(M[0].to(dev))
    out[f"inv{b}x{n}"] = inv.cpu()
torch.save(out, sys.argv[1])
print("saved", sys.argv[1])
