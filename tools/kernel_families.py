"""Group a rocprofv3 kernel_stats.csv by kernel family (not a test)."""
import csv, re, sys
from collections import defaultdict
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "spin_kernel" not in r["Name"]]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
fam = defaultdict(lambda: [0.0, 0])
def family(n):
    for k in ("k_lyap", "k_static_proj", "k_ot_", "k_inv_gj", "k_cert", "k_ode", "k_dyn", "k_qp", "k_spec_",
              "k_panel_", "k_sconv_", "k_groupsort"):
        if k in n:
            return k
    if n.startswith("Cijk") or "gemm" in n.lower():
        return "GEMM (hipBLASLt/Tensile)"
    if "fft" in n.lower():
        return "FFT"
    if "rocclr_copyBuffer" in n or "copy_kernel" in n or "CatArray" in n:
        return "copies/cat"
    if "fillBuffer" in n or "FillFunctor" in n:
        return "fills"
    if "reduce_kernel" in n:
        return "reductions"
    if "multi_tensor_apply" in n:
        return "optimizer (foreach)"
    m = re.search(r"at::native::[^<(]*?(\w+Functor|\w+_kernel\w*)", n)
    if "elementwise" in n or "Functor" in n:
        return "elementwise"
    return n[:60]
for r in rows:
    f = fam[family(r["Name"])]
    f[0] += float(r["TotalDurationNs"]); f[1] += int(r["Calls"])
tot = sum(v[0] for v in fam.values())
for k, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
    unit = "us/step" if steps != 1.0 else "us total"
    print(f"{t/1e3/steps:9.1f} {unit} {c/steps:7.1f} calls  {100*t/tot:5.1f}%  {k}")
print(f"total {tot/1e3/steps:.1f} us")
