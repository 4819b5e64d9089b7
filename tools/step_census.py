"""Kernel census of one captured training step from a rocprofv3 kernel trace (tools; not a test).

A replay window runs from one `k_ot_fwd4` launch to the next when the two are < 2 ms apart (the
bench's back-to-back graph replays; setup, eager warm-up and the companion configs fall outside).
Prints the number of windows, the library GEMMs (`Cijk_*`, hipBLASLt / Tensile) found inside any
window, and the kernels of the last window by family.

usage: python tools/step_census.py gpurun_out/<tag>/trace/run_kernel_trace.csv
"""
import collections
import csv
import sys


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ot = [s for s, _, n in ks if "k_ot_fwd4" in n]
    win = [(ot[i], ot[i + 1]) for i in range(len(ot) - 1) if ot[i + 1] - ot[i] < 2.0e6]
    print(f"replay windows: {len(win)}")
    lib = collections.Counter()
    for a, b in win:
        for s, _, n in ks:
            if a <= s < b and n.startswith("Cijk"):
                lib[n[:60]] += 1
    print(f"library GEMM (Cijk_) launches inside the windows: {sum(lib.values())}")
    for n, c in lib.most_common():
        print(f"  {c:5d} {n}")
    a, b = win[-1]
    fam = collections.Counter()
    for s, _, n in ks:
        if a <= s < b:
            m = n.replace("(anonymous namespace)::", "").replace("void ", "")
            base = m.split("(")[0]
            if "at::native" in m or "rocclr" in m:
                base = "torch/runtime: " + m.split("<")[0].split("::")[-1][:60]
            fam[base] += 1
    print(f"kernels in the last window: {sum(fam.values())}")
    for n, c in sorted(fam.items(), key=lambda t: (-t[1], t[0])):
        print(f"  {c:4d} {n}")


if __name__ == "__main__":
    main(sys.argv[1])
