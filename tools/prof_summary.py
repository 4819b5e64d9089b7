"""Turn a tools/gpu_profile.sh output directory into committed profile summaries.

python tools/prof_summary.py gpurun_out/r01 profiles/r01
  -> profiles/r01_kernel_stats.md   (rocprofv3 --kernel-trace --stats, top kernels + fused kernels)
  -> profiles/r01_kernel_stats.csv  (the rocprofv3 stats CSV, verbatim)
  -> profiles/r01_bench.json        (the bench line of the same pass)
  -> profiles/pmc_summary.json      (per-launch HBM bytes of the fused kernels, read by bench.py)

HBM bytes follow MI355X_MICROARCH.md section HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced reads on gfx950, so the read
side is doubled ("corrected"); the raw values are kept next to it.
"""
import csv
import json
import pathlib
import shutil
import sys
from collections import defaultdict

FUSED = ("k_static_proj", "k_lyap_prep", "k_lyap_fwd", "k_lyap_bwd", "k_lyap_wgrad", "k_lyap_reduce",
         "k_lyap_static_grads", "k_ot_masks", "k_ot_fwd", "k_ot_bwd", "k_inv_gj", "k_groupsort_fwd",
         "k_groupsort_bwd", "k_ode", "k_dyn", "k_qp", "k_cert", "k_spec_dft", "k_spec_fwd", "k_spec_bwd",
         "k_spec_taps", "k_spec_gram", "k_spec_inv", "k_spec_qbot", "k_spec_ginv", "k_spec_kk", "k_spec_gv",
         "k_panel_pad", "k_panel_pivot", "k_panel_update", "k_sconv_rfft2", "k_sconv_irfft2", "k_small_cayley",
         "k_ode_nll", "k_dense")


def short(name: str) -> str:
    if "k_inv_gj<" in name:          # keep the template: element type and padded size
        i = name.find("k_inv_gj<")
        t = name[i:].split(">(")[0].replace("(anonymous namespace)::", "")
        return t + ">"
    for k in FUSED:
        if k in name:
            i = name.find(k)
            return name[i:].split("(")[0]
    return name[:90]


def pmc(path: pathlib.Path, counter: str):
    f = path / f"pmc_{counter}" / "run_counter_collection.csv"
    if not f.exists():
        return {}
    acc = defaultdict(list)
    with f.open() as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(src: str, dst: str):
    src_p, dst_p = pathlib.Path(src), pathlib.Path(dst)
    dst_p.parent.mkdir(parents=True, exist_ok=True)
    stats = src_p / "trace" / "run_kernel_stats.csv"
    # bench.py's per-kernel timing parks the stream behind torch.cuda._sleep spins: not work
    rows = [r for r in csv.DictReader(stats.open()) if "spin_kernel" not in r["Name"]]
    shutil.copy(stats, f"{dst}_kernel_stats.csv")
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats  ({src_p.name})", "",
             "Command: `rocprofv3 --kernel-trace --stats --output-format csv -- python bench.py --steps 10 "
             "--warmup 3 --no-cpu-baseline --no-secondary` (tools/gpu_profile.sh; the step is a hipGraph replay, "
             "the fused kernels are also launched once more per rep by bench.py's per-kernel HIP-event timing).", "",
             f"Total kernel time {total / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches "
             "(torch.cuda._sleep spins of the per-kernel timing excluded).", "",
             "## Fused FI-ODE kernels (libfiode.so)", "",
             "| kernel | calls | avg us | min us | max us | % of total |", "|---|---|---|---|---|---|"]
    for r in rows:
        n = short(r["Name"])
        if n.startswith("k_"):
            lines.append(f"| {n} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | "
                         f"{float(r['MaxNs']) / 1e3:.2f} | {float(r['Percentage']):.2f} |")
    import subprocess
    fam = subprocess.run([sys.executable, str(pathlib.Path(__file__).with_name("kernel_families.py")), str(stats)],
                         capture_output=True, text=True).stdout
    lines += ["", "## Kernel families (all dispatches of the run)", "", "```", fam.rstrip(), "```"]
    lines += ["", "## Top 15 kernels overall", "", "| kernel | calls | avg us | % |", "|---|---|---|---|"]
    for r in rows[:15]:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['Percentage']):.2f} |")
    fetch, write = pmc(src_p, "FETCH_SIZE"), pmc(src_p, "WRITE_SIZE")
    summ = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        fr, wr = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        summ[k] = {"fetch_bytes_raw": fr, "write_bytes": wr, "hbm_bytes_per_launch": 2 * fr + wr,
                   "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->bytes"}
    if summ:
        lines += ["", "## HBM traffic per launch (separate --pmc passes)", "",
                  "| kernel | FETCH raw MB | WRITE MB | corrected total MB |", "|---|---|---|---|"]
        for k, v in summ.items():
            lines.append(f"| {k} | {v['fetch_bytes_raw'] / 1e6:.2f} | {v['write_bytes'] / 1e6:.2f} | "
                         f"{v['hbm_bytes_per_launch'] / 1e6:.2f} |")
        (dst_p.parent / "pmc_summary.json").write_text(json.dumps(summ, indent=1))
    bj = src_p / "bench.json"
    if bj.exists():
        shutil.copy(bj, f"{dst}_bench.json")
    pathlib.Path(f"{dst}_kernel_stats.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
