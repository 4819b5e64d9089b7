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
         "k_lyap_static_grads", "k_ot_masks", "k_ot_fwd", "k_ot_bwd", "k_odp_fwd", "k_odp_bwd", "k_inv_gj", "k_groupsort_fwd",
         "k_groupsort_bwd", "k_ode", "k_dyn", "k_qp", "k_cert", "k_spec_dft", "k_spec_fwd", "k_spec_bwd",
         "k_spec_taps", "k_spec_gram", "k_spec_inv", "k_spec_qbot", "k_spec_ginv", "k_spec_kk", "k_spec_gv",
         "k_panel_pad", "k_panel_pivot", "k_panel_update", "k_sconv_rfft2", "k_sconv_irfft2", "k_small_cayley", "k_adam",
         "k_ode_nll", "k_dense", "k_pinv", "k_cgemm", "k_gemm")


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


def pmc(path: pathlib.Path, counter: str, pass_dir: str = None):
    f = path / f"pmc_{pass_dir or counter}" / "run_counter_collection.csv"
    if not f.exists():
        return {}
    acc = defaultdict(list)
    with f.open() as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


# MFMA issue cycles per launch expected from the kernels' instruction counts at the bench shape
# (B = 128, S = 256: N = 32,768 rows; train_ode E = 40 evals of 8 tiles), per SIMD:
# v_mfma_f32_32x32x2_f32 = 64 cycles, v_mfma_f32_16x16x4_f32 = 32 cycles (MI355X_MICROARCH.md).
#   k_lyap_fwd   (20 + 256 + 64) MFMA32 per 32-row tile per pass x 2 passes x 1,024 tiles
#   k_lyap_bwd   fused: per tile and wave 20 (layer 1) + 64 (layer-2 block) + 5 (Q3^T) + 64 (Q2^T block)
#                + 64 (its quarter of dQ2) = 217 MFMA32, + 16 MFMA16 (dQ3 / dQ1, round 3) x 4 waves x 1,024 tiles
#   k_ot_fwd4    (4-row tiles, round 3) 77 v_mfma_f32_4x4x1_16b_f32 (8 cycles) per wave per eval x 4 waves
#                x 32 tiles x 40 evals
#   k_lyap_wgrad (the train_ode solve's weight gradients, N = B x 40 evals) 6 MFMA32 per wave per row pair x 4 waves x N / 2
#   k_ot_fwd     96 MFMA16 per wave per eval x 4 waves x 8 tiles x 40 evals (k_ot_bwd the same)
EXPECTED_MFMA_SIMD_CYCLES = {
    "k_lyap_fwd": 340 * 2 * 1024 * 64, "k_lyap_bwd": (217 * 64 + 16 * 32) * 4 * 1024, "k_lyap_wgrad": 24 * 2560 * 64,
    "k_ot_fwd": 96 * 4 * 8 * 40 * 32, "k_ot_fwd4": 77 * 4 * 32 * 40 * 8, "k_ot_bwd": 96 * 4 * 8 * 40 * 32}
N_CU, N_SIMD, N_XCD = 256, 4, 8


def mfma_lds(src_p: pathlib.Path) -> dict:
    """Per-kernel MFMA-busy fraction and LDS bank-conflict share from the MFMA pass."""
    c = {n: pmc(src_p, n, "MFMA") for n in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES", "SQ_LDS_BANK_CONFLICT",
                                          "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE")}
    out = {}
    for k in c["SQ_VALU_MFMA_BUSY_CYCLES"]:
        if not k.startswith("k_"):
            continue
        busy = c["SQ_VALU_MFMA_BUSY_CYCLES"][k]
        gui = c["GRBM_GUI_ACTIVE"].get(k)
        d = {"mfma_busy_cycles": busy, "grbm_gui_active": gui, "sq_busy_cu_cycles": c["SQ_BUSY_CU_CYCLES"].get(k)}
        if gui:
            cyc = gui / N_XCD                          # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles
            d["kernel_cycles"] = cyc
            d["mfma_busy_frac"] = busy / (cyc * N_CU * N_SIMD)
        if k in EXPECTED_MFMA_SIMD_CYCLES:
            d["expected_mfma_simd_cycles"] = EXPECTED_MFMA_SIMD_CYCLES[k]
            d["busy_over_expected"] = busy / EXPECTED_MFMA_SIMD_CYCLES[k]
        bc, ia = c["SQ_LDS_BANK_CONFLICT"].get(k), c["SQ_LDS_IDX_ACTIVE"].get(k)
        if bc is not None and ia:
            d["lds_bank_conflict_frac"] = bc / ia
        out[k] = d
    return out


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
    ml = mfma_lds(src_p)
    summ = {}
    for k in sorted(set(fetch) | set(write) | set(ml)):
        if not k.startswith("k_"):
            continue
        fr, wr = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        summ[k] = {"fetch_bytes_raw": fr, "write_bytes": wr, "hbm_bytes_per_launch": 2 * fr + wr,
                   "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->bytes"}
        summ[k].update(ml.get(k, {}))
    if summ:
        lines += ["", "## HBM traffic per launch (separate --pmc passes)", "",
                  "| kernel | FETCH raw MB | WRITE MB | corrected total MB |", "|---|---|---|---|"]
        for k, v in summ.items():
            lines.append(f"| {k} | {v['fetch_bytes_raw'] / 1e6:.2f} | {v['write_bytes'] / 1e6:.2f} | "
                         f"{v['hbm_bytes_per_launch'] / 1e6:.2f} |")
        if ml:
            lines += ["", "## MFMA busy and LDS bank conflicts per launch (--pmc SQ_VALU_MFMA_BUSY_CYCLES "
                      "SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE)", "",
                      "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs); "
                      "busy/expected = the counter over the MFMA issue cycles the kernel's instruction count implies "
                      "(unit check of the counter).", "",
                      "| kernel | MFMA busy | busy / expected | LDS bank-conflict share |", "|---|---|---|---|"]
            for k, v in summ.items():
                if "mfma_busy_cycles" not in v:
                    continue
                f = lambda x: "-" if x is None else f"{x:.4f}"
                lines.append(f"| {k} | {f(v.get('mfma_busy_frac'))} | {f(v.get('busy_over_expected'))} | "
                             f"{f(v.get('lds_bank_conflict_frac'))} |")
        summ["_source"] = (f"rocprofv3 --pmc passes of `bench.py --steps 2 --warmup 1` ({src_p.name}; "
                           "tools/gpu_profile.sh), not the timed run")
        (dst_p.parent / "pmc_summary.json").write_text(json.dumps(summ, indent=1))
    bj = src_p / "bench.json"
    if bj.exists():
        shutil.copy(bj, f"{dst}_bench.json")
    pathlib.Path(f"{dst}_kernel_stats.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
