"""Turn a tools/profile_r03.sh output directory into the committed profiles/ files:
  profiles/<R>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the bench command
  profiles/<R>_bench.json         the bench line measured in the same call
  profiles/<R>_ubench_valu.json   VALU issue rates per instruction (tools/ubench_valu.hip), the peak
  profiles/<R>_fet_traffic.json   HBM bytes per FET scan from the FETCH_SIZE / WRITE_SIZE passes
  profiles/<R>_fet_valu.json      VALU wave-instructions per FET scan (SQ_INSTS_VALU) + SQ cycles
  profiles/<R>_css_valu.json      VALU wave-instructions per window of the kernels each CSS leg
                                  dispatches: c3 (k_css_pack + k_css_mds_p40), c4 (k_css_pack +
                                  k_css_mds_t80), c5_perm (k_css_perm<80>)
  profiles/<R>_summary.md         per-kernel averages, per-scan traffic and instruction counts
Every kernel a figure is built from must be present in its counter file: a missing one
(e.g. a renamed kernel) stops the script instead of silently dropping out of a sum.
"""
import csv
import json
import shutil
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
R = sys.argv[1] if len(sys.argv) > 1 else "r03"
src = ROOT / "gpurun_out" / R
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)

FET_KERNELS = ("k_popsize", "k_bounds", "k_snp_fet", "k_fet_")
SQ = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVES", "SQ_INSTS_LDS",
      "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS")


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def find(d, suffix):
    hits = sorted(Path(d).rglob(f"*{suffix}"))
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def counters(d):
    """{kernel: {counter: sum over dispatches}}, {kernel: dispatches}"""
    f = find(d, "counter_collection.csv")
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for row in csv.DictReader(open(f)):
        k = short(row["Kernel_Name"])
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
    return per, {k: len(v) for k, v in disp.items()}


def need(per, names, where):
    missing = [n for n in names if n not in per]
    if missing:
        raise SystemExit(f"{where}: kernels {missing} absent from the counters (have {sorted(per)})")


def last_json(path):
    for line in reversed(Path(path).read_text().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


stats = find(src / "ktrace", "kernel_stats.csv")
shutil.copy(stats, dst / f"{R}_kernel_stats.csv")
bench = last_json(src / "bench.json")
(dst / f"{R}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")

# ---- VALU issue peak (tools/ubench_valu.hip: 8 waves per SIMD, 8 independent chains per lane)
rates = {}
for line in (src / "ubench_valu.txt").read_text().splitlines():
    parts = line.split()
    if len(parts) >= 2:
        try:
            rates[" ".join(parts[:-1]) if parts[-1] != "Tlane-op/s" else parts[0]] = float(
                parts[-2] if parts[-1] == "Tlane-op/s" else parts[-1])
        except ValueError:
            pass
ginst = {k: v * 1e12 / 64 / 1e9 for k, v in rates.items()}
simple = [ginst[k] for k in ("v_add_u32", "v_sub_u32", "v_and_b32", "v_lshrrev_b32", "v_max_i32", "v_mul_f32")
          if k in ginst]
if not simple:
    raise SystemExit("ubench_valu.txt holds no simple-op rates")
peak = statistics.median(simple)
ub = {"peak_ginsts": peak, "method": "tools/ubench_valu.hip on the box: median issue rate of v_add_u32, v_sub_u32, "
      "v_and_b32, v_lshrrev_b32, v_max_i32, v_mul_f32 (8 waves per SIMD, 8 independent chains per lane)",
      "ginsts_per_op": ginst, "tlane_ops_per_op": rates,
      "cycles_per_wave_inst_per_simd": {k: 256 * 4 * 2.4 / v for k, v in ginst.items() if v > 0}}
(dst / f"{R}_ubench_valu.json").write_text(json.dumps(ub, indent=1) + "\n")

# ---- FET HBM traffic and VALU per scan
fetch, nf = counters(src / "pmc_fetch")
write, _ = counters(src / "pmc_write")
need(fetch, ["k_popsize", "k_bounds", "k_fet_window_fast"], "pmc_fetch")
scans = nf["k_popsize"]
fk = {k: v["FETCH_SIZE"] for k, v in fetch.items() if k.startswith(FET_KERNELS)}
wk = {k: v["WRITE_SIZE"] for k, v in write.items() if k.startswith(FET_KERNELS)}
# rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB; gfx950 FETCH_SIZE counts half of a wide
# coalesced read (MI355X_MICROARCH.md, HBM section): double it
fetch_b = 2 * 1024 * sum(fk.values()) / scans
write_b = 1024 * sum(wk.values()) / scans
cfg = bench["config"]
config = [cfg["chromosomes_per_gpu"], cfg["snps_per_gpu"] // cfg["chromosomes_per_gpu"], cfg["asize"], cfg["bsize"]]
traffic = {
    "config": config, "bytes_per_scan": fetch_b + write_b, "fetch_bytes_per_scan": fetch_b,
    "write_bytes_per_scan": write_b, "scans": scans,
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the FET scan kernels; "
              "KiB -> bytes, FETCH_SIZE x2 (gfx950 wide-read correction)",
    "per_kernel_kib_per_scan": {k: {"fetch": fk.get(k, 0) / scans, "write": wk.get(k, 0) / scans}
                                for k in sorted(set(fk) | set(wk))},
}
(dst / f"{R}_fet_traffic.json").write_text(json.dumps(traffic, indent=1) + "\n")

valu, nv = counters(src / "pmc_valu")
need(valu, ["k_popsize", "k_bounds", "k_fet_window_fast"], "pmc_valu")
vscans = nv["k_popsize"]
vk = {k: v for k, v in valu.items() if k.startswith(FET_KERNELS)}
valu_doc = {
    "config": config,
    "valu_wave_insts_per_scan": sum(v["SQ_INSTS_VALU"] for v in vk.values()) / vscans,
    "scans": vscans,
    "method": "rocprofv3 --pmc SQ_INSTS_VALU (+ SQ cycle counters) over the FET scan kernels (wave-instructions)",
    "per_kernel_per_scan": {k: {c: v.get(c, 0.0) / vscans for c in SQ} for k, v in sorted(vk.items())},
}
(dst / f"{R}_fet_valu.json").write_text(json.dumps(valu_doc, indent=1) + "\n")

# ---- CSS legs: wave-instructions per window of the kernels each leg dispatches
css_doc = {}


def css_entry(key, d, kernels, windows, what):
    per, nd = counters(d)
    need(per, kernels, d.name)
    ipw = sum(per[k]["SQ_INSTS_VALU"] / nd[k] for k in kernels) / windows
    css_doc[key] = {"kernels": kernels, "windows_per_dispatch": windows, "valu_wave_insts_per_window": ipw,
                    "method": f"rocprofv3 --pmc SQ_INSTS_VALU ... over {' + '.join(kernels)} ({what}); "
                              "wave-instructions per dispatch / windows per dispatch",
                    "per_kernel_per_dispatch": {k: {c: per[k].get(c, 0.0) / nd[k] for c in SQ} for k in kernels}}


c3b = last_json(src / "pmc_c3.json")
css_entry("c3", src / "pmc_c3", ["k_css_pack", "k_css_mds_p40"], c3b["css"]["c3"]["windows_per_gpu"],
          "bench.py C3 leg: 20 x 500k SNPs, 20+20, runs=0")
c4t = last_json(src / "pmc_c4.txt")
css_entry("c4", src / "pmc_c4", ["k_css_pack", "k_css_mds_t80"], c4t["windows_per_scan"],
          "tools/css_time.py: 4 x 500k SNPs, 40+40, runs=0")
c5t = last_json(src / "pmc_c5.txt")
css_entry("c5_perm", src / "pmc_c5", ["k_css_perm<80>"], c5t["windows_per_scan"],
          "tools/css_time.py: 1 x 500k SNPs, 40+40, mcT=10, mcR=1000")
# matrix-core share of the permutation kernel (score_mfma): SQ_VALU_MFMA_BUSY_CYCLES counts
# busy SIMD cycles (32 per v_mfma_f32_32x32x16), GRBM_GUI_ACTIVE the GPU cycles summed over
# the 8 XCDs
if (src / "pmc_c5_mfma").exists():
    mf, nmf = counters(src / "pmc_c5_mfma")
    need(mf, ["k_css_perm<80>"], "pmc_c5_mfma")
    k = mf["k_css_perm<80>"]
    nd = nmf["k_css_perm<80>"]
    busy, active = k["SQ_VALU_MFMA_BUSY_CYCLES"] / nd, k["GRBM_GUI_ACTIVE"] / nd / 8
    css_doc["c5_perm"]["mfma"] = {
        "busy_simd_cycles_per_dispatch": busy, "kernel_cycles": active, "mfma_per_dispatch": busy / 32,
        "frac": busy / (1024 * active),
        "method": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES over "
                  "k_css_perm<80> (tools/css_time.py C5 shape); frac = busy / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)"}
(dst / f"{R}_css_valu.json").write_text(json.dumps(css_doc, indent=1) + "\n")

# ---- CSS distance build: k_css_pack's share of pack + MDS from the kernel traces
# of the C3 / C4 shapes, the popcount D build's share of the MDS kernel from the GD_CSS_PROFILE
# phase cycles (tools/ab/cssprof), the shapes' mean SNP rows per window
phase_doc = {}
PH = ("D", "fill+center", "tridiag", "bisect", "invit", "back", "score")
for key, mds in (("c3", "k_css_mds_p40"), ("c4", "k_css_mds_t80")):
    if not (src / f"kt_{key}").exists() or not (src / f"ph_{key}.err").exists():
        continue
    kavg = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(find(src / f"kt_{key}", "kernel_stats.csv")))}
    if "k_css_pack" not in kavg or mds not in kavg:
        raise SystemExit(f"kt_{key}: k_css_pack / {mds} absent (have {sorted(kavg)})")
    lines_ph = [ln for ln in (src / f"ph_{key}.err").read_text().splitlines() if ln.startswith("css-prof cycles:")]
    if not lines_ph:
        raise SystemExit(f"ph_{key}.err: no css-prof line (was the cssprof variant loaded?)")
    vals = [int(t) for t in lines_ph[-1].split(":", 1)[1].split() if t.isdigit()]
    cyc = dict(zip(PH, vals))
    tot = sum(cyc.values())
    t = last_json(src / f"kt_{key}.txt")
    phase_doc[key] = {
        "pack_us": kavg["k_css_pack"] / 1e3, "mds_us": kavg[mds] / 1e3,
        "pack_share": kavg["k_css_pack"] / (kavg["k_css_pack"] + kavg[mds]),
        "d_share": cyc["D"] / tot, "phase_cycles": cyc, "npos_mean": t["npos_mean"],
        "windows_per_scan": t["windows_per_scan"],
        "method": f"tools/css_time.py ({t['nch']} x {t['nsnp']} SNPs, {t['pop']}+{t['pop']}, runs 0): k_css_pack and "
                  f"{mds} average durations (rocprofv3 --kernel-trace --stats); D share = the phase-0 cycles "
                  "(regularity check + popcount compare_all) over all phases of the GD_CSS_PROFILE build"}
if phase_doc:
    (dst / f"{R}_css_phases.json").write_text(json.dumps(phase_doc, indent=1) + "\n")

# ---- summary
rows = list(csv.DictReader(open(stats)))
lines = [f"# {R} profile summary", "",
         "Commands: tools/profile_round.sh (bench line; `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 "
         "--warmup 1 --no-cpu --c45-steps 1`; PMC passes in runs of their own).", "",
         "| kernel | calls | avg us | total ms |", "|---|---|---|---|"]
for r in rows:
    lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                 f"{float(r['TotalDurationNs']) / 1e6:.2f} |")
alg = bench["roofline"]["alg_bytes_per_step"]
scan_ms = bench["stage_ms"]["scan_total"]
lines += ["", f"VALU issue peak (ubench, median of simple ops): {peak:.0f} G wave-instructions/s "
          f"= {256 * 4 * 2.4 / peak:.2f} cycles per wave64 instruction per SIMD at 2.4 GHz. Per op: "
          + ", ".join(f"{k} {v:.0f}" for k, v in ginst.items()) + ".",
          "", f"FET scan HBM traffic (PMC): {traffic['bytes_per_scan'] / 1e9:.3f} GB per scan "
          f"(fetch {fetch_b / 1e9:.3f} + write {write_b / 1e9:.3f}); algorithmic B = {alg / 1e9:.3f} GB.",
          "", f"FET scan VALU (PMC SQ_INSTS_VALU): {valu_doc['valu_wave_insts_per_scan'] / 1e9:.3f} G wave-instructions "
          f"per scan = {valu_doc['valu_wave_insts_per_scan'] / (scan_ms * 1e-3) / 1e9:.0f} G/s at the bench's scan time "
          f"({scan_ms:.3f} ms), {valu_doc['valu_wave_insts_per_scan'] / (scan_ms * 1e-3) / 1e9 / peak:.2f} of the "
          "measured issue peak.", ""]
for k, v in css_doc.items():
    lines.append(f"CSS {k}: {v['valu_wave_insts_per_window']:.0f} VALU wave-instructions per window "
                 f"({' + '.join(v['kernels'])})."
                 + (f" Matrix cores: {v['mfma']['mfma_per_dispatch'] / 1e6:.1f} M v_mfma_f32_32x32x16_f16 per "
                    f"dispatch, {100 * v['mfma']['frac']:.1f} % of the SIMD-cycles busy." if "mfma" in v else ""))
for k, v in phase_doc.items():
    lines.append(f"CSS {k} distance build: k_css_pack {v['pack_us']:.1f} us + popcount D "
                 f"{100 * v['d_share']:.1f} % of the MDS kernel ({v['mds_us']:.1f} us), "
                 f"{v['npos_mean']:.1f} SNP rows per window.")
lines += ["", "Bench line (same call):", "", "```", json.dumps(bench), "```"]
(dst / f"{R}_summary.md").write_text("\n".join(lines) + "\n")
print("\n".join(lines[:60]))
