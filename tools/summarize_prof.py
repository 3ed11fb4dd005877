"""Turn a tools/profile_round.sh output directory into the committed profiles/ files:
  profiles/<R>_kernel_stats_<leg>.csv  rocprofv3 --kernel-trace --stats summary per leg: fet (the
                                  FET bench command, C2), c3 / c4 / c5 (tools/css_time.py shapes)
  profiles/<R>_fet_timeline.md    one C2 scan's kernels (start / end per kernel and queue) from the
                                  fet trace, and the first window kernel's offset into the scan
  profiles/<R>_bench.json         the bench line measured in the same call
  profiles/<R>_bench_g2.json      the two-rank rehearsal line (--gpus 2 on one GPU, gloo)
  profiles/<R>_ubench_valu.json   VALU issue rates per instruction (tools/ubench_valu.hip), the peak
  profiles/<R>_fet_traffic.json   HBM bytes per FET scan from the FETCH_SIZE / WRITE_SIZE passes
  profiles/<R>_fet_valu.json      VALU wave-instructions per FET scan (SQ_INSTS_VALU) + SQ cycles
  profiles/<R>_css_valu.json      VALU wave-instructions per window of the kernels each CSS leg
                                  dispatches: c3 (k_css_pack + k_css_mds_h40), c4 (k_css_pack +
                                  k_css_mds_t80), c5_perm (k_css_perm<80>); per kernel the VALU
                                  busy fraction 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
                                  (SQ_ACTIVE_INST_* count quad-cycles, GRBM_GUI_ACTIVE sums the 8 XCDs)
  profiles/<R>_css_phases.json    phase cycles of the GD_CSS_PROFILE / GD_PERM_PROFILE builds
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


def valu_busy(c):
    """VALU-active fraction of the SIMD-cycles while the kernel ran"""
    g = c.get("GRBM_GUI_ACTIVE", 0.0)
    return 4.0 * c["SQ_ACTIVE_INST_VALU"] / (1024.0 * g / 8.0) if g > 0 else None


def last_json(path):
    for line in reversed(Path(path).read_text().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


LEGS = ("fet", "c3", "c4", "c5")
for leg in LEGS:
    shutil.copy(find(src / f"kt_{leg}", "kernel_stats.csv"), dst / f"{R}_kernel_stats_{leg}.csv")
stats = dst / f"{R}_kernel_stats_fet.csv"
bench = last_json(src / "bench.json")
(dst / f"{R}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")
if (src / "bench_g2.json").exists():
    (dst / f"{R}_bench_g2.json").write_text(json.dumps(last_json(src / "bench_g2.json"), indent=1) + "\n")

# ---- one C2 scan's timeline (the fourth scan of the fet trace: warm, not the last)
trace = sorted(csv.DictReader(open(find(src / "kt_fet", "kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(trace) if short(r["Kernel_Name"]).startswith(("k_fet_setup", "k_popsize"))]
if len(starts) < 5:
    raise SystemExit(f"kt_fet: {len(starts)} scans in the trace")
i0, i1 = starts[3], starts[4]
t0 = int(trace[i0]["Start_Timestamp"])
tl = ["# " + R + " one FET scan (C2) -- kernel timeline", "",
      "From the `rocprofv3 --kernel-trace` of `python3 bench.py --steps 5 --warmup 1 --no-cpu --no-css --no-extra` "
      "(the fourth scan); times in us from the scan's first kernel.", "",
      "| kernel | queue | start | end | us | workgroups |", "|---|---|---|---|---|---|"]
first_win = None
scan_end = 0.0
for r in trace[i0:i1]:
    nm = short(r["Kernel_Name"])
    if "rocclr" in nm or "__amd" in nm:
        continue
    a, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    wg = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]))
    tl.append(f"| {nm} | {r['Queue_Id']} | {a:.1f} | {e:.1f} | {e - a:.1f} | {wg} |")
    if nm.startswith("k_fet_window") and first_win is None:
        first_win = a
    scan_end = max(scan_end, e)
tl += ["", f"First window kernel starts {first_win:.1f} us into the scan; the scan's kernels end at {scan_end:.1f} us."]
(dst / f"{R}_fet_timeline.md").write_text("\n".join(tl) + "\n")

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
need(fetch, ["k_fet_setup", "k_bounds", "k_fet_window_fast"], "pmc_fetch")
scans = nf["k_fet_setup"]
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
need(valu, ["k_fet_setup", "k_bounds", "k_fet_window_fast"], "pmc_valu")
vscans = nv["k_fet_setup"]
vk = {k: v for k, v in valu.items() if k.startswith(FET_KERNELS)}
valu_doc = {
    "config": config,
    "valu_wave_insts_per_scan": sum(v["SQ_INSTS_VALU"] for v in vk.values()) / vscans,
    "scans": vscans,
    "method": "rocprofv3 --pmc SQ_INSTS_VALU (+ SQ cycle counters) over the FET scan kernels (wave-instructions)",
    "per_kernel_per_scan": {k: {c: v.get(c, 0.0) / vscans for c in SQ + ("GRBM_GUI_ACTIVE",)}
                            for k, v in sorted(vk.items())},
    "valu_busy": {k: valu_busy({c: v.get(c, 0.0) / vscans for c in SQ + ("GRBM_GUI_ACTIVE",)})
                  for k, v in sorted(vk.items())},
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
                    "per_kernel_per_dispatch": {k: {c: per[k].get(c, 0.0) / nd[k] for c in SQ + ("GRBM_GUI_ACTIVE",)}
                                                for k in kernels},
                    "valu_busy": {k: valu_busy({c: per[k].get(c, 0.0) / nd[k] for c in SQ + ("GRBM_GUI_ACTIVE",)})
                                  for k in kernels}}


c3t = last_json(src / "pmc_c3.txt")
css_entry("c3", src / "pmc_c3", ["k_css_pack", "k_css_mds_h40"], c3t["windows_per_scan"],
          "tools/css_time.py: 20 x 500k SNPs, 20+20, runs=0")
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
for key, mds in (("c3", "k_css_mds_h40"), ("c4", "k_css_mds_t80")):
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
if (src / "ph_c5.err").exists():
    pl = [ln for ln in (src / "ph_c5.err").read_text().splitlines() if ln.startswith("perm-prof cycles:")]
    if not pl:
        raise SystemExit("ph_c5.err: no perm-prof line (was the pprof variant loaded?)")
    body = pl[-1].split(":", 1)[1].replace("(", " ").replace(")", " ").replace(";", " ").replace(":", " ")
    toks = body.split()
    vals = {}
    for i, t in enumerate(toks):
        if t.isdigit():
            vals[toks[i - 1] if toks[i - 1] not in ("matrix",) else "fp16_matrix"] = int(t)
    phase_doc["c5_perm"] = {"phase_cycles": vals, "method": "GD_PERM_PROFILE build (varlib/pprof), tools/css_time.py "
                            "C5 shape; cycles of thread 0 per workgroup, accumulated in registers, summed over "
                            "workgroups; setup = the rest of the window setup after its parts"}
if phase_doc:
    (dst / f"{R}_css_phases.json").write_text(json.dumps(phase_doc, indent=1) + "\n")

# ---- summary
rows = list(csv.DictReader(open(stats)))
lines = [f"# {R} profile summary", "",
         "Commands: tools/profile_round.sh (bench line; per-leg `rocprofv3 --kernel-trace --stats` runs: FET = "
         "`python3 bench.py --steps 5 --warmup 1 --no-cpu --no-css --no-extra`, C3/C4/C5 = tools/css_time.py; PMC "
         "passes in runs of their own).  FET kernels (profiles/" + f"{R}_kernel_stats_fet.csv):", "",
         "| kernel | calls | avg us | total ms |", "|---|---|---|---|"]
for r in rows:
    lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                 f"{float(r['TotalDurationNs']) / 1e6:.2f} |")
alg = bench["roofline"]["alg_bytes_per_step"]
scan_ms = bench["stage_ms"]["scan"]
VPEAK = 1024 * 2.4 / 2  # bench.py VALU_PEAK_GINSTS: one wave64 instruction per SIMD per 2 cycles at 2.4 GHz
fet_gi = valu_doc["valu_wave_insts_per_scan"] / (scan_ms * 1e-3) / 1e9
wbusy = valu_doc["valu_busy"].get("k_fet_window_fast")
lines += ["", f"VALU ceiling used by every fraction (bench.py VALU_PEAK_GINSTS): {VPEAK:.1f} G wave-instructions/s = one "
          "wave64 instruction per SIMD per 2 cycles at the nominal 2.4 GHz (the 2-cycle class).  Measured issue rates per "
          f"op (ubench, 8 waves per SIMD; profiles/{R}_ubench_valu.json): "
          + ", ".join(f"{k} {v:.0f}" for k, v in ginst.items()) + ".",
          "", f"FET scan HBM traffic (PMC): {traffic['bytes_per_scan'] / 1e9:.3f} GB per scan "
          f"(fetch {fetch_b / 1e9:.3f} + write {write_b / 1e9:.3f}); algorithmic B = {alg / 1e9:.3f} GB.",
          "", f"FET scan VALU (PMC SQ_INSTS_VALU): {valu_doc['valu_wave_insts_per_scan'] / 1e9:.3f} G wave-instructions "
          f"per scan = {fet_gi:.0f} G/s at the bench's scan time ({scan_ms:.3f} ms) = {fet_gi / VPEAK:.3f} of the ceiling"
          + (f"; k_fet_window_fast VALU-active share {wbusy:.3f} (4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): "
             "the cycles a wave has a VALU instruction in flight per SIMD-cycle -- pipelined instructions of several "
             "waves overlap, so ~1 means the VALU never waits for work, not a fraction of a ceiling)."
             if wbusy else "."), ""]
for k, v in css_doc.items():
    lines.append(f"CSS {k}: {v['valu_wave_insts_per_window']:.0f} VALU wave-instructions per window "
                 f"({' + '.join(v['kernels'])}); VALU-active share "
                 + ", ".join(f"{kk} {bb:.3f}" for kk, bb in v["valu_busy"].items() if bb is not None) + "."
                 + (f" Matrix cores: {v['mfma']['mfma_per_dispatch'] / 1e6:.1f} M v_mfma_f32_32x32x16_f16 per "
                    f"dispatch, {100 * v['mfma']['frac']:.1f} % of the SIMD-cycles busy." if "mfma" in v else ""))
for k, v in phase_doc.items():
    if k == "c5_perm":
        tot = sum(v["phase_cycles"].values())
        lines.append("CSS c5 permutation phases (share of thread-0 cycles): "
                     + ", ".join(f"{kk} {100 * vv / tot:.1f} %" for kk, vv in v["phase_cycles"].items()) + ".")
        continue
    tot = sum(v["phase_cycles"].values())
    lines.append(f"CSS {k} distance build: k_css_pack {v['pack_us']:.1f} us + popcount D "
                 f"{100 * v['d_share']:.1f} % of the MDS kernel ({v['mds_us']:.1f} us), "
                 f"{v['npos_mean']:.1f} SNP rows per window.  Phases: "
                 + ", ".join(f"{kk} {100 * vv / tot:.1f} %" for kk, vv in v["phase_cycles"].items()) + ".")
if (dst / f"{R}_bench_g2.json").exists():
    g2 = json.loads((dst / f"{R}_bench_g2.json").read_text())
    lines += ["", f"Two-rank rehearsal (--gpus 2, both ranks on the one GPU, {g2['config']['collective_backend']}): "
              f"{g2['value'] / 1e6:.1f} M windows/s over both ranks, {g2['ms_per_step']:.3f} ms/step; cpu_baseline "
              + (f"{g2['cpu_baseline']['value']:.0f} {g2['cpu_baseline']['unit']} ({g2['cpu_baseline']['kind']})"
                 if "cpu_baseline" in g2 else "absent") + "."]
lines += ["", f"One-scan C2 timeline: profiles/{R}_fet_timeline.md."]
lines += ["", "Bench line (same call):", "", "```", json.dumps(bench), "```"]
(dst / f"{R}_summary.md").write_text("\n".join(lines) + "\n")
print("\n".join(lines[:60]))
