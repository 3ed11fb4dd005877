"""Turn a tools/profile_round.sh output directory into the committed profiles/ files:
  profiles/<R>_kernel_stats.csv   rocprofv3 --stats summary of the bench command
  profiles/<R>_bench.json         the bench line measured in the same call
  profiles/<R>_fet_traffic.json   HBM bytes per FET scan from the PMC passes
  profiles/<R>_fet_valu.json      VALU wave-instructions per FET scan (SQ_INSTS_VALU)
  profiles/<R>_summary.md         per-kernel averages, per-scan traffic, cross-checks
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
R = sys.argv[1] if len(sys.argv) > 1 else "r02"
src = ROOT / "gpurun_out" / R
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)

FET_KERNELS = ("k_popsize", "k_bounds", "k_snp_fet", "k_fet_")


def short(name):
    return name.split("(")[0].replace("void ", "")


def find(d, suffix):
    hits = sorted(Path(d).rglob(f"*{suffix}"))
    return hits[0] if hits else None


def counters(d, counter):
    f = find(d, "counter_collection.csv")
    per = defaultdict(float)
    n = defaultdict(int)
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] != counter:
            continue
        k = short(row["Kernel_Name"])
        per[k] += float(row["Counter_Value"])
        n[k] += 1
    return per, n


stats = find(src / "ktrace", "kernel_stats.csv")
shutil.copy(stats, dst / f"{R}_kernel_stats.csv")
bench = json.loads((src / "bench.json").read_text().strip().splitlines()[-1])
(dst / f"{R}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")

fetch, nf = counters(src / "pmc_fetch", "FETCH_SIZE")
write, nw = counters(src / "pmc_write", "WRITE_SIZE")
scans = nf.get("k_popsize", 0)
fk = {k: v for k, v in fetch.items() if k.startswith(FET_KERNELS)}
wk = {k: v for k, v in write.items() if k.startswith(FET_KERNELS)}
# rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB; gfx950 FETCH_SIZE counts half of
# a wide coalesced read (MI355X_MICROARCH.md, HBM section): double it
fetch_b = 2 * 1024 * sum(fk.values()) / scans
write_b = 1024 * sum(wk.values()) / scans
cfg = bench["config"]
traffic = {
    "config": [cfg["chromosomes_per_gpu"], cfg["snps_per_gpu"] // cfg["chromosomes_per_gpu"], cfg["asize"],
               cfg["bsize"]],
    "bytes_per_scan": fetch_b + write_b,
    "fetch_bytes_per_scan": fetch_b,
    "write_bytes_per_scan": write_b,
    "scans": scans,
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the FET scan kernels; "
              "KiB -> bytes, FETCH_SIZE x2 (gfx950 wide-read correction)",
    "per_kernel_kib_per_scan": {k: {"fetch": fk.get(k, 0) / scans, "write": wk.get(k, 0) / scans}
                                for k in sorted(set(fk) | set(wk))},
}
(dst / f"{R}_fet_traffic.json").write_text(json.dumps(traffic, indent=1) + "\n")

valu, nv = counters(src / "pmc_valu", "SQ_INSTS_VALU")
vscans = nv.get("k_popsize", 0)
vk = {k: v for k, v in valu.items() if k.startswith(FET_KERNELS)}
valu_doc = {
    "config": traffic["config"],
    "valu_wave_insts_per_scan": sum(vk.values()) / vscans,
    "scans": vscans,
    "method": "rocprofv3 --pmc SQ_INSTS_VALU over the FET scan kernels (wave-instructions)",
    "per_kernel_per_scan": {k: v / vscans for k, v in sorted(vk.items())},
}
(dst / f"{R}_fet_valu.json").write_text(json.dumps(valu_doc, indent=1) + "\n")

# CSS (C3 shape): VALU wave-instructions per call of the bit-plane pass and the m = 40 MDS kernel
cval, ncv = counters(src / "pmc_css_valu", "SQ_INSTS_VALU")
mds = [k for k in cval if k.startswith("k_css_mds<40")]
css_doc = None
if mds and ncv.get("k_css_pack", 0):
    per_call = cval[mds[0]] / ncv[mds[0]] + cval["k_css_pack"] / ncv["k_css_pack"]
    css_doc = {"config": traffic["config"], "valu_wave_insts_per_scan": per_call,
               "method": "rocprofv3 --pmc SQ_INSTS_VALU over k_css_pack + k_css_mds<40, 1> (wave-instructions "
                         "per call = per C3 scan)"}
    (dst / f"{R}_css_valu.json").write_text(json.dumps(css_doc, indent=1) + "\n")

# CSS permutations (C5 shape, tools/css_time.py): SQ counters of k_css_perm per dispatch
perm_doc = None
if (src / "pmc_perm").exists():
    pc = defaultdict(float)
    pd = set()
    for row in csv.DictReader(open(find(src / "pmc_perm", "counter_collection.csv"))):
        if short(row["Kernel_Name"]).startswith("k_css_perm"):
            pc[row["Counter_Name"]] += float(row["Counter_Value"])
            pd.add(row["Dispatch_Id"])
    if pd:
        per = {k: v / len(pd) for k, v in pc.items()}
        perm_doc = {"config": "1 chromosome x 500000 SNPs, 40+40, mcT=10, mcR=1000 (tools/css_time.py)",
                    "per_dispatch": per,
                    "method": "rocprofv3 --pmc SQ_* over k_css_perm<80> (one dispatch per scan)"}
        (dst / f"{R}_perm_pmc.json").write_text(json.dumps(perm_doc, indent=1) + "\n")

rows = list(csv.DictReader(open(stats)))
lines = [f"# {R} profile summary", "", "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 "
         "--warmup 1 --no-cpu` (FET + CSS legs), PMC passes separate (tools/profile_round.sh).", "",
         "| kernel | calls | avg us | total ms |", "|---|---|---|---|"]
for r in rows:
    lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                 f"{float(r['TotalDurationNs']) / 1e6:.2f} |")
alg = bench["roofline"]["alg_bytes_per_step"]
lines += ["", f"FET scan HBM traffic (PMC): {traffic['bytes_per_scan'] / 1e9:.3f} GB per scan "
          f"(fetch {fetch_b / 1e9:.3f} + write {write_b / 1e9:.3f}); algorithmic B = {alg / 1e9:.3f} GB.",
          "", f"FET scan VALU (PMC SQ_INSTS_VALU): {valu_doc['valu_wave_insts_per_scan'] / 1e9:.3f} G wave-instructions "
          f"per scan; at the bench's scan time that is {valu_doc['valu_wave_insts_per_scan'] / (bench['roofline']['stage_ms']['scan_total'] * 1e-3) / 1e9:.0f} "
          "G/s of the 614 G/s issue peak (256 CUs x 4 SIMDs x 2.4 GHz / 4).",
          "", "Bench line (same call):", "", "```", json.dumps(bench), "```"]
if perm_doc:
    lines[-5:-5] = ["", "k_css_perm<80> per dispatch (PMC): " + ", ".join(
        f"{k} {v:.4g}" for k, v in sorted(perm_doc["per_dispatch"].items()))]
(dst / f"{R}_summary.md").write_text("\n".join(lines) + "\n")
print("\n".join(lines[:40]))
