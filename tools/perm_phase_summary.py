"""profiles/<R>_perm_phase_counters.json from tools/perm_phase_pmc.sh: the permutation kernel's
SQ counters per dispatch in the four diagnostic builds (PERM_DIAG_NOEXIT; PERM_DIAG_SKIP 0 / 4 /
6 / 7) and each phase's share by differences.  usage: python tools/perm_phase_summary.py r05"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
R = sys.argv[1] if len(sys.argv) > 1 else "r05"
src = ROOT / "gpurun_out" / "pphase"
res, ms = {}, {}
for n in ("all", "nos", "noc", "nod"):
    f = glob.glob(str(src / f"pmc_{n}" / "**" / "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counters for {n}")
    agg, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(f[0])):
        if "k_css_perm<80>" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    if not disp:
        raise SystemExit(f"{n}: k_css_perm<80> absent")
    res[n] = {k: v / len(disp) for k, v in agg.items()}
    line = [ln for ln in (src / f"pmc_{n}.txt").read_text().splitlines() if ln.startswith("CSS")][0]
    ms[n] = float(line.split("stages [")[1].split(",")[2])  # the permutation stage (HIP events)
phases = {"setup, identity columns, hit count": ("nod", None), "Fisher-Yates draws": ("noc", "nod"),
          "compositions": ("nos", "noc"), "scores": ("all", "nos")}
keys = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT")
doc = {"kernel": "k_css_perm<80>", "shape": "tools/css_time.py C5 shape: 1 x 500k SNPs, 40+40, mcT 10, mcR 1000 "
       "(49,967 windows), every window's full 1000 permutations (PERM_DIAG_NOEXIT)",
       "method": "SQ counters per dispatch (rocprofv3 --pmc, one pass per build) of builds that skip phases "
                 "(PERM_DIAG_SKIP: 4 = no scores, 6 = no compositions or scores, 7 = no draws either); a phase's "
                 "figure = the difference of two builds; perm stage time from the HIP events of the same runs",
       "builds": {n: {"counters": res[n], "perm_ms": ms[n]} for n in res}, "phases": {}}
for name, (a, b) in phases.items():
    doc["phases"][name] = {k: res[a][k] - (res[b][k] if b else 0.0) for k in keys}
    doc["phases"][name]["perm_ms"] = ms[a] - (ms[b] if b else 0.0)
    doc["phases"][name]["share"] = {k: doc["phases"][name][k] / res["all"][k] for k in keys}
(ROOT / "profiles" / f"{R}_perm_phase_counters.json").write_text(json.dumps(doc, indent=1) + "\n")
for name, v in doc["phases"].items():
    print(f"{name:38s} " + " ".join(f"{k.replace('SQ_', '')} {100 * v['share'][k]:.0f}%" for k in keys)
          + f"  {v['perm_ms']:.2f} ms")
