"""One line per FET bench JSON: ms/step and stage times.  python tools/fetsum.py gpurun_out/sN"""
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        s = d.get("stage_ms") or d["roofline"]["stage_ms"]
        print(f"{f.split('/')[-1]:28s} {d['ms_per_step']:.4f} ms/step  mem {s['hbm_passes_done']:.4f} "
              f"win {s['fast_windows_done']:.4f} gen {s['general_path']:.4f} total {s['scan_total']:.4f}")
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
