"""Time the device-resident CSS scan on C3-shaped synthetic data (diagnostics)."""
import os, sys, time
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd"))
import torch
from gdscan import _lib, synth
from gdscan._lib import Chrom, check, lib

nch = int(os.environ.get("NCH", 20)); nsnp = int(os.environ.get("NSNP", 500_000))
a = b = int(os.environ.get("POP", 20)); runs = int(os.environ.get("RUNS", 0)); tres = int(os.environ.get("TRES", 10))
steps = int(os.environ.get("STEPS", 3))
dev = torch.device("cuda", 0)
alen, blen = nsnp * a, nsnp * b
av = torch.empty(nch * alen, dtype=torch.float64, device=dev); bv = torch.empty(nch * blen, dtype=torch.float64, device=dev)
ap = torch.empty(nch * alen, dtype=torch.int32, device=dev); bp = torch.empty(nch * blen, dtype=torch.int32, device=dev)
q = torch.from_numpy(synth.freq_table()).to(dev)
st = torch.cuda.current_stream().cuda_stream
for c in range(nch):
    check(lib.gd_synth_device(c, nsnp, a, b, synth.MASTER_SEED, q.data_ptr(), av.data_ptr() + c * alen * 8,
                              bv.data_ptr() + c * blen * 8, ap.data_ptr() + c * alen * 4, bp.data_ptr() + c * blen * 4, st))
torch.cuda.synchronize()
last = ap.view(nch, alen)[:, -1].cpu().numpy()
ch = (Chrom * nch)(); w = 0; nwin = 0
for c in range(nch):
    regend = int(last[c]) + 1
    ch[c].a_off, ch[c].b_off, ch[c].alen, ch[c].blen, ch[c].regend, ch[c].w_out, ch[c].seed = c * alen, c * blen, alen, blen, regend, w, 7 + c
    w += regend // 500; nwin += lib.gd_window_count(regend, 2500, 500, 0)
sc = torch.zeros(w, dtype=torch.float64, device=dev); pv = torch.zeros_like(sc)
ctx = lib.gd_ctx_create(0)
def step():
    check(lib.gd_css_scan_device(ctx, ch, nch, av.data_ptr(), bv.data_ptr(), ap.data_ptr(), bp.data_ptr(), 2500, 500,
                                 tres, runs, 0, sc.data_ptr(), pv.data_ptr(), st))
step(); torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / steps
print(f"CSS {nch}x{nsnp} {a}+{b} runs={runs}: {nwin} windows, {dt*1e3:.2f} ms/step, {nwin/dt/1e6:.2f} M windows/s, stages {_lib.last_stage_ms()}")
s = sc.cpu().numpy(); print("computed", (s != 0).sum(), "nan", np.isnan(s).sum(), "mean p", pv.cpu().numpy()[s != 0].mean())
import json
# mean SNP rows per window of the 2500 / 500 grid (the distance build's npos)
npw = []
for c in range(nch):
    pos = ap[c * alen:(c + 1) * alen:a].cpu().numpy()
    st0 = np.arange(0, int(last[c]) + 1, 500)
    k = np.searchsorted(pos, st0 + 2500) - np.searchsorted(pos, st0)
    npw.append(k[k > 0])
npos_mean = float(np.concatenate(npw).mean())
print(json.dumps({"css_time": True, "npos_mean": npos_mean, "nch": nch, "nsnp": nsnp, "pop": a, "runs": runs, "treshold": tres,
                  "windows_per_scan": int(nwin), "scans": steps + 1, "ms_per_step": dt * 1e3}))
