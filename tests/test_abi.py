"""CPU: the C-ABI library loads and exports every symbol include/gdscan.h declares
(no compute calls without a GPU); the reference-name compat libraries export the
reference's symbols."""
import ctypes
import re
import subprocess

import pytest

from conftest import PKG, ROOT


def header_symbols():
    text = (ROOT / "include" / "gdscan.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gd_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header():
    from gdscan import _lib
    syms = header_symbols()
    assert "gd_fet_threadcompute" in syms and "gd_css_scan_device" in syms
    assert sorted(_lib.EXPORTS) == syms
    for s in syms:
        assert hasattr(_lib.lib, s), s


@pytest.mark.parametrize("name", ["libgdscan_fisher.so", "libgdscan_css.so"])
def test_compat_libraries_export_reference_names(name):
    path = PKG / "lib" / name
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True, check=True).stdout
    assert " T threadcompute" in out and " T compute" in out
    ctypes.CDLL(str(path))


def test_product_has_no_oracle_dependency():
    """The shipped library never links the oracle or the reference."""
    out = subprocess.run(["ldd", str(PKG / "lib" / "libgdscan.so")], capture_output=True, text=True).stdout
    assert "oracle" not in out and "ref_fisher" not in out
    for src in (PKG / "csrc").glob("*"):
        assert "orc_" not in src.read_text(errors="ignore"), src


def test_no_gpu_errors_cleanly():
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from gdscan import GdError, fet
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(0, 3000, 4, 4)
    with pytest.raises(GdError):
        fet.scan(av, bv, ap, bp, regend)


def test_seed_is_per_thread():
    """gd_set_seed (the seed of the reference-signature entry points) affects only the
    calling thread, so two threads that each set a seed and then call fisher_exact_tester
    cannot race on it (no GPU call: set/get only)."""
    import threading
    from gdscan._lib import GD_DEFAULT_SEED, lib
    got = {}
    gate = threading.Barrier(2)

    def worker(name, seed):
        lib.gd_set_seed(seed)
        gate.wait()  # both threads have set their seed before either reads it back
        got[name] = lib.gd_get_seed()

    ts = [threading.Thread(target=worker, args=(k, s)) for k, s in (("a", 11), ("b", 22))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert got == {"a": 11, "b": 22}
    fresh = {}
    t = threading.Thread(target=lambda: fresh.setdefault("s", lib.gd_get_seed()))
    t.start()
    t.join()
    assert fresh["s"] == GD_DEFAULT_SEED
