"""CPU tests of the drop-in boundary: the built C-ABI library loads and exports
every symbol include/spe.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(spe_[a-z_]+|topology_[A-Za-z_]+)\s*\(", txt)))


def exported(so):
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_libspe_exports_every_declared_symbol():
    so = os.path.join(ROOT, "shadow_amd", "libspe.so")
    assert os.path.exists(so), "run __graft_entry__.build() first"
    ctypes.CDLL(so)
    missing = [s for s in declared("spe.h") if s not in exported(so)]
    assert not missing, missing
    from shadow_amd import spe
    assert sorted(spe.EXPORTS) == declared("spe.h")


def test_device_count_is_callable_without_gpu():
    from shadow_amd import spe
    assert spe.device_count() >= 0


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    from shadow_amd import spe
    monkeypatch.setattr(spe, "LIB_PATH", str(tmp_path / "absent.so"))
    monkeypatch.setattr(spe, "_lib", None)
    with pytest.raises(spe.SpeError):
        spe.lib()
