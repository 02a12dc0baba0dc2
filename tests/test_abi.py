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


def test_struct_layouts_match_the_header(tmp_path):
    """Every spe.h struct the ctypes mirror declares has the C size and field
    offsets (the mirror is what the tests and bench.py call through)."""
    from shadow_amd import spe
    structs = {"spe_graph_desc": spe.GraphDesc, "spe_graph_info": spe.GraphInfo, "spe_table_opts": spe.TableOpts,
               "spe_table_layout": spe.TableLayout, "spe_build_stats": spe.BuildStats, "spe_entry": spe.Entry,
               "spe_check_report": spe.CheckReport, "spe_compare_report": spe.CompareReport,
               "spe_kernel_profile": spe.KernelProfile}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "spe.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "sz.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, f"{cname}.{f}"


def test_stale_struct_size_is_refused_without_gpu():
    """The ABI guard: a caller built against another spe.h (struct_size differs)
    gets SPE_EINVAL before anything is read (spe_graph_create checks it first)."""
    from shadow_amd import spe
    d = spe.GraphDesc()
    d.struct_size = ctypes.sizeof(spe.GraphDesc) - 4
    h = ctypes.c_void_p()
    rc = spe.lib().spe_graph_create(ctypes.byref(d), 0, ctypes.byref(h))
    assert rc == -1   # SPE_EINVAL
    assert b"struct_size" in spe.lib().spe_last_error()
