"""Pins the gfx950 instruction encodings the XCD-local SMO exchange relies on (smo.hip, the
memory-model note in persist_solve): compiled here on the CPU with hipcc to device assembly.

* records are published with `global_store_dwordx2 ... sc0` (workgroup scope: written through the
  vL1D into the XCD's L2) in the XCD-local solver and `... sc1` (agent scope) in the device-wide one;
* the pollers read them with `global_load_dwordx2 ... sc1` (agent scope: served by the L2, never a
  stale vL1D line).
If a compiler or header change moves these bits, the exchange's correctness argument no longer
holds and this test fails before any GPU run."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

PKG = Path(__file__).resolve().parents[1] / "svm355"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def smo_asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "smo.s"
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only", "-S",
           f"-I{PKG / 'csrc/include'}", f"-I{PKG / 'csrc/hip'}", f"-I{PKG / 'csrc/cascade'}",
           str(PKG / "csrc/hip/smo.hip"), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return out.read_text()


def _kernel(asm: str, xlocal: bool) -> str:
    flag = "Lb1E" if xlocal else "Lb0E"
    names = re.findall(rf"^(_Z\w*smo_persistent_kernelILi512ELi4ELb0E{flag}\w*):", asm, re.M)
    assert names, "smo_persistent_kernel<512, 4, false, XLOCAL> not found"
    i = asm.index(names[0] + ":")
    return asm[i: asm.index(".Lfunc_end", i)]


def _record_stores(body: str):
    # the record publication: a 64-bit store addressed from an SGPR base (rec + g * stride)
    return [l.strip() for l in body.splitlines() if re.search(r"global_store_dwordx2 v\d+, v\[\d+:\d+\], s\[", l)]


def test_xcd_local_records_are_workgroup_scope_stores(smo_asm):
    st = _record_stores(_kernel(smo_asm, True))
    assert st and all(s.endswith(" sc0") for s in st), st


def test_device_wide_records_are_agent_scope_stores(smo_asm):
    st = _record_stores(_kernel(smo_asm, False))
    assert st and all(s.endswith(" sc1") for s in st), st


def test_record_polls_are_agent_scope_loads(smo_asm):
    for x in (True, False):
        loads = [l for l in _kernel(smo_asm, x).splitlines() if "global_load_dwordx2" in l and " sc1" in l]
        assert loads, "no agent-scope (sc1) 64-bit poll loads"
