"""CPU checks of the drop-in boundary: the HIP library loads, exports every
symbol include/partisan_gpu_sim.h declares, and the ctypes mirror matches the
C struct layout (no compute calls: there may be no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from partisan_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "partisan_gpu_sim.h")
LIB = os.path.join(ROOT, "partisan_amd", "csrc", "libpartisan_gpu_sim.so")


def declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"\b(psim_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_api():
    names = declared()
    for n in ["psim_create", "psim_destroy", "psim_step", "psim_join", "psim_crash",
              "psim_broadcast", "psim_get_nodes", "psim_set_partition"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r"\bT (psim_\w+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_library_loads_and_reports_abi():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    lib = C.CDLL(LIB)
    assert lib.psim_abi_version() == _abi.PSIM_ABI_VERSION
    lib.psim_strerror.restype = C.c_char_p
    assert lib.psim_strerror(-5) == b"node id out of range"
    cfg = _abi.PsimConfig()
    lib.psim_default_config(C.byref(cfg))
    assert (cfg.max_active_size, cfg.max_passive_size, cfg.arwl, cfg.prwl) == (6, 30, 5, 30)


def test_struct_layout_matches_header(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n'
        'int main(){printf("%%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu %%zu\\n", sizeof(psim_config),'
        'sizeof(psim_round_stats), sizeof(psim_node_view), offsetof(psim_config, comm_id),'
        'offsetof(psim_node_view, have), offsetof(psim_round_stats, digest),'
        'sizeof(psim_strategy_view), offsetof(psim_config, fanout),'
        'offsetof(psim_strategy_view, members_hash), sizeof(psim_histograms),'
        'offsetof(psim_histograms, components));return 0;}\n' % HDR)
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-o", str(exe), str(prog)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [C.sizeof(_abi.PsimConfig), C.sizeof(_abi.PsimRoundStats), C.sizeof(_abi.PsimNodeView),
            _abi.PsimConfig.comm_id.offset, _abi.PsimNodeView.have.offset,
            _abi.PsimRoundStats.digest.offset, C.sizeof(_abi.PsimStrategyView),
            _abi.PsimConfig.fanout.offset, _abi.PsimStrategyView.members_hash.offset,
            C.sizeof(_abi.PsimHistograms), _abi.PsimHistograms.components.offset]
    assert got == want


def test_oracle_mirrors_abi():
    from _oracle import load
    lib = load()
    for name in _abi.SIGNATURES:
        assert hasattr(lib, "orc_" + name)
