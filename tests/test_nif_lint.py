"""A compile check of the Erlang NIF shim (erlang/c_src/partisan_gpu_sim_nif.c)
in an image without Erlang: the C source is compiled with -Wall -Werror
against tests/nif_lint/erl_nif.h (a restatement of the erl_nif prototypes it
uses) and the product header, and every psim_ symbol the object needs must be
one the HIP library exports.  A lint of this repository's code only -- not a
build of the reference, and not proof that the real erl_nif.h agrees."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "erlang", "c_src", "partisan_gpu_sim_nif.c")
LIB = os.path.join(ROOT, "partisan_amd", "csrc", "libpartisan_gpu_sim.so")


def _compile(tmp_path, *extra):
    obj = tmp_path / "nif.o"
    cmd = ["gcc", "-std=c11", "-O2", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Werror",
           "-I", os.path.join(ROOT, "tests", "nif_lint"), "-I", os.path.join(ROOT, "include"),
           "-c", SRC, "-o", str(obj)] + list(extra)
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return obj


def test_nif_compiles_cleanly(tmp_path):
    _compile(tmp_path)


def test_nif_symbols_resolve_against_the_library(tmp_path):
    obj = _compile(tmp_path)
    und = subprocess.check_output(["nm", "-u", str(obj)]).decode()
    need = sorted(set(re.findall(r"\b(psim_\w+)", und)))
    assert "psim_step" in need and "psim_set_bucket_table" in need
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    have = set(re.findall(r"\bT (psim_\w+)", subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()))
    assert not [n for n in need if n not in have]
    enif = sorted(set(re.findall(r"\b(enif_\w+)", und)))
    assert "enif_get_resource" in enif


def test_nif_exports_every_erlang_stub():
    """Each `*_nif`/NIF name partisan_gpu_sim.erl stubs with nif_error is in
    the shim's function table with the same arity."""
    erl = open(os.path.join(ROOT, "erlang", "src", "partisan_gpu_sim.erl")).read()
    stubs = set()
    for name, args in re.findall(r"^(\w+)\(([^)]*)\)\s*->\s*erlang:nif_error", erl, re.M):
        stubs.add((name, 0 if not args.strip() else args.count(",") + 1))
    c = open(SRC).read()
    table = {(n, int(a)) for n, a in re.findall(r'\{"(\w+)",\s*(\d+),\s*nif_\w+', c)}
    assert stubs and stubs <= table, sorted(stubs - table)
