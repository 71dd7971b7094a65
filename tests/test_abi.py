"""The C-ABI library loads on a GPU-less host and exports every symbol include/brc.h declares;
ctypes layouts match the C structs (checked by compiling a probe against the header)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from byzantinerandomizedconsensus_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "brc.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(brc_\w+)\s*\(", src, re.M)))


def test_header_and_bindings_agree():
    assert declared_functions() == sorted(L.EXPORTS)


def test_library_exports_every_symbol():
    lib = L.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.brc_abi_version() == L.ABI_VERSION


def test_invalid_config_rejected_without_gpu():
    lib = L.load()
    h = ctypes.c_void_p()
    bad = L.Config(n=0, f=0, instances=1, delay_max=1, delay_const=1, key_window=4, variants=1)
    assert lib.brc_create(ctypes.byref(bad), ctypes.byref(h)) == L.E_INVALID
    bad = L.Config(n=257, f=0, instances=1, delay_max=1, delay_const=1, key_window=4, variants=1)
    assert lib.brc_create(ctypes.byref(bad), ctypes.byref(h)) == L.E_INVALID
    bad = L.Config(n=4, f=1, instances=1, delay_max=17, delay_const=1, key_window=4, variants=1)
    assert lib.brc_create(ctypes.byref(bad), ctypes.byref(h)) == L.E_INVALID
    assert not h.value


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "brc.h"
#define S(T) printf(#T " %zu\n", sizeof(T));
#define O(T, F) printf(#T "." #F " %zu\n", offsetof(T, F));
int main(void) {
  S(brc_config) S(brc_injection) S(brc_instance_result) S(brc_replica_result) S(brc_event) S(brc_stats)
  O(brc_config, seed) O(brc_config, byzantine_mask) O(brc_config, device)
  O(brc_injection, instance) O(brc_injection, dst_mask) O(brc_injection, dst_mask_hi) O(brc_event, a) O(brc_instance_result, msgs_sent)
  return 0;
}
"""


def test_struct_layouts_match_header():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "p.c"), os.path.join(d, "p")
        open(src, "w").write(PROBE)
        subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), src, "-o", exe])
        out = dict(line.rsplit(" ", 1) for line in subprocess.check_output([exe]).decode().splitlines())
    sizes = {"brc_config": L.Config, "brc_injection": L.Injection, "brc_instance_result": L.InstanceResult,
             "brc_replica_result": L.ReplicaResult, "brc_event": L.Event, "brc_stats": L.Stats}
    for name, cls in sizes.items():
        assert int(out[name]) == ctypes.sizeof(cls), name
    offs = {"brc_config.seed": L.Config.seed, "brc_config.byzantine_mask": L.Config.byzantine_mask,
            "brc_config.device": L.Config.device, "brc_injection.instance": L.Injection.instance,
            "brc_injection.dst_mask": L.Injection.dst_mask, "brc_injection.dst_mask_hi": L.Injection.dst_mask_hi,
            "brc_event.a": L.Event.a,
            "brc_instance_result.msgs_sent": L.InstanceResult.msgs_sent}
    for name, field in offs.items():
        assert int(out[name]) == field.offset, name


def test_engine_refuses_without_library(monkeypatch, tmp_path):
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(L.EngineUnavailable):
        L.load()


def test_create_failure_reason_is_reported():
    lib = L.load()
    h = ctypes.c_void_p()
    bad = L.Config(n=4, f=1, instances=1, delay_max=1, delay_const=1, key_window=3, variants=1)
    assert lib.brc_create(ctypes.byref(bad), ctypes.byref(h)) == L.E_INVALID
    assert b"invalid configuration" in lib.brc_last_error(None)
