"""CPU checks of the C-ABI boundary: layout and exported symbols (no GPU calls)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from crgc_hip import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "crgc.h")


def _declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(crgc_\w+)\s*\(", src, re.M)))


def test_header_declares_exactly_the_exported_list():
    assert _declared_functions() == sorted(abi.EXPORTED_SYMBOLS)


def test_struct_layout_matches_c_compiler(tmp_path):
    prog = tmp_path / "sz.c"
    structs = ["crgc_config", "crgc_entry_batch", "crgc_delta_batch", "crgc_undo_log",
               "crgc_trace_stats", "crgc_trace_out", "crgc_graph_export", "crgc_usage"]
    prog.write_text('#include <stdio.h>\n#include "%s"\nint main(void){%s return 0;}\n' % (
        HEADER, "".join('printf("%%zu\\n", sizeof(%s));' % s for s in structs)))
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(prog)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    py = [C.sizeof(t) for t in (abi.CrgcConfig, abi.CrgcEntryBatch, abi.CrgcDeltaBatch,
                                abi.CrgcUndoLog, abi.CrgcTraceStats, abi.CrgcTraceOut,
                                abi.CrgcGraphExport, abi.CrgcUsage)]
    assert sizes == py


def test_library_loads_and_exports_every_declared_symbol():
    if not os.path.exists(abi.LIB_PATH):
        pytest.fail("libcrgc_hip.so not built; run `python __graft_entry__.py build`")
    lib = abi.load_library()
    for name in _declared_functions():
        assert hasattr(lib, name), name
    assert lib.crgc_strerror(abi.E_NULL_SUPERVISOR).startswith(b"local garbage")
    # no call has failed on this thread: the failure detail is empty, and a
    # CrgcError carries it when there is one
    assert lib.crgc_last_error_detail() == b"" and abi.last_error_detail() == ""
    e = abi.CrgcError(abi.E_DEVICE, "crgc_merge_entries", "crgc_api.hip:1234: hipErrorLaunchFailure")
    assert "CRGC_E_DEVICE" in str(e) and e.detail.endswith("hipErrorLaunchFailure")


def test_library_is_gfx950_only(tmp_path):
    # --offloading extracts the code objects next to its input: work on a copy
    import shutil
    lib = tmp_path / "libcrgc_hip.so"
    shutil.copy(abi.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True).stdout
    arches = set(re.findall(r"gfx\d+", out))
    assert arches == {"gfx950"}, arches


def test_product_does_not_reference_the_oracle():
    pkg = os.path.join(REPO, "uigc-akka_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                text = open(os.path.join(root, f)).read()
                assert "oracle" not in text.lower(), \
                    f"{f} mentions the oracle"
