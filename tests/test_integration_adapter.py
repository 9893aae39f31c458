"""INTEGRATION.md section 2 (the MNN Creator / Execution adapter a maintainer adds to the reference)
type-checks against the reference's own headers: Execution (source/core/Execution.hpp:24-82),
CPUBackend::Creator and REGISTER_CPU_OP_CREATOR (source/backend/cpu/CPUBackend.hpp:85-91, :179-183),
the generated schema (schema/current/MNN_generated.h: OpType_NITI_* keys, NITI_CONV_Int8) and this
repository's include/niti_hip.h.  g++ -fsyntax-only: the reference's headers are only parsed, none of
its code is built, linked or run.  Skipped where /root/reference is absent (the GPU box)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/execution-engine"


def adapter_source():
    s = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blk = s[s.index("## 2. Adapter"):]
    code = blk[blk.index("```cpp") + len("```cpp"):]
    return code[:code.index("```")]


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("g++") is None, reason="reference headers or g++ absent")
def test_integration_adapter_type_checks(tmp_path):
    src = tmp_path / "NITI_HipExecution.cpp"
    src.write_text(adapter_source())
    inc = [f"-I{REF}/include", f"-I{REF}/source", f"-I{REF}/schema/current",
           f"-I{REF}/3rd_party/flatbuffers/include", f"-I{ROOT}/include"]
    r = subprocess.run(["g++", "-std=c++11", "-fsyntax-only", *inc, str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_integration_adapter_uses_declared_entry_points():
    """Every niti_* call in the adapter is a function include/niti_hip.h declares."""
    import re

    from niti_amd import _lib
    declared = set(_lib.header_functions())
    header = open(os.path.join(ROOT, "include", "niti_hip.h")).read()
    types = set(re.findall(r"}\s*(niti_[a-z0-9_]+)\s*;", header))  # typedef struct {...} niti_x;
    used = set(re.findall(r"\b(niti_[a-z0-9_]+)\s*\(", adapter_source())) - types
    assert used and used <= declared, used - declared
