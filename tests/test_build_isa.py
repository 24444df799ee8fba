"""ISA-level guards on the built gfx950 code objects (CPU: the objects are disassembled, not run).

* No packed-fp32 VALU instructions anywhere (`v_pk_add/mul/fma_f32`): beside another stream's MFMA
  GEMM they returned wrong values in lanes 48-63 of single registers of the LayerNorm backward
  pair (DESIGN §4 "Determinism", profiles/r4g_det_ln_packed.log), so _build.py compiles with the
  `packed-fp32-ops` feature off and this test keeps it that way.
* The LayerNorm kernels' wave reductions use DPP / permlane swaps, not `ds_bpermute` (an LDS round
  trip per step).
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

OBJ = ROOT / "speech_transcript_embeddings_amd" / "_obj"
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _disasm(obj, tmp_path):
    fat = tmp_path / (obj.stem + ".fatbin")
    co = tmp_path / (obj.stem + ".co")
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(obj)], check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}", f"--targets={TARGET}",
                    f"--output={co}"], check=True, capture_output=True)
    r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], check=True, capture_output=True, text=True)
    return r.stdout


def _objects():
    objs = sorted(OBJ.glob("*.o")) if OBJ.exists() else []
    if not objs or shutil.which("objcopy") is None or not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("built objects or ROCm binutils not present")
    return objs


def test_no_packed_fp32_in_any_kernel(tmp_path):
    bad = {}
    for obj in _objects():
        n = len(re.findall(r"\bv_pk_(?:add|mul|fma)_f32\b", _disasm(obj, tmp_path)))
        if n:
            bad[obj.name] = n
    assert not bad, f"packed fp32 instructions in {bad}"


def test_layernorm_reductions_without_bpermute(tmp_path):
    objs = [o for o in _objects() if o.stem == "layernorm"]
    if not objs:
        pytest.skip("layernorm.o not built")
    text = _disasm(objs[0], tmp_path)
    assert "ds_bpermute" not in text
    assert "row_mirror" in text and "permlane32_swap" in text


def test_shipped_library_reads_no_environment():
    """no switch in the shipped libste.so may change numerics from the environment.
    The A/B switches compile to their defaults unless -DSTE_AB (libste_ab.so, _build.py --ab), so
    the default build imports no getenv and carries none of the switch names."""
    lib = ROOT / "speech_transcript_embeddings_amd" / "libste.so"
    if not lib.exists() or shutil.which("nm") is None:
        pytest.skip("libste.so or binutils not present")
    und = subprocess.run(["nm", "-D", "--undefined-only", str(lib)], check=True, capture_output=True,
                         text=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", und), "libste.so imports getenv"
    data = lib.read_bytes()
    names = set(re.findall(rb"STE_[A-Z0-9_]{3,}", data))
    # the only STE_ strings allowed are none at all: every switch name lives in #ifdef STE_AB code
    assert not names, f"switch names in the shipped library: {sorted(names)}"
