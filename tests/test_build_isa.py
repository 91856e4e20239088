"""ISA-level guard on the built library (CPU, no GPU needed).

Round 3 root cause of the non-deterministic two-process frame: k_lbs_skin's
SLP-vectorised blend ran on packed-FP32 VALU (v_pk_mul_f32 op_sel_hi:[0,1] feeding a dependent
v_pk_add_f32 with no wait state between them), and one 16-lane pass of a wave intermittently
computed a wrong skinned y coordinate when other work shared the GPU. The Makefile now builds
every kernel without packed-FP32 instructions; this test disassembles every gfx950 code object in
libapn_hip.so and fails if any packed-FP32 VALU instruction is back.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "articulated-point-nerf_amd", "apn_amd", "libapn_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# every packed VALU form on 32-bit lanes (v_pk_add/mul/fma_f32 and the packed moves beside them):
# none is emitted today, and any that reappears is a candidate for the same missing wait state
PACKED_F32 = re.compile(r"\bv_pk_\w+_(f32|b32)\b")
LIBS = [LIB, os.path.join(os.path.dirname(LIB), "libapn_hip_debug.so")]


def _disassemble_device_code(lib):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not all(os.path.exists(t) for t in tools):
        pytest.skip("ROCm LLVM tools not found")
    objcopy, bundler, objdump = tools
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fatbin")
        subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", lib], check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        assert starts, "no offload bundle in .hip_fatbin"
        for i, s in enumerate(starts):
            chunk = data[s:starts[i + 1] if i + 1 < len(starts) else len(data)]
            src, co = os.path.join(d, f"b{i}"), os.path.join(d, f"b{i}.co")
            with open(src, "wb") as f:
                f.write(chunk)
            subprocess.run([bundler, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--input={src}", f"--output={co}"], check=True, capture_output=True)
            if os.path.getsize(co) == 0:
                continue
            out.append(subprocess.run([objdump, "-d", co], check=True, capture_output=True, text=True).stdout)
    return out


@pytest.mark.parametrize("lib", LIBS, ids=["product", "debug"])
def test_no_packed_fp32_valu_in_device_code(lib):
    if not os.path.exists(lib):
        pytest.skip(f"{os.path.basename(lib)} not built")
    texts = _disassemble_device_code(lib)
    assert len(texts) >= 10, len(texts)                       # one code object per .hip source
    allcode = "\n".join(texts)
    assert "v_mfma_f32_16x16x32_f16" in allcode                # really the MLP kernels' ISA
    bad = [ln.strip() for ln in allcode.splitlines() if PACKED_F32.search(ln)]
    assert not bad, f"{len(bad)} packed-FP32 VALU instructions, e.g. {bad[:3]}"
