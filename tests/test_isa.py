"""CPU checks of the gfx950 code libmpcd.so ships (no GPU): two code-generation pitfalls this build hit.

1. Packed-math reads of transcendental results ("Codegen hazards"). With the GroupNorm+Mish
   epilogue of csrc/unet_mx.hip SLP-packed by hipcc, the conv kernels gave wrong outputs on the GPU
   (tests/test_gpu_unet_bench_sizes.py, bit-identity across tilings, failed with -DMPCD_MX_NO_FENCE and passed
   with the fence or with -fno-slp-vectorize: tools/hazard_ab.sh, profiles/r3_hazard_ab.txt). The only code
   difference: 432 sites where a v_pk_fma_f32 reads a v_rcp_f32 result one wait state after it. The U-Net
   same pattern sat in the MLP samplers' Mish epilogues (626 sites in round 3); every kernel of the library must
   keep every packed reader of a transcendental result at >= 2 wait states.
2. `__builtin_bit_cast` of an element of a builtin's ext-vector result reads element 0 (clang, ROCm 7.2):
   the permlane-swap reductions of csrc/unet_fused.hip copy the element to a scalar first."""
import glob
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(ROOT, "mpc_via_diffusion_model_amd", "libmpcd.so")
LLVM = "/opt/rocm/lib/llvm/bin"
HIPCC = "/opt/rocm/bin/hipcc"
sys.path.insert(0, os.path.join(ROOT, "tools", "isa"))


def _disassemble(tmp_path):
    objdump = os.path.join(LLVM, "llvm-objdump")
    if not (os.path.exists(LIB) and os.path.exists(objdump)):
        pytest.skip("libmpcd.so or llvm-objdump not present")
    so = tmp_path / "libmpcd.so"
    shutil.copy(LIB, so)
    subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
    text = []
    for co in sorted(glob.glob(str(tmp_path / "libmpcd.so.*gfx950"))):
        r = subprocess.run([objdump, "-d", co], check=True, capture_output=True, text=True)
        text.append(r.stdout)
    assert text, "no gfx950 code object in libmpcd.so"
    return "\n".join(text).splitlines()


def test_every_kernel_keeps_packed_reads_of_transcendentals_two_wait_states_away(tmp_path):
    """Every kernel of the shipped code object: the MLP samplers (mlp_h2_kernel, the cfg1 / cfg2 headline kernel; the
    split-bf16 mlp_rw_kernel and mlp_x3_kernel, the exact-fp32 mlp_sample_kernel), the layer-by-layer and fused
    U-Nets, the prologues, the rollout and the training kernels."""
    import trans_hazard as th
    sites = th.scan(_disassemble(tmp_path))
    kernels = {s[0] for s in sites if s[0]}
    for k in ("unet_fused_kernel", "conv_mx_kernel", "mlp_h2_kernel", "mlp_rw_kernel", "mlp_x3_kernel", "mlp_sample_kernel"):
        assert any(k in n for n in kernels), f"{k} not found in the code object"
    packed = [s for s in sites if s[4]]
    close = [s for s in packed if s[3] < 2]
    assert not close, (f"{len(close)} packed reads of a transcendental result under 2 wait states in "
                       f"{len({s[0] for s in close})} kernels: {close[:3]}")
    assert any("unet_fused_kernel" in s[0] for s in packed), \
        "the fused U-Net's packed Mish should read exp / rcp results (pattern not found: scan broken?)"


def test_every_mfma_source_two_wait_states_after_a_valu_write(tmp_path):
    """csrc/mlp_rw.hip and csrc/mlp_h2.hip issue MFMAs with AGPR weight operands as inline asm, which the compiler's
    hazard pass does not treat as MFMAs: no MFMA of the library may read a register a VALU op wrote under 2 wait
    states before."""
    import mfma_hazard as mh
    lines = _disassemble(tmp_path)
    for k in ("mlp_rw_kernel", "mlp_h2_kernel"):
        assert any(k in ln for ln in lines), f"{k} not found in the code object"
    assert any("v_mfma" in ln and ", a[" in ln for ln in lines), "no MFMA with AGPR operands (resident weights?)"
    bad = mh.scan(lines)
    assert not bad, f"{len(bad)} MFMA sources written by a VALU op under 2 wait states: {bad[:3]}"


@pytest.mark.parametrize("op,kernel", [("v_mfma_f32_16x16x32_bf16", "mlp_rw_kernel"),
                                       ("v_mfma_f32_16x16x32_f16", "mlp_h2_kernel")])
def test_asm_mfma_results_wait_before_valu_reads(tmp_path, op, kernel):
    """The other direction for the inline-asm MFMAs (AGPR operands; csrc/mlp_rw.hip bf16, csrc/mlp_h2.hip f16): a VALU
    op may read an MFMA result - or overwrite it (write after write; in these in-place chains also the write after
    the in-flight MFMA's srcC read) - only as many wait states after it as hipcc leaves after the builtin form of the
    same opcode (its minimum over the whole library is the toolchain's requirement: 8 today for both, which the asm
    statements write out as s_nop 7). If a toolchain raises that requirement, the asm waits fall under it and this
    fails."""
    import mfma_hazard as mh
    lines = _disassemble(tmp_path)
    acc = mh.result_reads(lines)
    rs = [r for r in acc if r[1].startswith(op)]
    builtin = [r for r in rs if ", a[" not in r[1]]
    asm = [r for r in rs if ", a[" in r[1]]
    assert builtin and asm, f"expected both builtin and AGPR-operand {op} MFMAs"
    assert any(kernel in r[0] for r in asm), f"no AGPR-operand {op} in {kernel}"
    req = min(r[3] for r in builtin if r[4] == "read")
    assert req == 8, f"hipcc's own wait after {op} is now {req} (was 8): revisit the asm statements' s_nop 7"
    close = [r for r in asm if r[3] < req]
    assert not close, (f"{len(close)} VALU accesses of an asm {op} result under {req} wait states "
                       f"(reads {sum(r[4] == 'read' for r in close)}, writes {sum(r[4] == 'write' for r in close)}): "
                       f"{close[:3]}")


@pytest.mark.parametrize("op", ["v_mfma_f32_16x16x32_bf16", "v_mfma_f32_16x16x32_f16"])
def test_result_scan_reports_close_reads_and_writes(op):
    import mfma_hazard as mh
    asm = ["_Z1kv:", f"  {op} v[28:31], a[20:23], v[0:3], v[28:31]", "  s_nop 3",
           "  v_mov_b32_e32 v29, v33",
           f"  {op} v[8:11], a[20:23], v[0:3], v[8:11]", "  s_nop 1",
           "  v_add_f32_e32 v40, v9, v9"]
    got = [(r[2].split()[0], r[3], r[4]) for r in mh.result_reads(asm)]
    assert got == [("v_mov_b32_e32", 4, "write"), ("v_add_f32_e32", 2, "read")], got


def test_mfma_scan_finds_a_close_valu_write():
    import mfma_hazard as mh
    asm = ["_Z1kv:", "  v_mov_b32_e32 v31, v33", "  v_mfma_f32_16x16x32_bf16 v[28:31], a[20:23], v[0:3], v[28:31]",
           "  v_mov_b32_e32 v2, v33", "  s_nop 1", "  v_mfma_f32_16x16x32_bf16 v[28:31], a[20:23], v[0:3], v[28:31]",
           "  v_mov_b32_e32 v40, v33", "  v_mfma_f32_16x16x32_bf16 v[28:31], a[20:23], v[0:3], v[28:31]"]
    assert [(b[2].split()[1], b[3]) for b in mh.scan(asm)] == [("v31,", 0), ("v2,", 2)][:1]


def test_scan_finds_the_one_wait_state_pattern():
    import trans_hazard as th
    asm = ["_Z1kv:", "  v_rcp_f32_e32 v25, v25", "  s_nop 0", "  v_pk_fma_f32 v[24:25], v[24:25], -2.0, 1.0",
           "  v_rcp_f32_e32 v27, v27", "  s_nop 1", "  v_pk_fma_f32 v[26:27], v[26:27], -2.0, 1.0",
           "  v_exp_f32_e32 v30, v30", "  v_add_f32_e32 v31, v30, v30"]
    sites = th.scan(asm)
    assert [(s[3], s[4]) for s in sites] == [(1, True), (2, True), (0, False)]


def test_bit_cast_of_builtin_vector_element_reads_element_zero(tmp_path):
    """Evidence for the csrc/unet_fused.hip xor16_sum / xor32_sum workaround: r[0] + bit_cast(r[1]) compiles to
    r[0] + r[0]; copying r[1] to an unsigned first keeps both results of the swap."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not present")
    src = tmp_path / "k.hip"
    src.write_text(
        "#include <hip/hip_runtime.h>\n"
        "__global__ void bad(float *o, const float *in) {\n"
        "  const unsigned u = __builtin_bit_cast(unsigned, in[threadIdx.x]);\n"
        "  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);\n"
        "  o[threadIdx.x] = __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);\n"
        "}\n"
        "__global__ void good(float *o, const float *in) {\n"
        "  const unsigned u = __builtin_bit_cast(unsigned, in[threadIdx.x]);\n"
        "  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);\n"
        "  const unsigned a = r[0], b = r[1];\n"
        "  o[threadIdx.x] = __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b);\n"
        "}\n")
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", str(out), str(src)],
                   check=True, capture_output=True)
    asm = out.read_text()

    def adds(kernel):
        body = asm.split(f"{kernel}:", 1)[1].split("s_endpgm", 1)[0]
        return [ln.split()[1:] for ln in body.splitlines() if ln.strip().startswith("v_add_f32")]

    (bad,) = adds("_Z3badPfPKf")
    (good,) = adds("_Z4goodPfPKf")
    assert bad[1].rstrip(",") == bad[2], f"the miscompile is gone ({bad}): the workaround can be dropped"
    assert good[1].rstrip(",") != good[2], good
