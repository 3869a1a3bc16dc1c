"""Generate csrc/jit/gcn_opcodes.inc: gfx950 opcode numbers of every
instruction the baseline program JIT (csrc/jit/gcn_jit.hpp) emits.

Each entry is assembled with the ROCm llvm-mc for gfx950 and the opcode field
is read back out of the encoding for its format, so the table comes from the
assembler itself, never typed by hand.  The encoder test
(tests/test_gcn_jit.py) re-assembles every form through llvm-mc and compares
words with the C++ encoder.

    python tools/gen_gcn_opcodes.py      # rewrites csrc/jit/gcn_opcodes.inc
"""
import os
import re
import subprocess
import sys

MC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin", "llvm-mc")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "jit", "gcn_opcodes.inc")

# (enum name, format, sample)
FORMS = [
    # SOP1
    ("S_MOV_B32", "SOP1", "s_mov_b32 s1, s2"),
    ("S_MOV_B64", "SOP1", "s_mov_b64 s[2:3], s[4:5]"),
    ("S_NOT_B64", "SOP1", "s_not_b64 s[2:3], s[4:5]"),
    ("S_AND_SAVEEXEC_B64", "SOP1", "s_and_saveexec_b64 s[2:3], s[4:5]"),
    ("S_OR_SAVEEXEC_B64", "SOP1", "s_or_saveexec_b64 s[2:3], s[4:5]"),
    ("S_GETPC_B64", "SOP1", "s_getpc_b64 s[2:3]"),
    ("S_SETPC_B64", "SOP1", "s_setpc_b64 s[2:3]"),
    ("S_SWAPPC_B64", "SOP1", "s_swappc_b64 s[30:31], s[2:3]"),
    # SOP2
    ("S_ADD_U32", "SOP2", "s_add_u32 s1, s2, s3"),
    ("S_SUB_U32", "SOP2", "s_sub_u32 s1, s2, s3"),
    ("S_ADDC_U32", "SOP2", "s_addc_u32 s1, s2, s3"),
    ("S_SUBB_U32", "SOP2", "s_subb_u32 s1, s2, s3"),
    ("S_ADD_I32", "SOP2", "s_add_i32 s1, s2, s3"),
    ("S_SUB_I32", "SOP2", "s_sub_i32 s1, s2, s3"),
    ("S_AND_B32", "SOP2", "s_and_b32 s1, s2, s3"),
    ("S_AND_B64", "SOP2", "s_and_b64 s[2:3], s[4:5], s[6:7]"),
    ("S_OR_B64", "SOP2", "s_or_b64 s[2:3], s[4:5], s[6:7]"),
    ("S_XOR_B64", "SOP2", "s_xor_b64 s[2:3], s[4:5], s[6:7]"),
    ("S_ANDN2_B64", "SOP2", "s_andn2_b64 s[2:3], s[4:5], s[6:7]"),
    ("S_ORN2_B64", "SOP2", "s_orn2_b64 s[2:3], s[4:5], s[6:7]"),
    ("S_LSHR_B32", "SOP2", "s_lshr_b32 s1, s2, s3"),
    ("S_ASHR_I32", "SOP2", "s_ashr_i32 s1, s2, s3"),
    ("S_CSELECT_B64", "SOP2", "s_cselect_b64 s[2:3], s[4:5], s[6:7]"),
    # SOPK
    ("S_MOVK_I32", "SOPK", "s_movk_i32 s1, 0x1234"),
    # SOPC
    ("S_CMP_EQ_U32", "SOPC", "s_cmp_eq_u32 s1, s2"),
    ("S_CMP_LG_U32", "SOPC", "s_cmp_lg_u32 s1, s2"),
    ("S_CMP_EQ_U64", "SOPC", "s_cmp_eq_u64 s[2:3], s[4:5]"),
    ("S_CMP_LG_U64", "SOPC", "s_cmp_lg_u64 s[2:3], s[4:5]"),
    ("S_SET_GPR_IDX_ON", "SOPC", "s_set_gpr_idx_on s2, gpr_idx(SRC0)"),
    # SOPP
    ("S_NOP", "SOPP", "s_nop 1"),
    ("S_ENDPGM", "SOPP", "s_endpgm"),
    ("S_SET_GPR_IDX_OFF", "SOPP", "s_set_gpr_idx_off"),
    ("S_BRANCH", "SOPP", "s_branch 5"),
    ("S_CBRANCH_SCC0", "SOPP", "s_cbranch_scc0 5"),
    ("S_CBRANCH_SCC1", "SOPP", "s_cbranch_scc1 5"),
    ("S_CBRANCH_VCCZ", "SOPP", "s_cbranch_vccz 5"),
    ("S_CBRANCH_VCCNZ", "SOPP", "s_cbranch_vccnz 5"),
    ("S_CBRANCH_EXECZ", "SOPP", "s_cbranch_execz 5"),
    ("S_CBRANCH_EXECNZ", "SOPP", "s_cbranch_execnz 5"),
    ("S_WAITCNT", "SOPP", "s_waitcnt lgkmcnt(0)"),
    # SMEM
    ("S_LOAD_DWORDX2", "SMEM", "s_load_dwordx2 s[4:5], s[2:3], 0x0"),
    # VOP1 (emitted in their VOP3 form: op + 0x140)
    ("V_MOV_B32", "VOP1", "v_mov_b32_e32 v1, v2"),
    ("V_MOV_B64", "VOP1", "v_mov_b64_e32 v[2:3], v[4:5]"),
    ("V_READFIRSTLANE_B32", "VOP1", "v_readfirstlane_b32 s5, v3"),
    ("V_CVT_F64_I32", "VOP1", "v_cvt_f64_i32_e32 v[2:3], v1"),
    ("V_CVT_F64_U32", "VOP1", "v_cvt_f64_u32_e32 v[2:3], v1"),
    ("V_CVT_I32_F64", "VOP1", "v_cvt_i32_f64_e32 v1, v[2:3]"),
    ("V_CVT_U32_F64", "VOP1", "v_cvt_u32_f64_e32 v1, v[2:3]"),
    ("V_TRUNC_F64", "VOP1", "v_trunc_f64_e32 v[2:3], v[4:5]"),
    ("V_RNDNE_F64", "VOP1", "v_rndne_f64_e32 v[2:3], v[4:5]"),
    ("V_FLOOR_F64", "VOP1", "v_floor_f64_e32 v[2:3], v[4:5]"),
    ("V_RCP_F64", "VOP1", "v_rcp_f64_e32 v[2:3], v[4:5]"),
    ("V_NOT_B32", "VOP1", "v_not_b32_e32 v1, v2"),
    # VOP2 (VOP3 form: op + 0x100)
    ("V_CNDMASK_B32", "VOP2", "v_cndmask_b32_e32 v1, v2, v3, vcc"),
    ("V_AND_B32", "VOP2", "v_and_b32_e32 v1, v2, v3"),
    ("V_OR_B32", "VOP2", "v_or_b32_e32 v1, v2, v3"),
    ("V_XOR_B32", "VOP2", "v_xor_b32_e32 v1, v2, v3"),
    ("V_LSHLREV_B32", "VOP2", "v_lshlrev_b32_e32 v1, v2, v3"),
    ("V_LSHRREV_B32", "VOP2", "v_lshrrev_b32_e32 v1, v2, v3"),
    ("V_ASHRREV_I32", "VOP2", "v_ashrrev_i32_e32 v1, v2, v3"),
    ("V_ADD_U32", "VOP2", "v_add_u32_e32 v1, v2, v3"),
    ("V_SUB_U32", "VOP2", "v_sub_u32_e32 v1, v2, v3"),
    ("V_MAX_U32", "VOP2", "v_max_u32_e32 v1, v2, v3"),
    ("V_MIN_U32", "VOP2", "v_min_u32_e32 v1, v2, v3"),
    ("V_ADD_CO_U32", "VOP2", "v_add_co_u32_e32 v1, vcc, v2, v3"),
    ("V_SUB_CO_U32", "VOP2", "v_sub_co_u32_e32 v1, vcc, v2, v3"),
    ("V_ADDC_CO_U32", "VOP2", "v_addc_co_u32_e32 v1, vcc, v2, v3, vcc"),
    ("V_SUBB_CO_U32", "VOP2", "v_subb_co_u32_e32 v1, vcc, v2, v3, vcc"),
    # VOPC (VOP3 form: op)
    ("V_CMP_CLASS_F64", "VOPC", "v_cmp_class_f64_e32 vcc, v[2:3], v4"),
    ("V_CMP_LT_F64", "VOPC", "v_cmp_lt_f64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_EQ_F64", "VOPC", "v_cmp_eq_f64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_LE_F64", "VOPC", "v_cmp_le_f64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_GT_F64", "VOPC", "v_cmp_gt_f64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_GE_F64", "VOPC", "v_cmp_ge_f64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_NEQ_F64", "VOPC", "v_cmp_neq_f64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_U_F64", "VOPC", "v_cmp_u_f64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_LT_I32", "VOPC", "v_cmp_lt_i32_e32 vcc, v2, v4"),
    ("V_CMP_EQ_U32", "VOPC", "v_cmp_eq_u32_e32 vcc, v2, v4"),
    ("V_CMP_NE_U32", "VOPC", "v_cmp_ne_u32_e32 vcc, v2, v4"),
    ("V_CMP_GT_U32", "VOPC", "v_cmp_gt_u32_e32 vcc, v2, v4"),
    ("V_CMP_GE_U32", "VOPC", "v_cmp_ge_u32_e32 vcc, v2, v4"),
    ("V_CMP_LT_U32", "VOPC", "v_cmp_lt_u32_e32 vcc, v2, v4"),
    ("V_CMP_LT_I64", "VOPC", "v_cmp_lt_i64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_EQ_I64", "VOPC", "v_cmp_eq_i64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_LE_I64", "VOPC", "v_cmp_le_i64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_GT_I64", "VOPC", "v_cmp_gt_i64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_NE_I64", "VOPC", "v_cmp_ne_i64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_GE_I64", "VOPC", "v_cmp_ge_i64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_LT_U64", "VOPC", "v_cmp_lt_u64_e32 vcc, v[2:3], v[4:5]"),
    ("V_CMP_GT_U64", "VOPC", "v_cmp_gt_u64_e32 vcc, v[2:3], v[4:5]"),
    # VOP3-only
    ("V_ADD_F64", "VOP3", "v_add_f64 v[0:1], v[2:3], v[4:5]"),
    ("V_MUL_F64", "VOP3", "v_mul_f64 v[0:1], v[2:3], v[4:5]"),
    ("V_FMA_F64", "VOP3", "v_fma_f64 v[0:1], v[2:3], v[4:5], v[6:7]"),
    ("V_LDEXP_F64", "VOP3", "v_ldexp_f64 v[0:1], v[2:3], v4"),
    ("V_DIV_SCALE_F64", "VOP3B", "v_div_scale_f64 v[0:1], s[2:3], v[2:3], v[4:5], v[6:7]"),
    ("V_DIV_FMAS_F64", "VOP3", "v_div_fmas_f64 v[0:1], v[2:3], v[4:5], v[6:7]"),
    ("V_DIV_FIXUP_F64", "VOP3", "v_div_fixup_f64 v[0:1], v[2:3], v[4:5], v[6:7]"),
    ("V_MAD_U64_U32", "VOP3B", "v_mad_u64_u32 v[0:1], s[2:3], v4, v5, v[6:7]"),
    ("V_MAD_I64_I32", "VOP3B", "v_mad_i64_i32 v[0:1], s[2:3], v4, v5, v[6:7]"),
    ("V_MUL_LO_U32", "VOP3", "v_mul_lo_u32 v0, v1, v2"),
    ("V_MUL_HI_U32", "VOP3", "v_mul_hi_u32 v0, v1, v2"),
    ("V_LSHLREV_B64", "VOP3", "v_lshlrev_b64 v[0:1], v2, v[4:5]"),
    ("V_LSHRREV_B64", "VOP3", "v_lshrrev_b64 v[0:1], v2, v[4:5]"),
    ("V_ASHRREV_I64", "VOP3", "v_ashrrev_i64 v[0:1], v2, v[4:5]"),
    ("V_BFE_U32", "VOP3", "v_bfe_u32 v0, v1, v2, v3"),
    ("V_BFE_I32", "VOP3", "v_bfe_i32 v0, v1, v2, v3"),
    ("V_LSHL_ADD_U64", "VOP3", "v_lshl_add_u64 v[0:1], v[2:3], 0, v[4:5]"),
    ("V_READLANE_B32", "VOP3", "v_readlane_b32 s1, v2, 3"),
    ("V_WRITELANE_B32", "VOP3", "v_writelane_b32 v1, s2, 3"),
    # DS
    ("DS_READ_B64", "DS", "ds_read_b64 v[2:3], v29 offset:16"),
    # FLAT (global / scratch segments)
    ("GLOBAL_LOAD_DWORDX2", "FLAT", "global_load_dwordx2 v[2:3], v[4:5], off offset:8"),
    ("SCRATCH_LOAD_DWORD", "FLAT", "scratch_load_dword v5, off, s32 offset:4"),
    ("SCRATCH_LOAD_DWORDX2", "FLAT", "scratch_load_dwordx2 v[4:5], off, s32 offset:4"),
    ("SCRATCH_LOAD_DWORDX4", "FLAT", "scratch_load_dwordx4 v[4:7], off, s32 offset:4"),
    ("SCRATCH_STORE_DWORD", "FLAT", "scratch_store_dword off, v5, s32 offset:4"),
    ("SCRATCH_STORE_DWORDX2", "FLAT", "scratch_store_dwordx2 off, v[4:5], s32 offset:4"),
    ("SCRATCH_STORE_DWORDX4", "FLAT", "scratch_store_dwordx4 off, v[4:7], s32 offset:4"),
]

_ENC = re.compile(r"encoding:\s*\[([^\]]*)\]")


def assemble(lines):
    r = subprocess.run([MC, "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-show-encoding"],
                       input="\n".join(lines) + "\n", capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr)
    out = []
    for line in r.stdout.splitlines():
        m = _ENC.search(line)
        if m:
            bs = [int(x, 16) for x in m.group(1).split(",")]
            out.append([int.from_bytes(bytes(bs[i:i + 4]), "little") for i in range(0, len(bs), 4)])
    if len(out) != len(lines):
        raise SystemExit(f"expected {len(lines)} encodings, got {len(out)}")
    return out


def opcode(fmt, w):
    w0 = w[0]
    if fmt == "SOP1":
        return (w0 >> 8) & 0xFF
    if fmt == "SOP2":
        return (w0 >> 23) & 0x7F
    if fmt == "SOPK":
        return (w0 >> 23) & 0x1F
    if fmt in ("SOPC", "SOPP"):
        return (w0 >> 16) & 0x7F
    if fmt == "SMEM":
        return (w0 >> 18) & 0xFF
    if fmt == "VOP1":
        return (w0 >> 9) & 0xFF
    if fmt == "VOP2":
        return (w0 >> 25) & 0x3F
    if fmt == "VOPC":
        return (w0 >> 17) & 0xFF
    if fmt in ("VOP3", "VOP3B"):
        return (w0 >> 16) & 0x3FF
    if fmt == "DS":
        return (w0 >> 17) & 0xFF
    if fmt == "FLAT":
        return (w0 >> 18) & 0x7F
    raise ValueError(fmt)


def main():
    encs = assemble([s for _, _, s in FORMS])
    lines = ["// generated by tools/gen_gcn_opcodes.py from the ROCm llvm-mc (gfx950) -- do not edit",
             "// FKS_GCN_OP(name, format, opcode)"]
    for (name, fmt, sample), w in zip(FORMS, encs):
        lines.append(f"FKS_GCN_OP({name}, {fmt}, 0x{opcode(fmt, w):X})  // {sample}")
    with open(OUT, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"wrote {OUT} ({len(FORMS)} opcodes)")


if __name__ == "__main__":
    sys.exit(main())
