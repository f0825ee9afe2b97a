#!/usr/bin/env python3
"""Semantic probe kernel for the gfx950 primitives the assembly forward relies on (dev tool).

    python tools/probe_gen.py > probe.s      (tools/probe_run.py builds, runs and compares)

One workgroup of 64 lanes (one wave).  Kernargs: in (u64), out (u64).  Every result row is 64 lanes
x 1 dword, stored with buffer_store_dword at row * 256 + lane * 4 through a descriptor whose record
count is the exact output size (OUT_ROWS * 256 bytes), so no store can leave the buffer.
"""
OUT_ROWS = 128


def rows():
    r = []
    row = [0]

    def store(reg):
        t = row[0]
        row[0] += 1
        return [f"s_mov_b32 s30, {t * 256}", "s_nop 1", f"buffer_store_dword {reg}, v1, s[8:11], s30 offen", "s_nop 1"]
    L = []
    L += ["s_load_dwordx4 s[4:7], s[0:1], 0x0", "s_waitcnt lgkmcnt(0)",
          # in: s[12:15] (records 64 KiB), out: s[8:11]
          "s_mov_b32 s12, s4", "s_and_b32 s13, s5, 0xffff", "s_mov_b32 s14, 0x10000", "s_mov_b32 s15, 0x20000",
          "s_mov_b32 s8, s6", "s_and_b32 s9, s7, 0xffff", f"s_mov_b32 s10, {OUT_ROWS * 256}", "s_mov_b32 s11, 0x20000",
          "v_lshlrev_b32_e32 v1, 2, v0", "v_lshlrev_b32_e32 v2, 4, v0", "s_nop 4"]
    # R0: workgroup id, lane id
    L += ["v_mov_b32_e32 v3, s2"] + store("v3") + store("v0")
    # R1: LDS-DMA of in[lane*16 .. +16] to LDS at M0 = base (three bases incl. above 64 KiB), read back
    for base in (0, 70 * 1024, 150 * 1024):
        L += [f"s_mov_b32 m0, {base}", "s_nop 0", "buffer_load_dwordx4 v2, s[12:15], 0 offen lds",
              "s_waitcnt vmcnt(0)", "s_barrier", f"v_add_u32_e32 v4, {base}, v2", "s_nop 1",
              "ds_read_b128 v[8:11], v4", "s_waitcnt lgkmcnt(0)"]
        for k in range(4):
            L += store(f"v{8 + k}")
    # R2: LDS-DMA with inst_offset:64 (does it move the LDS destination too?)
    L += ["s_mov_b32 m0, 4096", "s_nop 0", "buffer_load_dwordx4 v2, s[12:15], 0 offen offset:64 lds",
          "s_waitcnt vmcnt(0)", "v_add_u32_e32 v4, 4096, v2", "s_nop 1",
          "ds_read_b128 v[8:11], v4", "ds_read_b128 v[12:15], v4 offset:64", "s_waitcnt lgkmcnt(0)"]
    for k in range(8):
        L += store(f"v{8 + k}")
    # R3: ds_read_b64_tr_b16 into VGPRs and AGPRs from LDS 0.. (filled by R1 base 0): per-lane address
    # = lane*8 (16 lanes x 8 B = one 128-B row group)
    L += ["v_lshlrev_b32_e32 v5, 3, v0", "s_nop 1", "ds_read_b64_tr_b16 v[16:17], v5", "ds_read_b64_tr_b16 a[16:17], v5",
          "s_waitcnt lgkmcnt(0)", "v_accvgpr_read_b32 v18, a16", "v_accvgpr_read_b32 v19, a17", "s_nop 1"]
    L += store("v16") + store("v17") + store("v18") + store("v19")
    # R4: buffer_load_dwordx4 into AGPRs (with inst_offset 32), read back through v_accvgpr_read
    L += ["buffer_load_dwordx4 a[20:23], v2, s[12:15], 0 offen offset:32", "s_waitcnt vmcnt(0)",
          "v_accvgpr_read_b32 v20, a20", "v_accvgpr_read_b32 v21, a21", "v_accvgpr_read_b32 v22, a22",
          "v_accvgpr_read_b32 v23, a23", "s_nop 1"]
    L += store("v20") + store("v21") + store("v22") + store("v23")
    # R5: MFMA bf16 32x32x16 with A, B from VGPRs (in[0..1023] as A, in[1024..2047] as B)
    L += ["buffer_load_dwordx4 v[24:27], v2, s[12:15], 0 offen", "buffer_load_dwordx4 v[28:31], v2, s[12:15], 0 offen offset:1024",
          "s_waitcnt vmcnt(0)", "s_nop 2",
          "v_mfma_f32_32x32x16_bf16 v[32:47], v[24:27], v[28:31], 0", "s_nop 15", "s_nop 3"]
    for g in range(16):
        L += store(f"v{32 + g}")
    # R6: the same MFMA with A, B from AGPRs, result in AGPRs; and A in AGPR / B VGPR / D VGPR
    L += ["v_accvgpr_write_b32 a24, v24", "v_accvgpr_write_b32 a25, v25", "v_accvgpr_write_b32 a26, v26",
          "v_accvgpr_write_b32 a27, v27", "v_accvgpr_write_b32 a28, v28", "v_accvgpr_write_b32 a29, v29",
          "v_accvgpr_write_b32 a30, v30", "v_accvgpr_write_b32 a31, v31", "s_nop 4",
          "v_mfma_f32_32x32x16_bf16 a[32:47], a[24:27], a[28:31], 0",
          "v_mfma_f32_32x32x16_bf16 v[48:63], a[24:27], v[28:31], 0", "s_nop 15", "s_nop 3"]
    for g in range(16):
        L += [f"v_accvgpr_read_b32 v64, a{32 + g}", "s_nop 1"] + store("v64")
    for g in range(16):
        L += store(f"v{48 + g}")
    # R7: permlane32_swap, exp, cvt_pk
    L += ["v_mov_b32_e32 v70, v0", "v_add_u32_e32 v71, 100, v0", "s_nop 1", "v_permlane32_swap_b32_e32 v70, v71", "s_nop 1"]
    L += store("v70") + store("v71")
    L += ["v_cvt_f32_u32_e32 v72, v0", "v_mul_f32_e32 v72, 0x3e000000, v72", "v_exp_f32_e32 v73, v72", "s_nop 1",
          "v_cvt_pk_bf16_f32 v74, v72, v73", "s_nop 1"]
    L += store("v73") + store("v74")
    L += ["s_waitcnt vmcnt(0)", "s_endpgm"]
    return L, row[0]


def main():
    L, n = rows()
    assert n <= OUT_ROWS
    name = "fa_probe"
    out = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 5", "\t.text",
           f"\t.globl {name}", "\t.p2align 8", f"\t.type {name},@function", f"{name}:"]
    out += ["\t" + x for x in L]
    out += [f".L{name}_fend:", f"\t.size {name}, .L{name}_fend-{name}"]
    out.append(f"""
	.rodata
	.p2align 6
	.amdhsa_kernel {name}
		.amdhsa_group_segment_fixed_size 163840
		.amdhsa_private_segment_fixed_size 0
		.amdhsa_kernarg_size 16
		.amdhsa_user_sgpr_count 2
		.amdhsa_user_sgpr_kernarg_segment_ptr 1
		.amdhsa_system_sgpr_workgroup_id_x 1
		.amdhsa_system_vgpr_workitem_id 0
		.amdhsa_next_free_vgpr 512
		.amdhsa_next_free_sgpr 40
		.amdhsa_accum_offset 256
		.amdhsa_reserve_vcc 1
		.amdhsa_float_denorm_mode_32 3
		.amdhsa_float_denorm_mode_16_64 3
		.amdhsa_ieee_mode 0
	.end_amdhsa_kernel
	.text
	.amdgpu_metadata
---
amdhsa.kernels:
  - .agpr_count: 256
    .args:
      - .offset: 0
        .size: 16
        .value_kind: by_value
    .group_segment_fixed_size: 163840
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: 64
    .name: {name}
    .private_segment_fixed_size: 0
    .sgpr_count: 42
    .sgpr_spill_count: 0
    .symbol: {name}.kd
    .uniform_work_group_size: 1
    .vgpr_count: 512
    .vgpr_spill_count: 0
    .wavefront_size: 64
amdhsa.target: amdgcn-amd-amdhsa--gfx950
amdhsa.version:
  - 1
  - 2
...
	.end_amdgpu_metadata""")
    print("\n".join(out))


if __name__ == "__main__":
    main()
