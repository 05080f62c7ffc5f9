"""Generates csrc/q4_kloop.inc: the K loop of the 4-wave GEMM (q4: 256 x 256 output tile, 4 waves of 128 x 128, one
wave per SIMD) as ONE inline-asm statement -- prologue, the steady-state loop in two per-SIMD copies, and the two
tail steps -- with every register named, so nothing the compiler does sits between the loop's instructions.

Why assembly: round 5 placed every read, DMA, wait and barrier of a HIP 4-wave loop at the
slot the vendor library's gfx950 kernel uses for this geometry (hipBLASLt MT256x256x64_MI16x16x1, read with
llvm-objdump) and stayed 3-4 % slower per K step; the two per-SIMD loop copies could not be expressed in HIP at all
(the compiler merged the copies' accumulators).  Here the accumulators are pinned AGPRs (a[4 m : 4 m + 3], m = 8 j + i
for output block (i, j)), the fragments pinned VGPRs, and the per-step work is the loop's own:
  * per 64-deep K step 128 MFMAs v_mfma_f32_16x16x32_bf16 (k-slice 0: m = 0..63, k-slice 1: 64..127; src0 = the B
    fragment j = (m & 63) >> 3 -- held for 8 MFMAs --, src1 = the A fragment i = m & 7);
  * 16 fragment reads per k-slice (ds_read_b128 at immediate offsets 2048 f from 4 per-lane bases: A / B x k-slice),
    the k-slice-1 fragments of this step in its first 43 slots, the next step's k-slice-0 fragments in the last 34;
  * 16 LDS-DMAs (buffer_load_dwordx4 ... lds, 16 B per lane, M0 stepping 1 KB per piece) of the step two ahead, the A
    half after the first barrier (slot 22: every wave has read this step's A fragments) and the B half after the
    second (slot 52);
  * vmcnt(13) + barrier at slot 92/93: every DMA of the previous step (= the next step's operands) has landed;
  * the K advance is one v_add per operand (the DMA voffset), the buffer switch 4 v_xor (read bases) + 2 s_xor (M0).
The slot tables below (instruction index = MFMAs issued before it) follow the vendor loop's two copies: even SIMDs
issue each DMA one slot before the fragment read beside it, odd SIMDs one slot after; picked once per wave by the
SIMD id (HW_REG_HW_ID bit 4).  Tail: step nk - 2 (no DMAs; vmcnt(0) before the last k-slice-0 reads) and step nk - 1
(no DMAs, no next-step reads).  LDS image: [2 buffers][A | B][256 rows][128 B], 16-B chunk c of row r at c ^ (r & 7)
(the ping-pong's KC layout: conflict-free ds_read_b128).

No instruction here writes through the scalar data cache; M0 is saved and restored by the statement.
Usage: python tools/gen_q4_kloop.py [out.inc [split|even|odd]]  (default: rewrites csrc/q4_kloop.inc, the per-SIMD
split; the build compiles the .inc, it does not run the generator)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "crosscoder-model-diff-replication_amd", "csrc", "q4_kloop.inc")

# ---- per-step slot tables of the steady loop: (slot, op, arg); slot = MFMAs issued before the instruction
COMMON_HEAD = ([(1 + 2 * i, "ra1", i) for i in range(8)] +
               [(4, "kadv_a", 0), (14, "kadv_b", 0), (16, "m0a", 0), (21, "wl", 0), (22, "bar", 0)])
EVEN = COMMON_HEAD + [
    (23, "da", 0), (24, "m0inc", 0), (25, "rb1", 0), (26, "da", 1), (27, "m0inc", 0), (28, "rb1", 1), (29, "da", 2),
    (30, "m0inc", 0), (31, "rb1", 2), (32, "da", 3), (33, "m0inc", 0), (34, "rb1", 3), (35, "da", 4), (36, "m0inc", 0),
    (37, "rb1", 4), (39, "rb1", 5), (41, "rb1", 6), (43, "rb1", 7),
    (51, "wl", 0), (52, "bar", 0),
    (53, "da", 5), (54, "m0inc", 0), (56, "da", 6), (57, "m0inc", 0), (59, "da", 7), (60, "m0b", 0), (62, "db", 0),
    (63, "m0inc", 0), (65, "db", 1), (66, "m0inc", 0), (66, "xma", 0),
    (85, "tog", 0), (86, "db", 2), (87, "m0inc", 0), (88, "db", 3), (89, "m0inc", 0), (90, "db", 4),
    (92, "wv13", 0), (93, "bar", 0),
    (94, "ra0", 0), (95, "ra0", 1), (95, "m0inc", 0), (96, "ra0", 2), (97, "db", 5), (98, "ra0", 3), (99, "ra0", 4),
    (99, "m0inc", 0), (101, "db", 6), (103, "ra0", 5), (103, "m0inc", 0), (104, "ra0", 6), (105, "ra0", 7),
    (106, "rb0", 0), (107, "rb0", 1), (110, "rb0", 2), (113, "rb0", 3), (115, "rb0", 4), (118, "rb0", 5),
    (121, "rb0", 6), (124, "rb0", 7), (125, "db", 7), (126, "xmb", 0), (126, "cdec", 0), (127, "ccmp", 0),
    (127, "wl", 0)]
ODD = COMMON_HEAD + [
    (23, "rb1", 0), (24, "da", 0), (25, "m0inc", 0), (26, "rb1", 1), (27, "da", 1), (28, "m0inc", 0), (29, "rb1", 2),
    (30, "da", 2), (31, "m0inc", 0), (32, "rb1", 3), (33, "da", 3), (34, "m0inc", 0), (35, "rb1", 4), (36, "da", 4),
    (37, "m0inc", 0), (39, "rb1", 5), (41, "rb1", 6), (43, "rb1", 7),
    (51, "wl", 0), (52, "bar", 0),
    (54, "da", 5), (55, "m0inc", 0), (57, "da", 6), (58, "m0inc", 0), (60, "da", 7), (61, "m0b", 0), (63, "db", 0),
    (64, "m0inc", 0), (66, "db", 1), (67, "m0inc", 0), (67, "xma", 0),
    (84, "tog", 0), (85, "db", 2), (86, "m0inc", 0), (87, "db", 3), (88, "m0inc", 0), (89, "db", 4),
    (92, "wv13", 0), (93, "bar", 0),
    (94, "ra0", 0), (95, "ra0", 1), (95, "m0inc", 0), (96, "db", 5), (97, "ra0", 2), (98, "ra0", 3), (99, "ra0", 4),
    (99, "m0inc", 0), (100, "db", 6), (103, "ra0", 5), (103, "m0inc", 0), (104, "ra0", 6), (105, "ra0", 7),
    (106, "rb0", 0), (107, "rb0", 1), (110, "rb0", 2), (113, "rb0", 3), (115, "rb0", 4), (118, "rb0", 5),
    (121, "rb0", 6), (123, "rb0", 7), (124, "db", 7), (126, "xmb", 0), (126, "cdec", 0), (127, "ccmp", 0),
    (127, "wl", 0)]
# tail steps: k-slice-1 reads A / B interleaved, no DMAs
TAIL_READS = ([(1, "ra1", 0), (3, "rb1", 0)] + [(5 + 2 * q, "ra1", 1 + q) for q in range(7)] +
              [(19 + 2 * q, "rb1", 1 + q) for q in range(7)])
TAIL_A = TAIL_READS + [(63, "tog", 0), (64, "wl", 0), (106, "wv0", 0), (107, "bar", 0)] + \
    [(108 + q, "ra0", q) for q in range(8)] + [(116 + q, "rb0", q) for q in range(8)] + [(127, "wl", 0)]
TAIL_B = TAIL_READS + [(64, "wl", 0)]


def mfma(m):
    kk, mm = m >> 6, m & 63
    j, i = mm >> 3, mm & 7
    b = (100 if kk else 68) + 4 * j
    a = (36 if kk else 4) + 4 * i
    return f"v_mfma_f32_16x16x32_bf16 a[{4 * mm}:{4 * mm + 3}], v[{b}:{b + 3}], v[{a}:{a + 3}], a[{4 * mm}:{4 * mm + 3}]"


def op(kind, arg):
    if kind == "ra1":
        return f"ds_read_b128 v[{36 + 4 * arg}:{39 + 4 * arg}], %[ra1] offset:{2048 * arg}"
    if kind == "rb1":
        return f"ds_read_b128 v[{100 + 4 * arg}:{103 + 4 * arg}], %[rb1] offset:{2048 * arg}"
    if kind == "ra0":
        return f"ds_read_b128 v[{4 + 4 * arg}:{7 + 4 * arg}], %[ra0] offset:{2048 * arg}"
    if kind == "rb0":
        return f"ds_read_b128 v[{68 + 4 * arg}:{71 + 4 * arg}], %[rb0] offset:{2048 * arg}"
    if kind == "da":
        so = "0" if arg == 0 else f"%[oa{arg}]"
        return f"buffer_load_dwordx4 %[vda], %[rsa], {so} offen lds"
    if kind == "db":
        so = "0" if arg == 0 else f"%[oa{arg}]"  # (the operands share their row stride: one set of piece offsets)
        return f"buffer_load_dwordx4 %[vdb], %[rsb], {so} offen lds"
    if kind == "m0inc":
        return "s_add_u32 m0, m0, 0x400"
    if kind == "m0a":
        return "s_mov_b32 m0, %[ma]"
    if kind == "m0b":
        return "s_mov_b32 m0, %[mb]"
    if kind == "wl":
        return "s_waitcnt lgkmcnt(0)"
    if kind == "wv13":
        return "s_waitcnt vmcnt(13)"
    if kind == "wv0":
        return "s_waitcnt vmcnt(0)"
    if kind == "bar":
        return "s_barrier"
    if kind == "kadv_a":
        return "v_add_u32_e32 %[vda], 0x80, %[vda]"
    if kind == "kadv_b":
        return "v_add_u32_e32 %[vdb], 0x80, %[vdb]"
    if kind == "tog":
        return ("v_xor_b32_e32 %[ra0], 0x10000, %[ra0]\nv_xor_b32_e32 %[rb0], 0x10000, %[rb0]\n"
                "v_xor_b32_e32 %[ra1], 0x10000, %[ra1]\nv_xor_b32_e32 %[rb1], 0x10000, %[rb1]")
    if kind == "xma":
        return "s_xor_b32 %[ma], 0x10000, %[ma]"
    if kind == "xmb":
        return "s_xor_b32 %[mb], 0x10000, %[mb]"
    if kind == "cdec":
        return "s_sub_u32 %[cnt], %[cnt], 1"
    if kind == "ccmp":
        return "s_cmp_eq_u32 %[cnt], 0"
    raise ValueError(kind)


def step(table):
    at = {}
    for s, k, a in table:
        at.setdefault(s, []).append(op(k, a))
    out = []
    for m in range(128):
        out += at.get(m, [])
        out.append(mfma(m))
    out += at.get(128, [])
    assert max(at) <= 128
    return out


def prologue():
    out = ["s_mov_b32 %[msave], m0"]
    for step_i in range(2):
        for opnd, m0 in (("a", "%[ma]"), ("b", "%[mb]")):
            out += [f"s_mov_b32 m0, {m0}", "s_nop 0"]
            for q in range(8):
                so = "0" if q == 0 else f"%[oa{q}]"
                out.append(f"buffer_load_dwordx4 %[vd{opnd}], %[rs{opnd}], {so} offen lds")
                if q < 7:
                    out += ["s_add_u32 m0, m0, 0x400", "s_nop 0"]
        if step_i == 0:
            out += ["v_add_u32_e32 %[vda], 0x80, %[vda]", "v_add_u32_e32 %[vdb], 0x80, %[vdb]",
                    "s_xor_b32 %[ma], 0x10000, %[ma]", "s_xor_b32 %[mb], 0x10000, %[mb]"]
    # (back to buffer 0: the loop's step t issues step t + 2 into buffer t & 1)
    out += ["s_xor_b32 %[ma], 0x10000, %[ma]", "s_xor_b32 %[mb], 0x10000, %[mb]",
            "s_waitcnt vmcnt(16)", "s_barrier"]
    out += [op("ra0", i) for i in range(8)] + [op("rb0", j) for j in range(8)]
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def program(variant="split"):
    """variant (experiments only): "split" = the per-SIMD copies; "even" / "odd" = every wave runs that copy."""
    even, odd = {"split": (EVEN, ODD), "even": (EVEN, EVEN), "odd": (ODD, ODD)}[variant]
    L = prologue()
    L += ["s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 L_q4tail_%=",
          "s_getreg_b32 %[tmp], hwreg(HW_REG_HW_ID, 4, 1)", "s_cmp_eq_u32 %[tmp], 0", "s_cbranch_scc0 L_q4odd_%=",
          "L_q4even_%=:"]
    L += step(even) + ["s_cbranch_scc0 L_q4even_%=", "s_branch L_q4tail_%=", "L_q4odd_%=:"]
    L += step(odd) + ["s_cbranch_scc0 L_q4odd_%=", "L_q4tail_%=:"]
    L += step(TAIL_A) + step(TAIL_B)
    # (the last MFMAs' results are read by the epilogue's v_accvgpr_read: 19 wait states)
    L += ["s_nop 7", "s_nop 7", "s_nop 2", "s_mov_b32 m0, %[msave]"]
    return L


def main():
    import sys

    out = sys.argv[1] if len(sys.argv) > 1 else OUT
    prog = program(sys.argv[2] if len(sys.argv) > 2 else "split")
    n_mfma = sum(1 for l in prog if l.startswith("v_mfma"))
    assert n_mfma == 4 * 128, n_mfma
    lines = []
    for l in prog:
        for part in l.split("\n"):
            lines.append(f'  "{part}\\n"')
    acc_ops = ", ".join(f'"+{{a[{4 * (8 * j + i)}:{4 * (8 * j + i) + 3}]}}"(ACC[{i}][{j}])'
                        for j in range(8) for i in range(8))
    clob = ", ".join(f'"v{r}"' for r in range(4, 132))
    with open(out, "w") as f:
        f.write("// GENERATED by tools/gen_q4_kloop.py -- do not edit.  The 4-wave GEMM's K loop as one inline-asm\n"
                "// statement (see the generator's docstring for the schedule).\n")
        f.write("#define Q4_KLOOP_ASM \\\n" + " \\\n".join(lines) + "\n")
        f.write(f"#define Q4_ACC_OPERANDS(ACC) {acc_ops}\n")
        f.write(f"#define Q4_FRAG_CLOBBERS {clob}\n")
    print(f"wrote {out}: {len(prog)} instructions ({n_mfma} MFMAs)")


if __name__ == "__main__":
    main()
