#!/usr/bin/env python3
"""EXPERIMENT, NOT BUILT (round 3): measured 2.4-5.7 % slower than the C++ visit and
reverted ("the visit in assembly").  Apply
ggs_kernels_asm_visit.patch and run this generator into csrc/ to reproduce.

Generates ggs_visit_asm.inc: the raster's (splat, strip) visit as ONE inline-asm
block for gfx950 with computed jumps instead of compare trees.

Why: a scalar compare-and-branch costs a wave ~10 ns at 3 waves per SIMD and ~35
cycles alone (tools/mb/pair_rate.hip); in the raster, one extra taken branch per
visit costs 1.4 % of the launch at 512^2 and 1.6 % at 2048^2.
The C++ visit took ~11.5 branches (dispatch trees on the first and last row pair:
the accumulators are statically named registers, so every entry and exit point is
its own code).  Here a visit takes two indirect jumps (s_setpc_b64) and one branch:

  head     x-terms, first-pair exponent and exps, ratio, seed guard, dispatch
  FULL     splat spans the strip's 128 rows: 16 unmasked pairs
  F1[k]    one-pair visit at pair k (both row masks)
  FM[k]    first pair k (top row mask), then jump into S_kB at pair k+1
  S_kB     pairs 1 .. kB-1 (row recurrence) then the masked last pair kB; a visit
           enters at pair kA+1, so one straight-line run serves every kA < kB
           ("end-aligned" blocks: start(S_kB) = S_1 + PSZ (kB-1)(kB-2)/2 + LSZ (kB-1))
  EXACT    seed guard tripped (flagged thin splats, ~0.3 % of visits): every pair
           with its own exponent and both row masks (pairs outside the AABB blend 0)
Every block of a kind has the same byte size; the jump offsets are label
differences resolved by the assembler and checked after the build
(check_visit_layout.py on the disassembly).

The arithmetic is exactly the C++ visit's (same operations in the same order on
the same values), so images and fitness are bit-identical (tools/probe/rtime.py).

Register map (pinned: the C++ side binds these with {v[..]} constraints):
  accumulators  pair k: R v[8k:8k+1], G v[8k+2:8k+3], B v[8k+4:8k+5], T v[8k+6:8k+7]
  scratch       v[128:143] (QY, F, RT, W, E pairs; QX, TMP, PX, BX), s[88:95]
  records       s[56:71] and s[72:87] (current / next, alternating; the visit issues the
                next record's s_load_dwordx16 after waiting for the current one)
  per lane      Xf v144, col v145, ph v146, (Yb, Yb+4) v[148:149]
Hazards: gfx950 needs one wait state between a VALU result and a dependent VALU
(or SALU) read (the compiler's own s_nop 0 placements in this kernel); the
generator inserts s_nop 0 wherever an instruction reads what the VALU instruction
just before it wrote.

    python3 gen_visit_asm.py > ggs_visit_asm.inc
"""
import re
import sys

NPK = 16


def acc(k, c):                       # c: 0 R, 1 G, 2 B, 3 T
    b = 8 * k + 2 * c
    return f"v[{b}:{b + 1}]"


QY, F, RT, W, E = "v[128:129]", "v[130:131]", "v[132:133]", "v[134:135]", "v[136:137]"
QX, TMP, PX, BX = "v138", "v139", "v140", "v142"
PXP, BXP = "v[140:141]", "v[142:143]"
XF, COL, PH, YB = "v144", "v145", "v146", "v[148:149]"
NINF_LIT = "0xff800000"                  # -inf
PC, WA, MX, MY = "s[88:89]", "s[90:91]", "s[92:93]", "s[94:95]"
PCLO, PCHI, WALO, WAHI = "s88", "s89", "s90", "s91"

lines = []


def L(s):
    lines.append(s)


def label(name):
    L(f".L{name}%=:")


def pair_step(k, r_update=True, f_update=True):
    """Pair k of the row recurrence: blend with F (= f_k), then F -> f_{k+1}, RT -> r_{k+1}."""
    L(f"v_pk_mul_f32 {W}, {acc(k, 3)}, {F}")
    if f_update:
        L(f"v_pk_mul_f32 {F}, {F}, {RT}")
    if r_update:
        L(f"v_pk_mul_f32 {RT}, {RT}, %[rl] op_sel_hi:[1,0]")
    L(f"v_pk_fma_f32 {acc(k, 0)}, %[rcy], {W}, {acc(k, 0)} op_sel_hi:[0,1,1]")
    L(f"v_pk_fma_f32 {acc(k, 1)}, %[ga], {W}, {acc(k, 1)} op_sel_hi:[0,1,1]")
    L(f"v_pk_fma_f32 {acc(k, 2)}, %[bb], {W}, {acc(k, 2)} op_sel_hi:[0,1,1]")
    L(f"v_pk_add_f32 {acc(k, 3)}, {acc(k, 3)}, {W} neg_lo:[0,1] neg_hi:[0,1]")


def blend_masked(k):
    """Blend pair k with E = the row-masked F (no recurrence update)."""
    L(f"v_pk_mul_f32 {W}, {acc(k, 3)}, {E}")
    L(f"v_pk_fma_f32 {acc(k, 0)}, %[rcy], {W}, {acc(k, 0)} op_sel_hi:[0,1,1]")
    L(f"v_pk_fma_f32 {acc(k, 1)}, %[ga], {W}, {acc(k, 1)} op_sel_hi:[0,1,1]")
    L(f"v_pk_fma_f32 {acc(k, 2)}, %[bb], {W}, {acc(k, 2)} op_sel_hi:[0,1,1]")
    L(f"v_pk_add_f32 {acc(k, 3)}, {acc(k, 3)}, {W} neg_lo:[0,1] neg_hi:[0,1]")


PSZ = 56                         # bytes of one pair step (7 VOP3P), asserted below
SSZ = "(.LS2%= - .LS1%=)"        # bytes of every S_kB block (padded), asserted below
DCUR, DNXT = "%[dcur]", "%[dnxt]"   # the visit descriptors (cull-computed, see raster_kernel)


def seed(k, ratio):
    """The exact first pair: qy += 8k (two VOP2 adds with a literal; -0.0 for k = 0, which
    leaves qy's value unchanged and keeps every block of a kind the same size), e, F = 2^e,
    and with `ratio` the recurrence ratio RT of the pair's two rows."""
    lit = float_lit(8.0 * k) if k else "0x80000000"
    L(f"v_add_f32_e32 v128, {lit}, v128")
    L(f"v_add_f32_e32 v129, {lit}, v129")
    L(f"v_pk_fma_f32 {E}, %[cc], {QY}, {BXP} op_sel_hi:[0,1,0]")   # Cc qy + bx
    L(f"v_pk_fma_f32 {E}, {QY}, {E}, {PXP} op_sel_hi:[1,1,0]")     # e = qy (Cc qy + bx) + px
    L("v_exp_f32_e32 v130, v136")                           # F = 2^e (the seed)
    L("v_exp_f32_e32 v131, v137")
    if ratio:
        L(f"v_mul_f32_e32 {TMP}, 0x41000000, {BX}")        # 16 Cc qy.y + 8 bx
        L(f"v_fmac_f32_e32 {TMP}, %[c16], v129")
        L(f"v_min_f32_e32 {TMP}, 0x42c80000, {TMP}")       # clamp at 100 (exact for live lanes)
        L(f"v_exp_f32_e32 v132, {TMP}")
        L("v_mul_f32_e64 v133, |%[rho4]|, v132")            # the pair's second row: x 2^(64 Cc)


def gen():
    # ---------------- head: x-terms, qy, dispatch by the descriptor ----------------
    L("s_sub_i32 %[d0], %[y0], %[ty0]")
    L("s_sub_i32 %[d1], %[y1], %[ty0]")
    L(f"v_subrev_f32_e32 {QX}, %[cx], {XF}")                # qx = Xf - cx
    L(f"v_mov_b32_e32 v141, {NINF_LIT}")                    # -inf (px's pair: high half unused)
    L(f"v_subrev_u32_e32 {TMP}, %[x0], {COL}")              # col - x0
    L("s_sub_i32 %[ta], %[x1], %[x0]")
    L(f"v_mul_f32_e32 {PX}, %[A], {QX}")                     # A qx
    L(f"v_cmp_ge_u32_e32 vcc, %[ta], {TMP}")                # col in [x0, x1]
    L(f"v_fma_f32 {PX}, {PX}, {QX}, %[la]")                 # A qx^2 + log2 a
    L("s_and_b32 %[ta], " + DCUR + ", 0xffff")              # this visit's block (offset from .Lpc)
    L(f"v_mul_f32_e32 {BX}, %[Bc], {QX}")                   # bx = Bc qx
    L(f"v_cndmask_b32_e32 {PX}, v141, {PX}, vcc")           # px = -inf outside [x0, x1]
    L(f"v_pk_add_f32 {QY}, {YB}, %[rcy] op_sel:[0,1] neg_lo:[0,1] neg_hi:[0,1]")   # qy = Yb - cy
    L(f"s_getpc_b64 {PC}")
    label("pc")
    L(f"s_add_u32 {PCLO}, {PCLO}, %[ta]")
    L(f"s_addc_u32 {PCHI}, {PCHI}, 0")
    L("s_bitcmp1_b32 %[rho4], 31")                          # flagged for the seed guard (make_rec)
    L("s_cbranch_scc1 .LGUARD%=")
    L(f"s_setpc_b64 {PC}")
    # ---------------- GUARD (flagged splats): a live lane's seed below 2^-100 ----------------
    label("GUARD")
    L("s_max_i32 %[tb], %[d0], 0")
    L("s_lshr_b32 %[tb], %[tb], 3")
    L("s_min_u32 %[tb], %[tb], 15")
    L("s_lshl_b32 %[tb], %[tb], 3")
    L(f"v_cvt_f32_i32_e32 {QX}, %[tb]")                     # 8 kA
    L(f"v_add_f32_e32 v134, v128, {QX}")                    # qy of pair kA
    L(f"v_add_f32_e32 v135, v129, {QX}")
    L(f"v_pk_fma_f32 {E}, %[cc], {W}, {BXP} op_sel_hi:[0,1,0]")
    L(f"v_pk_fma_f32 {E}, {W}, {E}, {PXP} op_sel_hi:[1,1,0]")
    L("v_exp_f32_e32 v136, v136")
    L("v_exp_f32_e32 v137, v137")
    L(f"v_min_u32_e32 {TMP}, v136, v137")
    L(f"v_cmp_lt_f32_e32 vcc, {NINF_LIT}, {PX}")            # live lane
    L(f"s_mov_b64 {WA}, vcc")
    L(f"v_cmp_gt_u32_e32 vcc, 0x0D800000, {TMP}")           # seed below 2^-100
    L(f"s_and_b64 {WA}, {WA}, vcc")
    L(f"s_cmp_lg_u64 {WA}, 0")
    L("s_cbranch_scc1 .LEXACT%=")
    L(f"s_setpc_b64 {PC}")

    # ---------------- FULL ----------------
    label("FULL")
    L(f"v_pk_fma_f32 {E}, %[cc], {QY}, {BXP} op_sel_hi:[0,1,0]")
    L(f"v_pk_fma_f32 {E}, {QY}, {E}, {PXP} op_sel_hi:[1,1,0]")
    L("v_exp_f32_e32 v130, v136")
    L("v_exp_f32_e32 v131, v137")
    L(f"v_mul_f32_e32 {TMP}, 0x41000000, {BX}")
    L(f"v_fmac_f32_e32 {TMP}, %[c16], v129")
    L(f"v_min_f32_e32 {TMP}, 0x42c80000, {TMP}")
    L(f"v_exp_f32_e32 v132, {TMP}")
    L("v_mul_f32_e64 v133, |%[rho4]|, v132")
    for k in range(NPK):
        pair_step(k, r_update=k < NPK - 2, f_update=k < NPK - 1)
    L("s_branch .Lend%=")

    # ---------------- F1[k]: one-pair visits ----------------
    for k in range(NPK):
        label(f"F1_{k}")
        # row limits relative to pair k (s_addk: a fixed-size 16-bit immediate, so
        # every block of the kind has the same length)
        L("s_mov_b32 %[sj], %[d0]")
        L(f"s_addk_i32 %[sj], {-8 * k}")
        L("s_mov_b32 %[sm], %[d1]")
        L(f"s_addk_i32 %[sm], {-8 * k}")
        seed(k, False)
        L("s_add_i32 %[sj4], %[sj], -4")                    # (the pair's second row is ph + 4)
        L("s_add_i32 %[sm4], %[sm], -4")
        L(f"v_cmp_ge_i32_e64 {MX}, {PH}, %[sj]")            # row >= y0
        L(f"v_cmp_ge_i32_e32 vcc, %[sm], {PH}")             # row <= y1
        L(f"s_and_b64 {MX}, {MX}, vcc")
        L(f"v_cmp_ge_i32_e64 {MY}, {PH}, %[sj4]")
        L(f"v_cmp_ge_i32_e32 vcc, %[sm4], {PH}")
        L(f"s_and_b64 {MY}, {MY}, vcc")
        L(f"v_cndmask_b32_e64 v136, 0, v130, {MX}")
        L(f"v_cndmask_b32_e64 v137, 0, v131, {MY}")
        blend_masked(k)
        L("s_branch .Lend%=")

    # ---------------- FM[k]: first pair k of a multi-pair visit ----------------
    # S_kB blocks all have SSZ bytes (front padding), so the walk entry for (k, kB)
    # is S_1 + (kB-1) SSZ + (15 - kB + k) PSZ: the descriptor's high half carries
    # kB (SSZ - PSZ), the rest is a constant of the block (relative to FM_k).
    for k in range(NPK):
        label(f"FM_{k}")
        L("s_mov_b32 %[sj], %[d0]")
        L(f"s_addk_i32 %[sj], {-8 * k}")
        seed(k, True)
        L("s_add_i32 %[sj4], %[sj], -4")
        L(f"v_cmp_ge_i32_e64 {MX}, {PH}, %[sj]")
        L(f"v_cmp_ge_i32_e64 {MY}, {PH}, %[sj4]")
        L("s_lshr_b32 %[tb], " + DCUR + ", 16")
        L(f"v_cndmask_b32_e64 v136, 0, v130, {MX}")
        L(f"v_cndmask_b32_e64 v137, 0, v131, {MY}")
        L(f"s_add_u32 %[tb], %[tb], .LS1%= - .LFM_{k}%= - {SSZ} + {(15 + k) * PSZ}")
        L(f"v_pk_mul_f32 {W}, {acc(k, 3)}, {E}")
        L(f"v_pk_mul_f32 {F}, {F}, {RT}")                   # f_{k+1}
        L(f"v_pk_mul_f32 {RT}, {RT}, %[rl] op_sel_hi:[1,0]")  # r_{k+1}
        L(f"v_pk_fma_f32 {acc(k, 0)}, %[rcy], {W}, {acc(k, 0)} op_sel_hi:[0,1,1]")
        L(f"v_pk_fma_f32 {acc(k, 1)}, %[ga], {W}, {acc(k, 1)} op_sel_hi:[0,1,1]")
        L(f"v_pk_fma_f32 {acc(k, 2)}, %[bb], {W}, {acc(k, 2)} op_sel_hi:[0,1,1]")
        L(f"v_pk_add_f32 {acc(k, 3)}, {acc(k, 3)}, {W} neg_lo:[0,1] neg_hi:[0,1]")
        L(f"s_add_u32 {WALO}, {PCLO}, %[tb]")               # PC = this block's address
        L(f"s_addc_u32 {WAHI}, {PCHI}, 0")
        L(f"s_setpc_b64 {WA}")

    # ---------------- S_kB: [padding] pairs 1 .. kB-1, then the masked last pair kB ----------------
    for kb in range(1, NPK):
        label(f"S{kb}")
        if kb < NPK - 1:
            L(f".skip {(NPK - 1 - kb) * PSZ}")             # never executed: keeps SSZ constant
        for k in range(1, kb):
            label(f"P{kb}_{k}")
            pair_step(k)
        label(f"LAST{kb}")
        L("s_mov_b32 %[sm], %[d1]")
        L(f"s_addk_i32 %[sm], {-8 * kb}")
        L("s_add_i32 %[sm4], %[sm], -4")
        L(f"v_cmp_ge_i32_e64 {MX}, %[sm], {PH}")            # row <= y1
        L(f"v_cmp_ge_i32_e64 {MY}, %[sm4], {PH}")
        L(f"v_cndmask_b32_e64 v136, 0, v130, {MX}")
        L(f"v_cndmask_b32_e64 v137, 0, v131, {MY}")
        blend_masked(kb)
        L("s_branch .Lend%=")
        label(f"END{kb}")

    # ---------------- EXACT: the guard tripped ----------------
    label("EXACT")
    L(f"v_pk_add_f32 {QY}, {YB}, %[rcy] op_sel:[0,1] neg_lo:[0,1] neg_hi:[0,1]")   # qy of pair 0
    for k in range(NPK):
        L(f"v_mov_b32_e32 {QX}, {float_lit(8.0 * k)}")
        L("s_sub_i32 %[ta], %[d0], " + str(8 * k))          # row limits rel. to pair k
        L("s_sub_i32 %[tb], %[d1], " + str(8 * k))
        L("s_sub_i32 %[sj4], %[d0], " + str(8 * k + 4))
        L("s_sub_i32 %[sm4], %[d1], " + str(8 * k + 4))
        L(f"v_pk_add_f32 {W}, {QY}, v[138:139] op_sel_hi:[1,0]")       # qy + 8k (one rounding)
        L(f"v_pk_fma_f32 {E}, %[cc], {W}, {BXP} op_sel_hi:[0,1,0]")
        L(f"v_pk_fma_f32 {E}, {W}, {E}, {PXP} op_sel_hi:[1,1,0]")
        L(f"v_exp_f32_e32 v136, v136")
        L(f"v_exp_f32_e32 v137, v137")
        L(f"v_cmp_ge_i32_e64 {MX}, {PH}, %[ta]")
        L(f"v_cmp_ge_i32_e32 vcc, %[tb], {PH}")
        L(f"s_and_b64 {MX}, {MX}, vcc")
        L(f"v_cmp_ge_i32_e64 {MY}, {PH}, %[sj4]")
        L(f"v_cmp_ge_i32_e32 vcc, %[sm4], {PH}")
        L(f"s_and_b64 {MY}, {MY}, vcc")
        L(f"v_cndmask_b32_e64 v136, 0, v136, {MX}")
        L(f"v_cndmask_b32_e64 v137, 0, v137, {MY}")
        blend_masked(k)
    label("end")
    L("s_nop 0")                     # the code after the asm may read what the last VALU op wrote


def float_lit(x):
    import struct
    return "0x%08x" % struct.unpack("<I", struct.pack("<f", x))[0]


# ---------------- hazard pass ----------------
REG = re.compile(r"\b([vs])\[(\d+):(\d+)\]|\b([vs])(\d+)\b|\bvcc\b|%\[(\w+)\]")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out |= {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
        elif m.group(4):
            out.add(f"{m.group(4)}{m.group(5)}")
        elif m.group(6):
            out.add("%" + m.group(6))
        else:
            out.add("vcc")
    return out


def dst_src(line):
    """(opcode, registers written, registers read) of one instruction line."""
    op, _, rest = line.partition(" ")
    parts = [p.strip() for p in rest.split(",")] if rest else []
    if not parts:
        return op, set(), set()
    if op.startswith(("s_cmp", "s_setpc", "s_branch", "s_cbranch", "s_nop")):
        return op, set(), regs(rest)
    d, s = regs(parts[0]), regs(",".join(parts[1:]))
    if op == "v_fmac_f32_e32":
        s |= d
    return op, d, s


def with_hazard_nops(src):
    """One wait state (s_nop 0) between a VALU result and an instruction that reads
    it next (labels are transparent: jumps only ever come from SALU instructions)."""
    out, prev_valu_dst = [], set()
    for line in src:
        if line.startswith(".L"):
            out.append(line)
            continue
        op, d, s = dst_src(line)
        if prev_valu_dst & s:
            out.append("s_nop 0")
        out.append(line)
        prev_valu_dst = d if op.startswith("v_") else set()
    return out


INLINE_INT = range(-16, 65)
INLINE_F32 = {0x00000000, 0x3F000000, 0xBF000000, 0x3F800000, 0xBF800000, 0x40000000, 0xC0000000,
              0x40800000, 0xC0800000, 0x3E22F983}


def has_literal(ops):
    for o in ops:
        o = o.strip()
        if ".L" in o:
            return True                                   # label expression: a fixup literal
        if re.fullmatch(r"-?\d+", o):
            if int(o) not in INLINE_INT:
                return True
        elif re.fullmatch(r"0x[0-9a-fA-F]+", o):
            v = int(o, 16)
            if v not in INLINE_F32 and v not in INLINE_INT:
                return True
    return False


def isize(line):
    """Encoded bytes of one line (gfx950): the layout model behind the C++ constants,
    checked against the assembler by the .if assertions."""
    if line.startswith(".skip"):
        return int(line.split()[1])
    if line.startswith("."):
        return 0
    op, _, rest = line.partition(" ")
    ops = [o.strip().split(" ")[0] for o in rest.split(",")] if rest else []
    if op.startswith("v_pk_") or op.endswith("_e64") or op in ("v_fma_f32", "v_readlane_b32"):
        return 8
    if op.startswith("s_load"):
        return 8
    if op.startswith(("s_addk", "s_branch", "s_cbranch", "s_nop", "s_waitcnt")):
        return 4                                          # SOPK / SOPP: immediate in the word
    return 4 + (4 if has_literal(ops) else 0)


def offsets(body):
    pos, labels = 0, {}
    for ln in body:
        if ln.startswith(".L") and ln.endswith(":"):
            labels[ln[2:-3]] = pos                          # ".Lname%=:" -> name
        pos += isize(ln)
    return labels


# Record sets: the current record's 16 dwords in s[cur:cur+15], the next one is
# loaded into s[nxt:nxt+15] at the start of the visit (SplatRec field order).
REC_A, REC_B = 56, 72
DESC_A, DESC_B = 54, 55
FIELDS = ["Cc", "cx", "r", "cy", "g", "A", "b", "Bc", "rho", "la", "c16", "rho4", "x0", "x1", "y0", "y1"]
PAIRS = {"cc": 0, "rcy": 2, "ga": 4, "bb": 6, "rl": 8}


def bind(text, cur, dcur, dnxt):
    for name, off in PAIRS.items():
        text = text.replace(f"%[{name}]", f"s[{cur + off}:{cur + off + 1}]")
    for i, name in enumerate(FIELDS):
        text = text.replace(f"%[{name}]", f"s{cur + i}")
    return text.replace("%[dcur]", f"s{dcur}").replace("%[dnxt]", f"s{dnxt}")


def main():
    gen()
    print("// Generated by gen_visit_asm.py -- do not edit.  The raster visit as one asm block:")
    print("// wait for the current record, prefetch the next record and descriptor, visit.")
    print(f"// _A: current record s[{REC_A}:{REC_A + 15}] / descriptor s{DESC_A}, next into "
          f"s[{REC_B}:{REC_B + 15}] / s{DESC_B}; _B: the other way round.")
    lay = None
    for tag, cur, nxt, dcur, dnxt in (("A", REC_A, REC_B, DESC_A, DESC_B), ("B", REC_B, REC_A, DESC_B, DESC_A)):
        head = ["s_waitcnt lgkmcnt(0)",
                "v_readlane_b32 %[ta], %[offv], %[lane]",
                f"v_readlane_b32 s{dnxt}, %[descv], %[lane]",
                f"s_load_dwordx16 s[{nxt}:{nxt + 15}], %[base], %[ta]"]
        body = with_hazard_nops([bind(ln, cur, dcur, dnxt) for ln in head + lines])
        o = offsets(body)
        rel = {k: v - o["pc"] for k, v in o.items()}
        mine = {"FULL": rel["FULL"], "F1_0": rel["F1_0"], "F1SZ": rel["F1_1"] - rel["F1_0"],
                "FM_0": rel["FM_0"], "FMSZ": rel["FM_1"] - rel["FM_0"], "SSZ": rel["S2"] - rel["S1"]}
        assert lay is None or lay == mine, "A and B layouts differ"
        lay = mine
        chk = []

        def same(a, b, what):
            chk.append(f".if ({a}) != ({b})")
            chk.append(f'.error "visit asm layout: {what}"')
            chk.append(".endif")
        for k in range(NPK):
            same(f".LF1_{k}%= - .Lpc%=", lay["F1_0"] + k * lay["F1SZ"], f"F1 block {k}")
            same(f".LFM_{k}%= - .Lpc%=", lay["FM_0"] + k * lay["FMSZ"], f"FM block {k}")
        same(".LFULL%= - .Lpc%=", lay["FULL"], "FULL")
        same(".LS1%= - .LFM_15%=", lay["FMSZ"], "FM block 15")
        same(".LP3_2%= - .LP3_1%=", PSZ, "pair step size")
        for kb in range(1, NPK):
            same(f".LS{kb}%= - .LS1%=", lay["SSZ"] * (kb - 1), f"S{kb} start")
            for k in range(1, kb):
                same(f".LP{kb}_{k}%= - .LS{kb}%=", PSZ * (NPK - 1 - kb + k - 1), f"P{kb}_{k}")
            same(f".LLAST{kb}%= - .LS{kb}%=", PSZ * (NPK - 2), f"LAST{kb}")
        same(".LEXACT%= - .LS15%=", lay["SSZ"], "S15 end")
        print(f"#define GGS_VISIT_ASM_{tag} \\")
        for ln in body + chk:
            print('    "' + ln.replace('"', '\\"') + '\\n\\t" \\')
        print('    ""')
    print("// block offsets from the dispatch point (.Lpc), for the cull's visit descriptors")
    print(f"#define GGS_VOFF_FULL {lay['FULL']}")
    print(f"#define GGS_VOFF_F1 {lay['F1_0']}")
    print(f"#define GGS_VF1SZ {lay['F1SZ']}")
    print(f"#define GGS_VOFF_FM {lay['FM_0']}")
    print(f"#define GGS_VFMSZ {lay['FMSZ']}")
    print(f"#define GGS_VSSZ_PSZ {lay['SSZ'] - PSZ}")


if __name__ == "__main__":
    main()
