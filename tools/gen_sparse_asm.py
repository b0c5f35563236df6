"""Generate fastselect_amd/csrc/fs_sparse_asm.inc: the inner loop of
k_score_sparse (continuous feature blocks) as one inline-asm block.

Layout (k_weights_sparse): the 128 columns of a tile are dealt to the 16
waves of a workgroup, wave w taking jj = w, w + 16, ... (8 columns).  Its
stream is the groups of those columns back to back: group = 8 entries
(roff, w) = 16 dwords = one s_load_dwordx16; roff = row * 1024 (the row's
byte offset in the LDS block, 64 lanes x float4); a column's entries are
padded with (0, 0) to whole groups and the lowest mantissa bit of the first
weight of the column's last group is set (every other weight has it clear;
the 1-ulp change is far below the 1e-5 parity bar).  Lane l scores features
f0 + l + 64k, k = 0..3, held in LDS as one float4 per row.

feats=2, low=True (measured, not shipped): a 64 KB row block and <= 64
VGPRs, so two 1024-thread workgroups share a CU (8 waves per SIMD).  On
synthetic 42%-dense streams (tools/ubench/sparse_bench) it took 7.77 cycles
per entry-feature against 8.68 for feats=4 at 4 waves per SIMD.  In
k_score_sparse at cfg4 (profiles/ubench/r01k_*) VALU busy rose from 53.5% to
64.6%, but the clock fell from 2.26 to 2.04 GHz (power) and the loop issues
9% more VALU instructions per pair-feature (one address add per 2 features
instead of per 4): 105.4 ms against 104.6, so feats=4 stays.  The register
numbers below are those of feats=4; low=True maps the SGPRs as described at
the remap.

pk=True (measured, not shipped): the four differences of an entry as two
v_pk_add_f32 (7 instead of 9 VALU instructions per entry).  In
k_score_sparse at cfg4, alternating on one box (tools/pk_ab.sh,
profiles/ubench/r01k_pk_ab.txt): 124.1 / 124.1 ms against 104.2 / 105.0 for
the v_sub_f32 loop -- packed f32 costs more issue time than its two halves.

lead (default 2): rows of g+1 issued before g's first entry; the rest one per
entry.  Same-box A/B (tools/lead_ab.sh, profiles/ubench/r01l_lead_ab.txt):
lead 1 / 0 / 2 within run-to-run noise (102.0-105.5 ms), 3 / 4 / 6 slower
(103.3 / 104.3 / 104.9 against 102.6), -1 (last row after the last entry)
106.1-106.4.

prio (A/B only): s_setprio 1 or 3 from the group's wait to its second entry.
Same box, alternating (profiles/ubench/r01l_prio_ab.txt, "lead" column = V):
104.3 / 104.7 ms plain, 103.3 / 104.0 with 1, 104.1 / 103.9 with 3 -- noise.

Pipeline per group g (unrolled x6: 3 SGPR sets x 2 A sets):
  s_waitcnt lgkmcnt(0)            A values of g (LDS) and entries of g+1 (SMEM) landed
  s_load_dwordx16                 entries of g+2 (stream offset += 64)
  8 x 4 x (v_sub_f32, v_fma_f32)  group g: acc += w * |a - b|, with the 8
                                  (v_add_u32, ds_read_b128) of g+1's rows spread
                                  over it (2 up front, then one per entry: 5%
                                  faster than issuing them in one burst)
  s_bitcmp1_b32 / s_cbranch       end of g's column -> out-of-line switch: next
                                  column's B values (prefetched one column ahead)
SMEM returns out of order, so every wait is lgkmcnt(0), placed where both
the LDS reads and the scalar load it covers were issued a whole group of
arithmetic earlier.  Each group is ~72 VALU of the ~85 instructions issued.

Fixed registers (clobbered; the compiler keeps its own values elsewhere):
  v64..v127 two A sets (8 x float4)     v56..v59 B (current column), v60..v63 next
  v48..v55  |diff| temporaries          s40..s87 three entry sets (16 SGPRs)
  s[36:37]  stream base                 s34 stream offset, s35 temporary
  s88       column counter              s[90:91] B row pointer
"""
import os
import re

SETS = [40, 56, 72]


def gen(name="FS_SPARSE_STREAM_ASM", no_ds=False, same_stream=False, feats=4, spread=True, low=False,
        pk=False, lead=2, prio=0, warm=0):
    """Macro text.  feats: features per lane (4: 128 KB LDS block, float4 rows;
    2: 64 KB, float2 rows, 64-VGPR budget).  no_ds / same_stream:
    microbenchmark variants that skip the LDS reads / keep re-reading the
    stream's first groups (scalar-cache hits)."""
    F = feats
    if F == 4:
        ASETS, BCUR, BNXT, TMP, VLO = [64, 96], 56, 60, [48, 52], 48
        rd = "ds_read_b128"
    else:
        ASETS, BCUR, BNXT, TMP, VLO = [32, 48], 26, 28, [22, 24], 22
        rd = "ds_read_b64"

    def issue_rows(k, a):
        s, A = SETS[k], ASETS[a]
        L = [f"v_add_u32 v{A + F * q}, s{s + 2 * q}, %[lane16]" for q in range(8)]
        if not no_ds:
            L += [f"{rd} v[{A + F * q}:{A + F * q + F - 1}], v{A + F * q}" for q in range(8)]
        return L

    def compute(k, a):
        s, A = SETS[k], ASETS[a]
        L = []
        for q in range(8):
            t = TMP[q % 2]
            w = f"s{s + 2 * q + 1}"
            if pk:  # two differences per instruction (b negated in both halves)
                for f in range(0, F, 2):
                    L.append(f"v_pk_add_f32 v[{t + f}:{t + f + 1}], v[{A + F * q + f}:{A + F * q + f + 1}], "
                             f"v[{BCUR + f}:{BCUR + f + 1}] neg_lo:[0,1] neg_hi:[0,1]")
            else:
                for f in range(F):
                    L.append(f"v_sub_f32 v{t + f}, v{A + F * q + f}, v{BCUR + f}")
            for f in range(F):
                acc = f"%[acc{2 * f + (q & 1)}]"
                L.append(f"v_fma_f32 {acc}, {w}, |v{t + f}|, {acc}")
        return L

    def bload(dst):
        return [f"global_load_dword v{dst + f}, %[lane4], s[90:91]" + (f" offset:{256 * f}" if f else "")
                for f in range(F)]

    def step(x):
        c, n, nn = x % 3, (x + 1) % 3, (x + 2) % 3
        ac, an = x % 2, (x + 1) % 2
        L = ["s_waitcnt lgkmcnt(0)"]
        if prio:  # raised while the wave issues the group's loads (A/B)
            L.append(f"s_setprio {prio}")
        rows = issue_rows(n, an)
        if not spread:
            L += rows
        L.append("s_add_u32 s34, s34, 64")
        if same_stream:  # two groups re-read (scalar-cache hits); s89 bounds the loop
            L += ["s_and_b32 s34, s34, 0x40", "s_add_u32 s89, s89, 1"]
        L.append(f"s_load_dwordx16 s[{SETS[nn]}:{SETS[nn] + 15}], s[36:37], s34")
        if warm:
            # L2 warm-up of the group `warm` groups beyond the one just
            # requested: a vector load (vmcnt, not lgkmcnt) whose value is
            # discarded, so the scalar load of that group ~warm steps later
            # finds its line in L2 instead of HBM
            L += ["s_add_u32 s92, s36, s34", "s_addc_u32 s93, s37, 0",
                  f"global_load_dword v47, v46, s[92:93] offset:{64 * warm}"]
        if not spread:
            L += compute(c, ac)
        else:
            # (v_add, ds_read) of row q of g+1 after entry q-2 of g: the LDS
            # requests spread over the first 3/4 of the arithmetic
            comp = compute(c, ac)
            per = len(comp) // 8
            adds, reads = rows[:8], rows[8:] if not no_ds else [""] * 8
            for q in range(8):
                if q < lead:
                    L += [adds[q]] + ([reads[q]] if reads[q] else [])
            for e in range(8):
                L += comp[e * per:(e + 1) * per]
                if prio and e == 1:
                    L.append("s_setprio 0")
                q = e + lead
                if 0 <= q < 8:
                    L += [adds[q]] + ([reads[q]] if reads[q] else [])
            for q in range(max(0, 8 + lead), 8):  # lead < 0: the rest after the last entry
                L += [adds[q]] + ([reads[q]] if reads[q] else [])
        L.append(f"s_bitcmp1_b32 s{SETS[c] + 1}, 0")
        L.append(f"s_cbranch_scc1 {10 + x}f")
        L.append(f"{20 + x}:")
        return L

    def switch(x):
        # column switch after step x (out of line); returns to label 20+x
        return [f"{10 + x}:",
                "s_add_u32 s88, s88, 1",
                "s_cmp_ge_u32 s88, %[ncols]",
                "s_cbranch_scc1 8f",
                "s_waitcnt vmcnt(0)",
                *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(F)],
                "s_add_u32 s35, s88, 1",
                "s_cmp_ge_u32 s35, %[ncols]",
                f"s_cbranch_scc1 {20 + x}b",
                "s_add_u32 s90, s90, %[bstride]",
                "s_addc_u32 s91, s91, 0",
                *bload(BNXT),
                f"s_branch {20 + x}b"]

    lines = [
        *(["v_mov_b32 v46, 0"] if warm else []),  # the warm loads' zero offset (own register:
        # an input operand holding 0 may share the register of an accumulator)
        "s_mov_b32 s88, 0",
        "s_mov_b64 s[90:91], %[bp]",
        *bload(BCUR),
        "s_add_u32 s90, s90, %[bstride]",
        "s_addc_u32 s91, s91, 0",
        *bload(BNXT),
        "s_mov_b64 s[36:37], %[eb]",
        "s_mov_b32 s34, 0",
        "s_load_dwordx16 s[40:55], s[36:37], s34",
        "s_waitcnt lgkmcnt(0)",
    ]
    lines += issue_rows(0, 0)
    lines.append("s_add_u32 s34, s34, 64")
    lines.append("s_load_dwordx16 s[56:71], s[36:37], s34")
    lines.append(f"s_waitcnt vmcnt({F})")
    lines.append("7:")
    for x in range(6):
        lines += step(x)
    # safety bound: a stream holds at most 8 columns x 16 groups (8 KB)
    if same_stream:
        lines.insert(0, "s_mov_b32 s89, 0")
        lines += ["s_cmp_gt_u32 s89, 128", "s_cbranch_scc0 7b", "s_branch 8f"]
    else:
        lines += ["s_cmp_gt_u32 s34, 0x2040", "s_cbranch_scc0 7b", "s_branch 8f"]
    for x in range(6):
        lines += switch(x)
    lines.append("8:")
    lines.append("s_waitcnt vmcnt(0) lgkmcnt(0)")

    # low: the fixed SGPRs moved below s72 (reserved at 8 waves/SIMD), around
    # s32/s33 (the ABI's stack and frame pointers): entry sets at s16, s36,
    # s52; stream base s[12:13], column counter s14, s15; offset s68,
    # temporary s69, B row pointer s[70:71].  The compiler keeps s0..s11.
    remap = {}
    if low:
        for k, base in enumerate((16, 36, 52)):
            for i in range(16):
                remap[SETS[k] + i] = base + i
        remap.update({34: 68, 35: 69, 36: 12, 37: 13, 88: 14, 89: 15, 90: 70, 91: 71})

        def sub(m):
            lo, hi = int(m.group(1)), m.group(2)
            if lo not in remap:
                return m.group(0)
            return f"s[{remap[lo]}:{remap[int(hi)]}]" if hi else f"s{remap[lo]}"
        lines = [re.sub(r"(?<![a-z_])s\[?(\d+)(?::(\d+)\])?", sub, l) for l in lines]
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vlo = VLO - 2 if warm else VLO
    vclob = ", ".join(f'"v{i}"' for i in range(vlo, ASETS[1] + 8 * F))
    nacc = 2 * F
    # low: clobber only the SGPRs the loop names (the compiler has few left)
    named = set()
    for l in lines:
        for lo, hi in re.findall(r"(?<![a-z_])s\[?(\d+)(?::(\d+)\])?", l):
            named.update(range(int(lo), int(hi or lo) + 1))
    sregs = sorted(named & set(remap.values())) if low else range(34, 94 if warm else 92)
    sclob = ", ".join(f'"s{i}"' for i in sregs)
    vz = ""
    return f'''#define {name}(acc, lane16, lane4, eb, bp, bstride, ncols)  \\
  asm volatile(  \\
{body}
      : {", ".join(f'[acc{i}] "+v"(acc[{i}])' for i in range(nacc))}  \\
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [eb] "s"(eb), [bp] "s"(bp),  \\
        [bstride] "s"(bstride), [ncols] "s"(ncols){vz}  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
'''


HEADER = """// Generated by tools/gen_sparse_asm.py -- do not edit by hand.
// Inner loops of k_score_sparse2 for continuous feature blocks (see the
// generator's docstring for the layout, the pipeline and the fixed registers).
"""

# ---------------------------------------------------------------------------
# v2 stream: entries through vector memory + DPP broadcast (no scalar loads)
# ---------------------------------------------------------------------------
DPP_DOC = """
Entries through vector memory (no scalar loads in the loop).  A stream (one
wave, one tile) is its groups back to back (64 B = 8 entries (roff, w)); the
group counts of its 8 columns come once per stream (s_load_dwordx4 of
{counts 0-3, counts 4-7, total, 0}).  Lane l loads entry (l & 15) of a group
pair (global_load_dwordx2, every 16-lane row holds the same 16 entries), and
entry q of group g is broadcast by DPP row_newbcast:(q + 8 (g & 1)) straight
into the instruction that uses it:
  v_add_u32_dpp    addr = roff + lane16           (LDS address of the row)
  v_fmac_f32_dpp   acc += w * |a - b|
so the pipeline waits are in-order counters only (vmcnt for entries and B,
lgkmcnt for the LDS rows) and can run several groups ahead:
  step g:  [g even] load entry pair g/2 + 3
           wait entries of g+1; 8 x (v_add_u32_dpp, ds_read_b128) rows of g+1
           wait B of g and rows of g (lgkmcnt(8))
           8 x (4 v_sub_f32, 4 v_fmac_f32_dpp)        group g
           4 x global_load_dword B of group g+4 (its column's row)
Fixed registers: v64..v127 two A sets, v48..v63 four B sets, v40..v47 four
entry pairs, v32..v39 |diff| temporaries; s36..s47 stream state.
"""


def gen_dpp(name="FS_SPARSE_STREAM_ASM", plain_fma=False, no_b=False, no_ds=False, plain_add=False):
    ASET = [64, 96]
    BSET = [48, 52, 56, 60]
    ESET = [40, 42, 44, 46]
    TMP = [32, 36]
    # s[36:37] entry pointer (next pair load), s[38:39] B row of the prefetch column,
    # s40 groups left in that column, s41 groups left to compute, s[42:43] counts of
    # the columns after it, s44 / s45 temporaries, s[46:47] {.., ..} of the count load
    vm = []      # issue log of vector-memory ops (labels), for the vmcnt values

    def eload(p):
        vm.append(("E", p))
        e = ESET[p % 4]
        return [f"global_load_dwordx2 v[{e}:{e + 1}], %[laneoff], s[36:37]",
                "s_add_u32 s36, s36, 0x80", "s_addc_u32 s37, s37, 0"]

    def bload(h):
        b = BSET[h % 4]
        L = []
        if no_b and h >= 4:
            return L
        for f in range(4):
            vm.append(("B", h))
            L.append(f"global_load_dword v{b + f}, %[lane4], s[38:39]" + (f" offset:{256 * f}" if f else ""))
        # advance the prefetch cursor: next group's column
        L += ["s_sub_u32 s40, s40, 1", "s_cmp_eq_u32 s40, 0", f"s_cbranch_scc0 {60 + h % 8}f",
              "s_and_b32 s40, s42, 0xff", "s_lshr_b64 s[42:43], s[42:43], 8",
              "s_cmp_eq_u32 s40, 0",
              "s_cselect_b32 s40, 0x7fffffff, s40",      # past the last column: stay
              "s_cselect_b32 s44, 0, %[bstride]",
              "s_add_u32 s38, s38, s44", "s_addc_u32 s39, s39, 0",
              f"{60 + h % 8}:"]
        return L

    def count_after(kind, idx):
        # VMEM ops issued after the newest op of (kind, idx)
        hits = [i for i, v in enumerate(vm) if v == (kind, idx)]
        return min(63, len(vm) - 1 - max(hits)) if hits else 63

    def rows(g):
        a = ASET[(g + 0) % 2]
        e = ESET[(g // 2) % 4]
        L = []
        for q in range(8):
            ln = q + 8 * (g % 2)
            L.append(f"v_add_u32_dpp v{a + 4 * q}, v{e}, %[lane16] row_newbcast:{ln} row_mask:0xf bank_mask:0xf")
        for q in range(8):
            L.append(f"ds_read_b128 v[{a + 4 * q}:{a + 4 * q + 3}], v{a + 4 * q}")
        return L

    def rows_into(g):
        a, e = ASET[g % 2], ESET[(g // 2) % 4]
        L = []
        for q in range(8):
            ln = q + 8 * (g % 2)
            if plain_add:
                L.append(f"v_add_u32 v{a + 4 * q}, v{e}, %[lane16]")
            else:
                L.append(f"v_add_u32_dpp v{a + 4 * q}, v{e}, %[lane16] row_newbcast:{ln} row_mask:0xf bank_mask:0xf")
        if not no_ds:
            for q in range(8):
                L.append(f"ds_read_b128 v[{a + 4 * q}:{a + 4 * q + 3}], v{a + 4 * q}")
        return L

    def compute(g):
        a, e, b = ASET[g % 2], ESET[(g // 2) % 4], BSET[g % 4]
        L = []
        for q in range(8):
            ln = q + 8 * (g % 2)
            t = TMP[q % 2]
            for f in range(4):
                L.append(f"v_sub_f32 v{t + f}, v{a + 4 * q + f}, v{b + f}")
            for f in range(4):
                acc = f"%[acc{2 * f + (q & 1)}]"
                if plain_fma:
                    L.append(f"v_fma_f32 {acc}, v{e + 1}, |v{t + f}|, {acc}")
                else:
                    L.append(f"v_fmac_f32_dpp {acc}, v{e + 1}, |v{t + f}| row_newbcast:{ln} row_mask:0xf bank_mask:0xf")
        return L

    head = ["s_load_dwordx4 s[40:43], %[cb], 0x0",   # s40 c0..3, s41 c4..7, s42 total
            "s_mov_b64 s[36:37], %[eb]", "s_mov_b64 s[38:39], %[bp]",
            "s_waitcnt lgkmcnt(0)",
            "s_mov_b32 s44, s42",                      # total groups
            "s_mov_b32 s42, s40", "s_mov_b32 s43, s41",   # counts word
            "s_mov_b32 s41, s44",
            "s_and_b32 s40, s42, 0xff", "s_lshr_b64 s[42:43], s[42:43], 8",
            "s_cmp_eq_u32 s41, 0", "s_cbranch_scc1 9f"]
    head += eload(0) + eload(1) + eload(2)
    for h in range(4):
        head += bload(h)
    head.append(f"s_waitcnt vmcnt({count_after('E', 0)})")
    head += rows(0)

    # Loop body: 8 steps.  vmcnt(N) is safe when N <= the number of vector
    # memory ops issued after the awaited one; the body is simulated for
    # several passes (pass 0 follows the prologue) and each wait takes the
    # minimum over the passes.
    waits = {}

    def body(pas, emit):
        out = []
        for g in range(8):
            G = 8 * pas + g                  # global group index in the simulation
            if g % 2 == 0:
                out += eload(G // 2 + 3)
            k = ("E", g)
            if not emit:
                waits[k] = min(waits.get(k, 99), count_after("E", (G + 1) // 2))
            out.append(f"s_waitcnt vmcnt({waits[k] if emit else 0})")
            out += rows_into(G + 1)
            k = ("B", g)
            if not emit:
                waits[k] = min(waits.get(k, 99), count_after("B", G))
            out.append(f"s_waitcnt vmcnt({waits[k] if emit else 0}) lgkmcnt(8)")
            out += compute(G)
            out += bload(G + 4)
            out += ["s_sub_u32 s41, s41, 1", "s_cmp_eq_u32 s41, 0", "s_cbranch_scc1 8f"]
        return out

    for pas in range(4):
        body(pas, False)
    lines = head
    lines.append("7:")
    lines += body(0, True)
    lines.append("s_branch 7b")
    lines.append("8:")
    lines.append("9:")
    lines.append("s_waitcnt vmcnt(0) lgkmcnt(0)")
    return lines, waits


def gen_dpp_macro(name="FS_SPARSE_STREAM_ASM", **opts):
    lines, _ = gen_dpp(name, **opts)
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(32, 128))
    sclob = ", ".join(f'"s{i}"' for i in range(36, 48))
    return f'''#define {name}(acc, lane16, lane4, laneoff, eb, cb, bp, bstride)  \\
  asm volatile(  \\
{body}
      : {", ".join(f'[acc{i}] "+v"(acc[{i}])' for i in range(8))}  \\
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [laneoff] "v"(laneoff), [eb] "s"(eb),  \\
        [cb] "s"(cb), [bp] "s"(bp), [bstride] "s"(bstride)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
'''


# ---------------------------------------------------------------------------
# 12-entry groups: weights and row bytes in one 64-byte scalar load
# ---------------------------------------------------------------------------
G12_DOC = """
Group of 12 entries = 16 dwords: weights w0..w11 (dwords 0-11), the rows as
bytes (dwords 12-14, row q in byte q % 4 of dword 12 + q / 4) and a flags
dword (15: bit 0 ends the column).  Same pipeline as the 8-entry loop; the
step is 1.5x longer per scalar load (cover) and a scalar-cache miss feeds 12
entries instead of 8.  Rows are unpacked by SALU (s_bfe_u32) and addressed
with v_lshl_add_u32 (row << 10) + lane16; the A values are differenced in
place (no temporaries).
Fixed registers: v32..v127 two A sets (12 x float4), v24..v27 B, v28..v31
next B; s40..s87 three entry sets, s88 column counter, s[90:91] B row
pointer, s[36:37] stream base, s34 stream offset, s35 / s89 temporaries.
"""


def gen12(name="FS_SPARSE_STREAM_ASM", spread=True, same_stream=False, no_ds=False):
    SETS12 = [40, 56, 72]
    ASETS12 = [32, 80]
    BCUR, BNXT = 24, 28

    def issue_rows(k, a):
        s, A = SETS12[k], ASETS12[a]
        adds, reads = [], []
        for q in range(12):
            adds.append([f"s_bfe_u32 s89, s{s + 12 + q // 4}, 0x{(8 << 16) | (8 * (q % 4)):x}",
                         f"v_lshl_add_u32 v{A + 4 * q}, s89, 10, %[lane16]"])
            reads.append([] if no_ds else [f"ds_read_b128 v[{A + 4 * q}:{A + 4 * q + 3}], v{A + 4 * q}"])
        return adds, reads

    def compute_entry(k, a, q):
        s, A = SETS12[k], ASETS12[a]
        w = f"s{s + q}"
        L = [f"v_sub_f32 v{A + 4 * q + f}, v{A + 4 * q + f}, v{BCUR + f}" for f in range(4)]
        for f in range(4):
            acc = f"%[acc{2 * f + (q & 1)}]"
            L.append(f"v_fma_f32 {acc}, {w}, |v{A + 4 * q + f}|, {acc}")
        return L

    def bload(dst):
        return [f"global_load_dword v{dst + f}, %[lane4], s[90:91]" + (f" offset:{256 * f}" if f else "")
                for f in range(4)]

    def step(x):
        c, n, nn = x % 3, (x + 1) % 3, (x + 2) % 3
        ac, an = x % 2, (x + 1) % 2
        L = ["s_waitcnt lgkmcnt(0)"]
        adds, reads = issue_rows(n, an)
        lead = 3 if spread else 12
        for q in range(lead):
            L += adds[q] + reads[q]
        L.append("s_add_u32 s34, s34, 64")
        if same_stream:
            L += ["s_and_b32 s34, s34, 0x40", "s_add_u32 s35, s35, 1"]
        L.append(f"s_load_dwordx16 s[{SETS12[nn]}:{SETS12[nn] + 15}], s[36:37], s34")
        for e in range(12):
            L += compute_entry(c, ac, e)
            q = e + lead
            if q < 12:
                L += adds[q] + reads[q]
        L.append(f"s_bitcmp1_b32 s{SETS12[c] + 15}, 0")
        L.append(f"s_cbranch_scc1 {10 + x}f")
        L.append(f"{20 + x}:")
        return L

    def switch(x):
        return [f"{10 + x}:",
                "s_add_u32 s88, s88, 1",
                "s_cmp_ge_u32 s88, %[ncols]",
                "s_cbranch_scc1 8f",
                "s_waitcnt vmcnt(0)",
                *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(4)],
                "s_add_u32 s89, s88, 1",
                "s_cmp_ge_u32 s89, %[ncols]",
                f"s_cbranch_scc1 {20 + x}b",
                "s_add_u32 s90, s90, %[bstride]",
                "s_addc_u32 s91, s91, 0",
                *bload(BNXT),
                f"s_branch {20 + x}b"]

    lines = ["s_mov_b32 s88, 0", "s_mov_b32 s35, 0",
             "s_mov_b64 s[90:91], %[bp]", *bload(BCUR),
             "s_add_u32 s90, s90, %[bstride]", "s_addc_u32 s91, s91, 0", *bload(BNXT),
             "s_mov_b64 s[36:37], %[eb]", "s_mov_b32 s34, 0",
             "s_load_dwordx16 s[40:55], s[36:37], s34",
             "s_waitcnt lgkmcnt(0)"]
    adds, reads = issue_rows(0, 0)
    for q in range(12):
        lines += adds[q] + reads[q]
    lines += ["s_add_u32 s34, s34, 64", "s_load_dwordx16 s[56:71], s[36:37], s34", "s_waitcnt vmcnt(4)", "7:"]
    for x in range(6):
        lines += step(x)
    if same_stream:
        lines += ["s_cmp_gt_u32 s35, 96", "s_cbranch_scc0 7b", "s_branch 8f"]
    else:
        # safety bound: a stream holds at most 8 columns x 11 groups (5632 B)
        lines += ["s_cmp_gt_u32 s34, 0x1640", "s_cbranch_scc0 7b", "s_branch 8f"]
    for x in range(6):
        lines += switch(x)
    lines += ["8:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(24, 128))
    sclob = ", ".join(f'"s{i}"' for i in range(34, 92))
    return f'''#define {name}(acc, lane16, lane4, eb, bp, bstride, ncols)  \\
  asm volatile(  \\
{body}
      : {", ".join(f'[acc{i}] "+v"(acc[{i}])' for i in range(8))}  \\
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [eb] "s"(eb), [bp] "s"(bp),  \\
        [bstride] "s"(bstride), [ncols] "s"(ncols)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
'''


# ---------------------------------------------------------------------------
# v3: entries staged through an LDS ring (LDS-DMA), no scalar loads in the loop
# ---------------------------------------------------------------------------
RING_DOC = """
Stream layout (SoA groups): group = 16 dwords, rows' LDS byte offsets r0..r7
then weights w0..w7; per stream a uint4 {group counts of columns 0-3 as bytes,
of columns 4-7, total groups, 0}.  Each wave owns a 2 KB LDS ring (32 groups,
two 1 KB halves) filled by LDS-DMA (global_load_lds_dwordx4: 16 groups per
instruction) one half ahead; the entries reach VGPRs by wave-uniform
ds_read_b128 (every lane the same 16 bytes), so every wait is an in-order
counter: lgkmcnt for LDS (no scalar loads outstanding in the loop) and vmcnt
for LDS-DMA and B.  Step g (unrolled x32: static ring offsets):
  lgkmcnt(2)                  roffs of g+1 landed (weights of g may be in flight)
  [g+2 starts a ring half: wait for its LDS-DMA]
  8 x (v_add_u32, ds_read_b128)  rows of g+1
  2 x ds_read_b128 roffs of g+2, 2 x ds_read_b128 weights of g+1
  lgkmcnt(12)                 rows and weights of g landed
  [g+1 starts a ring half: LDS-DMA of the half after next into the free half]
  8 x 4 x (v_sub_f32 in place, v_fma_f32 w * |d|)   group g
  column / stream bookkeeping in SALU (group counts from the stream's uint4)
Fixed registers: v64..v127 two A sets, v48..v63 two roff sets, v32..v47 two
weight sets, v24..v27 B, v28..v31 next B; s36..s50 (M0 saved in s46).
"""


def gen_ring(name="FS_SPARSE_RING_ASM", spread=False):
    ASET = [64, 96]
    RSET = [48, 56]
    WSET = [32, 40]
    BCUR, BNXT = 24, 28

    def bload(dst):
        return [f"global_load_dword v{dst + f}, %[lane4], s[38:39]" + (f" offset:{256 * f}" if f else "")
                for f in range(4)]

    def rows(g):
        A, R = ASET[g % 2], RSET[g % 2]
        adds = [f"v_add_u32 v{A + 4 * q}, v{R + q}, %[lane16]" for q in range(8)]
        reads = [f"ds_read_b128 v[{A + 4 * q}:{A + 4 * q + 3}], v{A + 4 * q}" for q in range(8)]
        return adds, reads

    def entry_reads(g):
        R, W = RSET[(g + 2) % 2], WSET[(g + 1) % 2]
        ro = ((g + 2) % 32) * 64
        wo = ((g + 1) % 32) * 64 + 32
        return [f"ds_read_b128 v[{R}:{R + 3}], %[ringv] offset:{ro}",
                f"ds_read_b128 v[{R + 4}:{R + 7}], %[ringv] offset:{ro + 16}",
                f"ds_read_b128 v[{W}:{W + 3}], %[ringv] offset:{wo}",
                f"ds_read_b128 v[{W + 4}:{W + 7}], %[ringv] offset:{wo + 16}"]

    def compute_entry(g, q):
        A, W = ASET[g % 2], WSET[g % 2]
        L = [f"v_sub_f32 v{A + 4 * q + f}, v{A + 4 * q + f}, v{BCUR + f}" for f in range(4)]
        for f in range(4):
            acc = f"%[acc{2 * f + (q & 1)}]"
            L.append(f"v_fma_f32 {acc}, v{W + q}, |v{A + 4 * q + f}|, {acc}")
        return L

    def dma(half_off):
        return ([f"s_add_u32 s44, s47, {half_off}"] if half_off else ["s_mov_b32 s44, s47"]) + [
            "s_mov_b32 m0, s44", "s_nop 0",
            "global_load_lds_dwordx4 %[laneoff], s[36:37]",
            "s_add_u32 s36, s36, 0x400", "s_addc_u32 s37, s37, 0"]

    def step(x):
        g = x
        L = ["s_waitcnt lgkmcnt(2)"]
        if (g + 2) % 16 == 0:   # g+2 opens a ring half: its LDS-DMA must have landed
            L += ["s_cmp_eq_u32 s48, 0", f"s_cbranch_scc1 {100 + x}f", "s_waitcnt vmcnt(4)",
                  f"s_branch {200 + x}f", f"{100 + x}:", "s_waitcnt vmcnt(0)", f"{200 + x}:"]
        adds, reads = rows(g + 1)
        if not spread:
            for q in range(8):
                L += [adds[q], reads[q]]
            L += entry_reads(g)
            L.append("s_waitcnt lgkmcnt(12)")
        else:
            raise NotImplementedError
        if (g + 1) % 16 == 0:   # the half after next goes into the half g's group left
            L += dma(0x400 if ((g + 1) // 16) % 2 == 0 else 0)
            L += ["s_mov_b32 s48, 0", "s_add_u32 s49, s49, 1"]
        for q in range(8):
            L += compute_entry(g, q)
        L += ["s_sub_u32 s40, s40, 1", "s_cmp_eq_u32 s40, 0", f"s_cbranch_scc1 {300 + x}f",
              f"{400 + x}:",
              "s_sub_u32 s41, s41, 1", "s_cmp_eq_u32 s41, 0", "s_cbranch_scc1 8f"]
        return L

    def switch(x):
        return [f"{300 + x}:",
                "s_and_b32 s40, s42, 0xff", "s_lshr_b64 s[42:43], s[42:43], 8",
                "s_cmp_eq_u32 s49, 0", f"s_cbranch_scc1 {500 + x}f", "s_waitcnt vmcnt(1)",
                f"s_branch {600 + x}f", f"{500 + x}:", "s_waitcnt vmcnt(0)", f"{600 + x}:",
                *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(4)],
                "s_cmp_eq_u32 s45, 0", f"s_cbranch_scc1 {400 + x}b",
                "s_sub_u32 s45, s45, 1",
                "s_add_u32 s38, s38, %[bstride]", "s_addc_u32 s39, s39, 0",
                *bload(BNXT),
                "s_add_u32 s48, s48, 4", "s_mov_b32 s49, 0",
                f"s_branch {400 + x}b"]

    lines = ["s_mov_b32 s46, m0",
             "s_load_dwordx4 s[40:43], %[cb], 0x0",
             "s_mov_b64 s[36:37], %[eb]", "s_mov_b64 s[38:39], %[bp]", "s_mov_b32 s47, %[ring]",
             "s_waitcnt lgkmcnt(0)",
             "s_mov_b32 s44, s42", "s_mov_b32 s42, s40", "s_mov_b32 s43, s41", "s_mov_b32 s41, s44",
             "s_and_b32 s40, s42, 0xff", "s_lshr_b64 s[42:43], s[42:43], 8",
             "s_mov_b32 s45, 6",
             "s_cmp_eq_u32 s41, 0", "s_cbranch_scc1 9f"]
    lines += dma(0) + dma(0x400)
    lines += bload(BCUR) + ["s_add_u32 s38, s38, %[bstride]", "s_addc_u32 s39, s39, 0"] + bload(BNXT)
    lines += ["s_mov_b32 s48, 8", "s_mov_b32 s49, 0", "s_waitcnt vmcnt(4)"]
    R0 = RSET[0]
    lines += [f"ds_read_b128 v[{R0}:{R0 + 3}], %[ringv] offset:0",
              f"ds_read_b128 v[{R0 + 4}:{R0 + 7}], %[ringv] offset:16", "s_waitcnt lgkmcnt(0)"]
    adds, reads = rows(0)
    for q in range(8):
        lines += [adds[q], reads[q]]
    R1, W0 = RSET[1], WSET[0]
    lines += [f"ds_read_b128 v[{R1}:{R1 + 3}], %[ringv] offset:64",
              f"ds_read_b128 v[{R1 + 4}:{R1 + 7}], %[ringv] offset:80",
              f"ds_read_b128 v[{W0}:{W0 + 3}], %[ringv] offset:32",
              f"ds_read_b128 v[{W0 + 4}:{W0 + 7}], %[ringv] offset:48"]
    lines.append("7:")
    for x in range(32):
        lines += step(x)
    lines.append("s_branch 7b")
    for x in range(32):
        lines += switch(x)
    lines += ["8:", "s_waitcnt vmcnt(0) lgkmcnt(0)", "9:", "s_mov_b32 m0, s46"]
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(24, 128))
    sclob = ", ".join(f'"s{i}"' for i in range(36, 51))
    return f'''#define {name}(acc_, lane16_, lane4_, laneoff_, ringv_, ring_, eb_, cb_, bp_, bstride_)  \\
  asm volatile(  \\
{body}
      : {", ".join(f'[acc{i}] "+v"(acc_[{i}])' for i in range(8))}  \\
      : [lane16] "v"(lane16_), [lane4] "v"(lane4_), [laneoff] "v"(laneoff_), [ringv] "v"(ringv_),  \\
        [ring] "s"(ring_), [eb] "s"(eb_), [cb] "s"(cb_), [bp] "s"(bp_), [bstride] "s"(bstride_)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
'''


# ---------------------------------------------------------------------------
# v4: 16-entry steps, rows read just in time with counted lgkmcnt
# ---------------------------------------------------------------------------
JIT_DOC = """
Rows read just in time.  A step is 16 entries (two 8-entry groups, two
s_load_dwordx16) and starts with the only s_waitcnt lgkmcnt(0): the entries of
this step (loaded one step earlier) landed, and no LDS read is in flight.
It then requests the next step's 32 entry dwords into the other SGPR set --
one whole 16-entry step of cover for the scalar loads, twice the 8-entry
loop's -- and walks its 16 entries with each row read issued L entries ahead
into a ring of L + 1 four-VGPR slots, waited with a counted lgkmcnt(M), M =
the reads issued after it.  Counted waits stay correct with the two scalar
loads outstanding: if read e were pending, reads e..e+M would be too (LDS
completes in order), so the count could not be <= M; the scalar loads only
make a wait stricter (effective lead L - 2 while they are in flight).  The
differences are formed in place (v_sub_f32 into the slot).  A column ending
in the step's first group switches B between its two groups.
Registers: v56..v59 B, v60..v63 next B, v64.. the ring; entry sets s36..s67
and s68..s99; s24 stream offset (next step), s25 temporary, s[26:27] stream
base, s22 column counter, s23 temporary, s[20:21] B row pointer.
"""


def gen_jit(name="FS_SPARSE_STREAM_ASM", lead=6, bank_shift=False, half_lds=False, wait_every=1):
    L = lead
    SET = [36, 68]
    # bank_shift (A/B only): B in v57..v60 so that v_sub_f32's two VGPR
    # operands (slot + f, B + f) sit in different VGPR banks (v mod 4).
    # Measured against the round-1 loop on one box (profiles/r02/
    # jit_bankshift_ab.txt): 103.35-103.4 vs 103.5-103.56 ms -- no better
    # than the unshifted JIT loop (102.2-102.4 vs 103.0-103.2); not shipped.
    BCUR, BNXT, RING = (57, 61, 68) if bank_shift else (56, 60, 64)
    OFF, TMP, BASE, COLS, TMP2, BPTR = 24, 25, 26, 22, 23, 20

    def slot(e):
        return RING + 4 * (e % (L + 1))

    def entry_sgprs(k, e):
        g, q = divmod(e, 8)
        base = SET[k] + 16 * g + 2 * q
        return base, base + 1     # roff, weight

    def read(k, e):
        r, _ = entry_sgprs(k, e)
        a = slot(e)
        if half_lds:  # diagnostic only (wrong scores): half the LDS bytes per entry
            return [f"v_add_u32 v{a}, s{r}, %[lane16]", f"ds_read_b64 v[{a}:{a + 1}], v{a}"]
        return [f"v_add_u32 v{a}, s{r}, %[lane16]", f"ds_read_b128 v[{a}:{a + 3}], v{a}"]

    def compute(k, e):
        _, w = entry_sgprs(k, e)
        a = slot(e)
        L_ = [f"v_sub_f32 v{a + f}, v{a + f}, v{BCUR + f}" for f in range(4)]
        for f in range(4):
            acc = f"%[acc{2 * f + (e & 1)}]"
            L_.append(f"v_fma_f32 {acc}, s{w}, |v{a + f}|, {acc}")
        return L_

    def bload(dst):
        return [f"global_load_dword v{dst + f}, %[lane4], s[{BPTR}:{BPTR + 1}]" + (f" offset:{256 * f}" if f else "")
                for f in range(4)]

    def switch(lab, ret):
        return [f"{lab}:",
                f"s_add_u32 s{COLS}, s{COLS}, 1",
                f"s_cmp_ge_u32 s{COLS}, %[ncols]",
                "s_cbranch_scc1 8f",
                "s_waitcnt vmcnt(0)",
                *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(4)],
                f"s_add_u32 s{TMP2}, s{COLS}, 1",
                f"s_cmp_ge_u32 s{TMP2}, %[ncols]",
                f"s_cbranch_scc1 {ret}b",
                f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
                f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
                *bload(BNXT),
                f"s_branch {ret}b"]

    out_of_line = []

    def step(x):
        k, o = x % 2, 1 - x % 2
        S = ["s_waitcnt lgkmcnt(0)",
             f"s_load_dwordx16 s[{SET[o]}:{SET[o] + 15}], s[{BASE}:{BASE + 1}], s{OFF}",
             f"s_add_u32 s{TMP}, s{OFF}, 64",
             f"s_load_dwordx16 s[{SET[o] + 16}:{SET[o] + 31}], s[{BASE}:{BASE + 1}], s{TMP}",
             f"s_add_u32 s{OFF}, s{OFF}, 128"]
        for e in range(min(L, 16)):
            S += read(k, e)
        issued = min(L, 16)
        for e in range(16):
            if e == 8:  # group A's column ended: next column's B before group B
                S += [f"s_bitcmp1_b32 s{SET[k] + 1}, 0", f"s_cbranch_scc1 {10 + 2 * x}f", f"{40 + 2 * x}:"]
                out_of_line.extend(switch(10 + 2 * x, 40 + 2 * x))
            if e + L < 16:
                S += read(k, e + L)
                issued = e + L + 1
            after = issued - (e + 1)          # reads issued after entry e's
            if e % wait_every == 0:           # wait_every > 1: one wait covers the next entries too
                last = min(e + wait_every - 1, 15)
                after_last = issued - (last + 1)
                S.append(f"s_waitcnt lgkmcnt({min(max(after_last, 0), 15)})")
            S += compute(k, e)
        S += [f"s_bitcmp1_b32 s{SET[k] + 17}, 0", f"s_cbranch_scc1 {11 + 2 * x}f", f"{41 + 2 * x}:"]
        out_of_line.extend(switch(11 + 2 * x, 41 + 2 * x))
        return S

    lines = [f"s_mov_b32 s{COLS}, 0",
             f"s_mov_b64 s[{BPTR}:{BPTR + 1}], %[bp]",
             *bload(BCUR),
             f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
             f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
             *bload(BNXT),
             f"s_mov_b64 s[{BASE}:{BASE + 1}], %[eb]",
             f"s_load_dwordx16 s[{SET[0]}:{SET[0] + 15}], s[{BASE}:{BASE + 1}], 0x0",
             f"s_load_dwordx16 s[{SET[0] + 16}:{SET[0] + 31}], s[{BASE}:{BASE + 1}], 0x40",
             f"s_mov_b32 s{OFF}, 128",
             "s_waitcnt vmcnt(4)",
             "7:"]
    for x in range(2):
        lines += step(x)
    # safety bound: a stream holds at most 8 columns x 16 groups (8 KB)
    lines += [f"s_cmp_gt_u32 s{OFF}, 0x2100", "s_cbranch_scc0 7b", "s_branch 8f"]
    lines += out_of_line
    lines += ["8:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(BCUR, RING + 4 * (L + 1)))
    named = set()
    for l in lines:
        for lo, hi in re.findall(r"(?<![a-z_])s\[?(\d+)(?::(\d+)\])?", l):
            named.update(range(int(lo), int(hi or lo) + 1))
    sclob = ", ".join(f'"s{i}"' for i in sorted(named))
    return f'''#define {name}(acc, lane16, lane4, eb, bp, bstride, ncols)  \\
  asm volatile(  \\
{body}
      : {", ".join(f'[acc{i}] "+v"(acc[{i}])' for i in range(8))}  \\
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [eb] "s"(eb), [bp] "s"(bp),  \\
        [bstride] "s"(bstride), [ncols] "s"(ncols)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
'''


# ---------------------------------------------------------------------------
# v2 (round 3, shipped): 64-row half tiles, F = 8 (or 4) features per lane,
# unpadded streams with per-entry column-end flags
# ---------------------------------------------------------------------------
V2_DOC = """
Sparse v2 loop (k_score_sparse2).  Stream = the entries (roff, w) of one
wave's 8 columns in one 64-row half tile, unpadded: roff = row * 2048 (the
row's byte offset in the LDS block: 64 lanes x 8 floats), w the pair weight
with its lowest mantissa bit set on the last entry of a column.  Lane l
scores features f0 + 4l + k (chunk 0, LDS offset 0) and f0 + 256 + 4l + k
(chunk 1, LDS offset 1024), k = 0..3.  Per entry: v_add_u32 (address),
ds_read_b128 x F/4 (chunk 1 first: the chunk-0 read overwrites the address
register), F x (v_sub_f32 in place, v_fma_f32 acc += w * |d|) -- 2F + 1 VALU
per F pair-features.
A step is 16 entries (two s_load_dwordx16, issued at the start of the
previous step) and starts with the only lgkmcnt(0); the rows of entry e are
read L entries ahead into a ring of L + 1 F-VGPR slots and waited with a
counted lgkmcnt(M) (correct with the scalar loads in flight: LDS completes in
order, so if e's read were pending the M reads after it would be too).  After
each entry an SCC test of the weight's flag branches out of line to the
column switch: B <- next B (prefetched one column ahead, two
global_load_dwordx4), the load of the column after it, or the exit after the
stream's 8th column.  A safety bound on the stream offset ends the loop on a
malformed stream.
Registers: v24.. B (F), then next B (F), then the ring; s20..s27 and
s36..s99 as the v1 JIT loop.
"""


def gen_v2(name, F=8, lead=4, diag="", grp=1, pfn=True, tprof=False, salu_pad=0):
    """diag (A/B diagnostics only, wrong scores): "lds1" skips the chunk-1
    row read (half the LDS traffic), "nosub" drops the v_sub_f32 (half the
    VALU), "nolds" skips every row read (the slots keep stale values).
    tprof (profiling builds, -DFS_SP2_PROF): one more output, the s_memtime
    stamp taken once the stream's first entries and B rows have landed (the
    caller stamps the macro's start and end: tile-start stall vs walk)."""
    L = lead
    R = F // 4                      # ds_read_b128 per entry
    SET = [36, 68]
    # bpre2: B prefetched two columns ahead (a third B set, two moves per switch)
    NB = 3 if diag == "bpre2" else 2
    BCUR, BNXT = 24, 24 + F
    BNX2 = 24 + 2 * F
    RING = 24 + NB * F
    PF = RING + F * (L + 1)          # two scratch VGPRs of the next-tile prefetch
    OFF, TMP, BASE, COLS, TMP2, BPTR = 24, 25, 26, 22, 23, 20

    def slot(e):
        return RING + F * (e % (L + 1))

    def entry_sgprs(k, e):
        base = SET[k] + 2 * e
        return base, base + 1       # roff, weight

    def read(k, e):
        r, _ = entry_sgprs(k, e)
        a = slot(e)
        L_ = [f"v_add_u32 v{a}, s{r}, %[lds_lane]"]
        if diag == "nolds":
            return L_
        if F == 8 and diag != "lds1":  # chunk 1 first: the chunk-0 read overwrites the address
            L_.append(f"ds_read_b128 v[{a + 4}:{a + 7}], v{a} offset:1024")
        L_.append(f"ds_read_b128 v[{a}:{a + 3}], v{a}")
        return L_

    def compute(k, e):
        _, w = entry_sgprs(k, e)
        a = slot(e)
        L_ = [] if diag == "nosub" else [f"v_sub_f32 v{a + f}, v{a + f}, v{BCUR + f}" for f in range(F)]
        L_ += [f"v_fma_f32 %[acc{f}], s{w}, |v{a + f}|, %[acc{f}]" for f in range(F)]
        # A/B diagnostics only: salu_pad extra SALU instructions per entry
        # (results unchanged) price the per-entry scalar work of the walk
        L_ += ["s_mov_b32 s29, s28"] * salu_pad
        return L_

    ntm = " nt" if diag == "bnt" else ""   # A/B: B rows as non-temporal loads

    def bload(dst):
        L_ = [f"global_load_dwordx4 v[{dst}:{dst + 3}], %[glb_lane], s[{BPTR}:{BPTR + 1}]{ntm}"]
        if F == 8:
            L_.append(f"global_load_dwordx4 v[{dst + 4}:{dst + 7}], %[glb_lane], "
                      f"s[{BPTR}:{BPTR + 1}] offset:1024{ntm}")
        return L_

    out_of_line = []

    def switch(lab, ret):
        if diag == "bpre2":
            # BNXT was requested two switches ago, BNX2 at the last one
            return [f"{lab}:",
                    f"s_add_u32 s{COLS}, s{COLS}, 1",
                    f"s_cmp_ge_u32 s{COLS}, %[ncols]",
                    "s_cbranch_scc1 8f",
                    f"s_waitcnt vmcnt({R})",
                    *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(F)],
                    "s_waitcnt vmcnt(0)",
                    *[f"v_mov_b32 v{BNXT + f}, v{BNX2 + f}" for f in range(F)],
                    f"s_add_u32 s{TMP2}, s{COLS}, 2",
                    f"s_cmp_ge_u32 s{TMP2}, %[ncols]",
                    f"s_cbranch_scc1 {ret}b",
                    f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
                    f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
                    *bload(BNX2),
                    f"s_branch {ret}b"]
        return [f"{lab}:",
                f"s_add_u32 s{COLS}, s{COLS}, 1",
                f"s_cmp_ge_u32 s{COLS}, %[ncols]",
                "s_cbranch_scc1 8f",
                "s_waitcnt vmcnt(0)",
                *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(F)],
                f"s_add_u32 s{TMP2}, s{COLS}, 1",
                f"s_cmp_ge_u32 s{TMP2}, %[ncols]",
                f"s_cbranch_scc1 {ret}b",
                *([] if diag == "bhot" else [f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
                                             f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0"]),
                *bload(BNXT),
                f"s_branch {ret}b"]

    if diag in ("lds1", "nolds"):
        R = 1 if diag == "lds1" else 0

    def step(x):
        k, o = x % 2, 1 - x % 2
        S = ["s_waitcnt lgkmcnt(0)",
             f"s_load_dwordx16 s[{SET[o]}:{SET[o] + 15}], s[{BASE}:{BASE + 1}], s{OFF}",
             f"s_add_u32 s{TMP}, s{OFF}, 64",
             f"s_load_dwordx16 s[{SET[o] + 16}:{SET[o] + 31}], s[{BASE}:{BASE + 1}], s{TMP}",
             f"s_add_u32 s{OFF}, s{OFF}, 128"]
        for e in range(min(L, 16)):
            S += read(k, e)
        issued = min(L, 16)
        for e in range(16):
            if e + L < 16:
                S += read(k, e + L)
                issued = e + L + 1
            after = (issued - (e + 1)) * R      # LDS reads issued after entry e's last one
            S.append(f"s_waitcnt lgkmcnt({min(after, 15)})")
            S += compute(k, e)
            if (e + 1) % grp == 0:  # columns are padded to whole groups of grp entries
                _, w = entry_sgprs(k, e)
                sw, ret = 100 + 16 * x + e, 200 + 16 * x + e
                S += [f"s_bitcmp1_b32 s{w}, 0", f"s_cbranch_scc1 {sw}f", f"{ret}:"]
                out_of_line.extend(switch(sw, ret))
        return S

    lines = [f"s_mov_b32 s{COLS}, 0",
             f"s_mov_b64 s[{BPTR}:{BPTR + 1}], %[bp]",
             *bload(BCUR),
             f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
             f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
             *bload(BNXT)]
    if diag == "bpre2":
        lines += [f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
                  f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
                  *bload(BNX2)]
    if pfn:
        # warm L2 with the next tile's first two B rows (this wave's columns
        # 0 and 1 there: 2 KB each, one 32-byte piece per lane): the stream
        # start of the next tile would otherwise wait for them from HBM.  The
        # loaded values are never used; the exit's vmcnt(0) retires them.
        lines += ["s_mov_b64 s[28:29], %[bpn]",
                  f"global_load_dword v{PF}, %[pf_lane], s[28:29]",
                  "s_add_u32 s28, s28, %[bstride]",
                  "s_addc_u32 s29, s29, 0",
                  f"global_load_dword v{PF + 1}, %[pf_lane], s[28:29]"]
    if diag == "spf":
        # A/B: warm the scalar cache / L2 with the next tile's stream head
        lines += ["s_load_dword s28, %[enb], 0x0", "s_load_dword s29, %[enb], 0x40"]
    lines += [f"s_mov_b64 s[{BASE}:{BASE + 1}], %[eb]",
              f"s_load_dwordx16 s[{SET[0]}:{SET[0] + 15}], s[{BASE}:{BASE + 1}], 0x0",
              f"s_load_dwordx16 s[{SET[0] + 16}:{SET[0] + 31}], s[{BASE}:{BASE + 1}], 0x40",
              f"s_mov_b32 s{OFF}, 128",
              f"s_waitcnt vmcnt({(NB - 1) * R + (2 if pfn else 0)})"]
    if tprof:
        lines += ["s_waitcnt lgkmcnt(0)", "s_memtime %[tpro]", "s_waitcnt lgkmcnt(0)"]
    lines += ["7:"]
    for x in range(2):
        lines += step(x)
    # safety bound: a stream holds at most 8 columns x 64 rows (4 KB)
    lines += [f"s_cmp_gt_u32 s{OFF}, 0x1100", "s_cbranch_scc0 7b", "s_branch 8f"]
    lines += out_of_line
    lines += ["8:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(BCUR, PF + (2 if pfn else 0)))
    named = set()
    for l in lines:
        for lo, hi in re.findall(r"(?<![a-z_])s\[?(\d+)(?::(\d+)\])?", l):
            named.update(range(int(lo), int(hi or lo) + 1))
    sclob = ", ".join(f'"s{i}"' for i in sorted(named))
    targ = ", tpro_" if tprof else ""
    tout = ', [tpro] "=s"(tpro_)' if tprof else ""
    return f"""#define {name}(acc_, lds_lane_, glb_lane_, eb_, bp_, bstride_, ncols_, bpn_, pf_lane_, enb_{targ})  \\
  asm volatile(  \\
{body}
      : {", ".join(f'[acc{i}] "+v"(acc_[{i}])' for i in range(F))}{tout}  \\
      : [lds_lane] "v"(lds_lane_), [glb_lane] "v"(glb_lane_), [eb] "s"(eb_), [bp] "s"(bp_),  \\
        [bstride] "s"(bstride_), [ncols] "s"(ncols_), [bpn] "s"(bpn_), [pf_lane] "v"(pf_lane_),  \\
        [enb] "s"(enb_)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
"""


V2X_DOC = """
Sparse v2 loop with cross-step lookahead (k_score_sparse2; FS_GEN_V2X).
The plain v2 loop drains the LDS pipeline at every step: the step's lgkmcnt(0)
(the only safe wait while scalar loads are in flight, since they return out
of order) comes before the step's first row reads can be issued, because
their addresses are in the entries that wait is for.  Here the scalar loads
run two steps ahead through three SGPR sets (steps of S = 8 or 12 entries:
3 x 2S SGPRs), so at the start of step k the entries of step k + 1 are
already in SGPRs and the rows of the first L entries of each step are read
during the previous step: the lgkmcnt(0) at a step's start then waits only
for scalar loads issued a whole step earlier and row reads issued L entries
earlier.
"""


def gen_v2x(name, F=8, lead=3, S=8):
    L = lead
    assert 1 <= L <= S
    R = F // 4
    NS = 3
    W = 2 * S                        # SGPRs per set
    SET = [28 + W * i for i in range(NS)]
    assert SET[-1] + W <= 102
    BCUR, BNXT = 24, 24 + F
    RING = 24 + 2 * F
    OFF, TMP, BASE, COLS, TMP2, BPTR = 24, 25, 26, 22, 23, 20
    NSTEP = NS                       # unrolled steps (set rotation)
    TOT = S * NSTEP                  # entries per unrolled body
    # reads run L entries ahead across the loop's back edge: ring slots must
    # line up with the next pass of the body
    assert TOT % (L + 1) == 0, "3 * S must be a multiple of lead + 1"

    def slot(e):
        return RING + F * (e % (L + 1))

    def entry_sgprs(g):              # g = entry index within the unrolled body
        st, e = divmod(g % TOT, S)
        base = SET[st % NS] + 2 * e
        return base, base + 1

    def read(g):
        r, _ = entry_sgprs(g)
        a = slot(g)
        L_ = [f"v_add_u32 v{a}, s{r}, %[lds_lane]"]
        if F == 8:
            L_.append(f"ds_read_b128 v[{a + 4}:{a + 7}], v{a} offset:1024")
        L_.append(f"ds_read_b128 v[{a}:{a + 3}], v{a}")
        return L_

    def compute(g):
        _, w = entry_sgprs(g)
        a = slot(g)
        L_ = [f"v_sub_f32 v{a + f}, v{a + f}, v{BCUR + f}" for f in range(F)]
        L_ += [f"v_fma_f32 %[acc{f}], s{w}, |v{a + f}|, %[acc{f}]" for f in range(F)]
        return L_

    def bload(dst):
        L_ = [f"global_load_dwordx4 v[{dst}:{dst + 3}], %[glb_lane], s[{BPTR}:{BPTR + 1}]"]
        if F == 8:
            L_.append(f"global_load_dwordx4 v[{dst + 4}:{dst + 7}], %[glb_lane], "
                      f"s[{BPTR}:{BPTR + 1}] offset:1024")
        return L_

    def sload(st, off_reg):          # entries of one step into set st
        b = SET[st % NS]
        if S == 8:
            return [f"s_load_dwordx16 s[{b}:{b + 15}], s[{BASE}:{BASE + 1}], s{off_reg}"]
        return [f"s_load_dwordx16 s[{b}:{b + 15}], s[{BASE}:{BASE + 1}], s{off_reg}",
                f"s_add_u32 s{TMP}, s{off_reg}, 64",
                f"s_load_dwordx8 s[{b + 16}:{b + 23}], s[{BASE}:{BASE + 1}], s{TMP}"]

    out_of_line = []

    def switch(lab, ret):
        return [f"{lab}:",
                f"s_add_u32 s{COLS}, s{COLS}, 1",
                f"s_cmp_ge_u32 s{COLS}, %[ncols]",
                "s_cbranch_scc1 8f",
                "s_waitcnt vmcnt(0)",
                *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(F)],
                f"s_add_u32 s{TMP2}, s{COLS}, 1",
                f"s_cmp_ge_u32 s{TMP2}, %[ncols]",
                f"s_cbranch_scc1 {ret}b",
                f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
                f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
                *bload(BNXT),
                f"s_branch {ret}b"]

    def step(st):
        # entries st*S .. st*S + S-1 of the body; rows of the first L of them
        # were read during the previous step (or the prologue)
        S_ = ["s_waitcnt lgkmcnt(0)"]
        S_ += sload(st + 2, OFF)
        S_.append(f"s_add_u32 s{OFF}, s{OFF}, {8 * S}")
        issued_upto = st * S + L      # entries whose rows were requested (exclusive)
        for e in range(S):
            g = st * S + e
            S_ += read(g + L)
            issued_upto = g + L + 1
            after = (issued_upto - (g + 1)) * R
            S_.append(f"s_waitcnt lgkmcnt({min(after, 15)})")
            S_ += compute(g)
            _, w = entry_sgprs(g)
            sw, ret = 100 + g, 200 + g
            S_ += [f"s_bitcmp1_b32 s{w}, 0", f"s_cbranch_scc1 {sw}f", f"{ret}:"]
            out_of_line.extend(switch(sw, ret))
        return S_

    lines = [f"s_mov_b32 s{COLS}, 0",
             f"s_mov_b64 s[{BPTR}:{BPTR + 1}], %[bp]",
             *bload(BCUR),
             f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
             f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
             *bload(BNXT),
             f"s_mov_b64 s[{BASE}:{BASE + 1}], %[eb]",
             f"s_mov_b32 s{OFF}, 0"]
    lines += sload(0, OFF)
    lines.append(f"s_add_u32 s{OFF}, s{OFF}, {8 * S}")
    lines += sload(1, OFF)
    lines.append(f"s_add_u32 s{OFF}, s{OFF}, {8 * S}")
    lines += ["s_waitcnt lgkmcnt(0)", f"s_waitcnt vmcnt({R})"]
    for g in range(L):
        lines += read(g)
    lines.append("7:")
    for st in range(NSTEP):
        lines += step(st)
    # safety bound: a stream holds at most 8 columns x 64 rows (4 KB)
    lines += [f"s_cmp_gt_u32 s{OFF}, 0x1200", "s_cbranch_scc0 7b", "s_branch 8f"]
    lines += out_of_line
    lines += ["8:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(BCUR, RING + F * (L + 1)))
    named = set()
    for l in lines:
        for lo, hi in re.findall(r"(?<![a-z_])s\[?(\d+)(?::(\d+)\])?", l):
            named.update(range(int(lo), int(hi or lo) + 1))
    sclob = ", ".join(f'"s{i}"' for i in sorted(named))
    return f"""#define {name}(acc_, lds_lane_, glb_lane_, eb_, bp_, bstride_, ncols_)  \\
  asm volatile(  \\
{body}
      : {", ".join(f'[acc{i}] "+v"(acc_[{i}])' for i in range(F))}  \\
      : [lds_lane] "v"(lds_lane_), [glb_lane] "v"(glb_lane_), [eb] "s"(eb_), [bp] "s"(bp_),  \\
        [bstride] "s"(bstride_), [ncols] "s"(ncols_)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
"""


SEG_DOC = """
Segment walk (measured in round 4, not shipped: profiles/r04/pass2_seg_ab.txt,
+0.7 ms at cfg4; the function stays for the record): the
tile loop of one unit inside the asm block.  Per tile: the stream base and
the B pointer from the lane-indexed tile list (v_readlane), the v2 stream
walk (16 entries per step, rows read 3 entries ahead), the tile's f32
partials flushed into the unit's f64 sums, the progress counter in LDS and
s_setprio as in the C++ loop.  What the C++ loop cannot do: the next tile's
columns 0 and 1 are loaded into spare VGPRs (BN0 / BN1) when the current
stream enters its last column, so a tile starts with its B rows in
registers, and no SGPR is spilled around a per-tile asm statement.
"""


def gen_v2seg(name, lead=3):
    F, L, R = 8, lead, 2
    SET = [36, 68]
    BCUR, BNXT = 24, 32
    RING = 40                       # (L + 1) slots of 8
    ACC = RING + F * (L + 1)        # 72: the tile's f32 partials
    BN0, BN1 = ACC + 8, ACC + 16    # 80, 88: next tile's columns 0 / 1
    T64 = ACC + 24                  # 96-97: f64 temporary
    VTOT = T64 + 2                  # 98
    OFF, TMP, BASE, COLS, TMP2, BPTR = 24, 25, 26, 22, 23, 20
    # s32 / s33 are the ABI's stack and frame pointers: not touched
    KT, DONE, TT, NB, TY = 28, 29, 30, 34, 25
    assert RING + F * (L + 1) == ACC

    def slot(e):
        return RING + F * (e % (L + 1))

    def entry_sgprs(k, e):
        base = SET[k] + 2 * e
        return base, base + 1

    def read(k, e):
        r, _ = entry_sgprs(k, e)
        a = slot(e)
        return [f"v_add_u32 v{a}, s{r}, %[lds_lane]",
                f"ds_read_b128 v[{a + 4}:{a + 7}], v{a} offset:1024",
                f"ds_read_b128 v[{a}:{a + 3}], v{a}"]

    def compute(k, e):
        _, w = entry_sgprs(k, e)
        a = slot(e)
        L_ = [f"v_sub_f32 v{a + f}, v{a + f}, v{BCUR + f}" for f in range(F)]
        L_ += [f"v_fma_f32 v{ACC + f}, s{w}, |v{a + f}|, v{ACC + f}" for f in range(F)]
        return L_

    def bload(dst, ptr):
        return [f"global_load_dwordx4 v[{dst}:{dst + 3}], %[glb_lane], s[{ptr}:{ptr + 1}]",
                f"global_load_dwordx4 v[{dst + 4}:{dst + 7}], %[glb_lane], s[{ptr}:{ptr + 1}] offset:1024"]

    def next_tile_ptr(idx_sgpr):
        # NB = xs_wave + y(tile idx) * tstride  (64-bit product)
        return [f"v_readlane_b32 s{TY}, %[ys], s{idx_sgpr}",
                f"s_mul_i32 s{TT}, s{TY}, %[tstride]",
                f"s_mul_hi_u32 s{TT + 1}, s{TY}, %[tstride]",
                f"s_add_u32 s{NB}, %[xsw_lo], s{TT}",
                f"s_addc_u32 s{NB + 1}, %[xsw_hi], s{TT + 1}"]

    def prefetch_next():
        # the next tile's columns 0 / 1 into BN0 / BN1 (if there is one)
        return [f"s_add_u32 s{TMP2}, s{KT}, 1",
                f"s_cmp_ge_u32 s{TMP2}, %[nt]",
                "s_cbranch_scc1 61f",
                *next_tile_ptr(TMP2),
                *bload(BN0, NB),
                f"s_add_u32 s{NB}, s{NB}, %[bstride]",
                f"s_addc_u32 s{NB + 1}, s{NB + 1}, 0",
                *bload(BN1, NB),
                "61:"]

    out_of_line = []

    def switch(lab, ret):
        pf_lab = 300 + (lab - 100)
        # column switch; entering the last column, prefetch the next tile
        out_of_line.extend([
            f"{lab}:",
            f"s_add_u32 s{COLS}, s{COLS}, 1",
            f"s_cmp_ge_u32 s{COLS}, %[ncols]",
            "s_cbranch_scc1 8f",
            "s_waitcnt vmcnt(0)",
            *[f"v_mov_b32 v{BCUR + f}, v{BNXT + f}" for f in range(F)],
            f"s_add_u32 s{TMP2}, s{COLS}, 1",
            f"s_cmp_ge_u32 s{TMP2}, %[ncols]",
            f"s_cbranch_scc1 {pf_lab}f",
            f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
            f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
            *bload(BNXT, BPTR),
            f"s_branch {ret}b",
            f"{pf_lab}:"])
        # (prefetch_next uses the local labels 61; each copy is its own block)
        blk = prefetch_next()
        blk = [l.replace("61f", f"{pf_lab + 1000}f").replace("61:", f"{pf_lab + 1000}:") for l in blk]
        out_of_line.extend(blk)
        out_of_line.append(f"s_branch {ret}b")

    def step(x):
        k, o = x % 2, 1 - x % 2
        S = ["s_waitcnt lgkmcnt(0)",
             f"s_load_dwordx16 s[{SET[o]}:{SET[o] + 15}], s[{BASE}:{BASE + 1}], s{OFF}",
             f"s_add_u32 s{TMP}, s{OFF}, 64",
             f"s_load_dwordx16 s[{SET[o] + 16}:{SET[o] + 31}], s[{BASE}:{BASE + 1}], s{TMP}",
             f"s_add_u32 s{OFF}, s{OFF}, 128"]
        for e in range(min(L, 16)):
            S += read(k, e)
        issued = min(L, 16)
        for e in range(16):
            if e + L < 16:
                S += read(k, e + L)
                issued = e + L + 1
            after = (issued - (e + 1)) * R
            S.append(f"s_waitcnt lgkmcnt({min(after, 15)})")
            S += compute(k, e)
            _, w = entry_sgprs(k, e)
            sw, ret = 100 + 16 * x + e, 200 + 16 * x + e
            S += [f"s_bitcmp1_b32 s{w}, 0", f"s_cbranch_scc1 {sw}f", f"{ret}:"]
            switch(sw, ret)
        return S

    lines = [f"s_mov_b32 s{KT}, 0",
             f"s_mov_b32 s{DONE}, %[done0]",
             # tile 0's columns 0 / 1 into the prefetch registers
             *next_tile_ptr(KT),
             *bload(BN0, NB),
             f"s_add_u32 s{NB}, s{NB}, %[bstride]",
             f"s_addc_u32 s{NB + 1}, s{NB + 1}, 0",
             *bload(BN1, NB),
             "50:",
             # this tile: stream base and B pointer (column 1)
             f"v_readlane_b32 s{TY}, %[tiles], s{KT}",
             f"s_lshl_b32 s{TT}, s{TY}, 17",
             f"s_lshr_b32 s{TT + 1}, s{TY}, 15",
             f"s_add_u32 s{BASE}, %[entw_lo], s{TT}",
             f"s_addc_u32 s{BASE + 1}, %[entw_hi], s{TT + 1}",
             f"v_readlane_b32 s{TY}, %[ys], s{KT}",
             f"s_mul_i32 s{TT}, s{TY}, %[tstride]",
             f"s_mul_hi_u32 s{TT + 1}, s{TY}, %[tstride]",
             f"s_add_u32 s{BPTR}, %[xsw_lo], s{TT}",
             f"s_addc_u32 s{BPTR + 1}, %[xsw_hi], s{TT + 1}",
             f"s_add_u32 s{BPTR}, s{BPTR}, %[bstride]",
             f"s_addc_u32 s{BPTR + 1}, s{BPTR + 1}, 0",
             f"s_mov_b32 s{COLS}, 0",
             *[f"v_mov_b32 v{ACC + f}, 0" for f in range(F)],
             f"s_load_dwordx16 s[{SET[0]}:{SET[0] + 15}], s[{BASE}:{BASE + 1}], 0x0",
             f"s_load_dwordx16 s[{SET[0] + 16}:{SET[0] + 31}], s[{BASE}:{BASE + 1}], 0x40",
             f"s_mov_b32 s{OFF}, 128",
             "s_waitcnt vmcnt(0)",
             *[f"v_mov_b32 v{BCUR + f}, v{BN0 + f}" for f in range(F)],
             *[f"v_mov_b32 v{BNXT + f}, v{BN1 + f}" for f in range(F)],
             "7:"]
    for x in range(2):
        lines += step(x)
    lines += [f"s_cmp_gt_u32 s{OFF}, 0x1100", "s_cbranch_scc0 7b", "s_branch 8f"]
    lines += out_of_line
    # Every column of a stream ends with a flagged entry (an empty one holds
    # a single flagged zero entry), so with ncols >= 2 the switch into the
    # last column -- and with it the next tile's prefetch -- always runs.
    lines += ["8:",
              "s_waitcnt lgkmcnt(0)",
              # the tile's partials into the unit's float64 sums
              *sum(([f"v_cvt_f64_f32 v[{T64}:{T64 + 1}], v{ACC + f}",
                     f"v_add_f64 %[s{f}], %[s{f}], v[{T64}:{T64 + 1}]"] for f in range(F)), []),
              # progress: lane 0 adds 1 to the LDS counter (the other lanes 0,
              # so EXEC stays whole); behind the mean -> priority 2
              f"ds_add_rtn_u32 v{VTOT}, %[wgd], %[one0]",
              "s_waitcnt lgkmcnt(0)",
              f"v_readfirstlane_b32 s{TY}, v{VTOT}",
              f"s_add_u32 s{TY}, s{TY}, 1",
              f"s_add_u32 s{DONE}, s{DONE}, 1",
              f"s_lshl_b32 s{TMP2}, s{DONE}, 4",
              f"s_cmp_lt_u32 s{TMP2}, s{TY}",
              "s_cbranch_scc1 64f",
              "s_setprio 0",
              "s_branch 65f",
              "64:",
              "s_setprio 2",
              "65:",
              f"s_add_u32 s{KT}, s{KT}, 1",
              f"s_cmp_lt_u32 s{KT}, %[nt]",
              "s_cbranch_scc1 50b",
              "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(BCUR, VTOT + 1))
    named = set()
    for l in lines:
        for lo, hi in re.findall(r"(?<![a-z_])s\[?(\d+)(?::(\d+)\])?", l):
            named.update(range(int(lo), int(hi or lo) + 1))
    sclob = ", ".join(f'"s{i}"' for i in sorted(named))
    outs = ", ".join(f'[s{i}] "+v"(s_[{i}])' for i in range(F))
    return f"""#define {name}(s_, lds_lane_, glb_lane_, tiles_, ys_, nt_, entw_lo_, entw_hi_, xsw_lo_, xsw_hi_, tstride_, bstride_, ncols_, wgd_, done0_, one0_)  \\
  asm volatile(  \\
{body}
      : {outs}  \\
      : [lds_lane] "v"(lds_lane_), [glb_lane] "v"(glb_lane_), [tiles] "v"(tiles_), [ys] "v"(ys_),  \\
        [nt] "s"(nt_), [entw_lo] "s"(entw_lo_), [entw_hi] "s"(entw_hi_), [xsw_lo] "s"(xsw_lo_),  \\
        [xsw_hi] "s"(xsw_hi_), [tstride] "s"(tstride_), [bstride] "s"(bstride_), [ncols] "s"(ncols_),  \\
        [wgd] "v"(wgd_), [done0] "s"(done0_), [one0] "v"(one0_)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
"""


if __name__ == "__main__":
    # The product uses the v2 loops only (k_score_sparse2; round 4 retired the
    # round-1/2 v1 loop and its A/B variants -- the functions above stay for
    # the microbenchmarks under tools/ubench and their logs in profiles/).
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fastselect_amd", "csrc",
                        "fs_sparse_asm.inc")
    text = HEADER
    text += "\n" + gen_v2("FS_SPARSE2_ASM_F8", F=8, lead=3, pfn=False)
    text += "\n" + gen_v2("FS_SPARSE2_ASM_F4", F=4, lead=6, pfn=False)
    open(path, "w").write(text)
    print("wrote", os.path.normpath(path))
    # (round 4's clock-stamp variant of the F = 8 loop, gen_v2(tprof=True),
    # fed a profiling build that is no longer part of the library sources:
    # its measurements are in profiles/r04/pass2_prio.txt)
