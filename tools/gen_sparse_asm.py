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

Pipeline per group g (unrolled x6: 3 SGPR sets x 2 A sets):
  s_waitcnt lgkmcnt(0)            A values of g (LDS) and entries of g+1 (SMEM) landed
  8 x (v_add_u32, ds_read_b128)   rows of g+1 (the address lives in the destination)
  s_load_dwordx16                 entries of g+2 (stream offset += 64)
  8 x 4 x (v_sub_f32, v_fma_f32)  group g: acc += w * |a - b|
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

SETS = [40, 56, 72]
ASETS = [64, 96]


def gen(name="FS_SPARSE_STREAM_ASM", no_ds=False, same_stream=False):
    """Macro text.  no_ds / same_stream: microbenchmark variants that skip the
    LDS reads / keep re-reading the stream's first group (scalar-cache hits)."""

    def issue_rows(k, a):
        s, A = SETS[k], ASETS[a]
        L = [f"v_add_u32 v{A + 4 * q}, s{s + 2 * q}, %[lane16]" for q in range(8)]
        if not no_ds:
            L += [f"ds_read_b128 v[{A + 4 * q}:{A + 4 * q + 3}], v{A + 4 * q}" for q in range(8)]
        return L

    def compute(k, a):
        s, A = SETS[k], ASETS[a]
        L = []
        for q in range(8):
            t = 48 if q % 2 == 0 else 52
            w = f"s{s + 2 * q + 1}"
            for f in range(4):
                L.append(f"v_sub_f32 v{t + f}, v{A + 4 * q + f}, v{56 + f}")
            for f in range(4):
                acc = f"%[acc{2 * f + (q & 1)}]"
                L.append(f"v_fma_f32 {acc}, {w}, |v{t + f}|, {acc}")
        return L

    def step(x):
        c, n, nn = x % 3, (x + 1) % 3, (x + 2) % 3
        ac, an = x % 2, (x + 1) % 2
        L = ["s_waitcnt lgkmcnt(0)"]
        L += issue_rows(n, an)
        L.append("s_add_u32 s34, s34, 64")
        if same_stream:  # two groups re-read (scalar-cache hits); s89 bounds the loop
            L += ["s_and_b32 s34, s34, 0x40", "s_add_u32 s89, s89, 1"]
        L.append(f"s_load_dwordx16 s[{SETS[nn]}:{SETS[nn] + 15}], s[36:37], s34")
        L += compute(c, ac)
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
                "v_mov_b32 v56, v60", "v_mov_b32 v57, v61", "v_mov_b32 v58, v62", "v_mov_b32 v59, v63",
                "s_add_u32 s35, s88, 1",
                "s_cmp_ge_u32 s35, %[ncols]",
                f"s_cbranch_scc1 {20 + x}b",
                "s_add_u32 s90, s90, %[bstride]",
                "s_addc_u32 s91, s91, 0",
                "global_load_dword v60, %[lane4], s[90:91]",
                "global_load_dword v61, %[lane4], s[90:91] offset:256",
                "global_load_dword v62, %[lane4], s[90:91] offset:512",
                "global_load_dword v63, %[lane4], s[90:91] offset:768",
                f"s_branch {20 + x}b"]

    lines = [
        "s_mov_b32 s88, 0",
        "s_mov_b64 s[90:91], %[bp]",
        "global_load_dword v56, %[lane4], s[90:91]",
        "global_load_dword v57, %[lane4], s[90:91] offset:256",
        "global_load_dword v58, %[lane4], s[90:91] offset:512",
        "global_load_dword v59, %[lane4], s[90:91] offset:768",
        "s_add_u32 s90, s90, %[bstride]",
        "s_addc_u32 s91, s91, 0",
        "global_load_dword v60, %[lane4], s[90:91]",
        "global_load_dword v61, %[lane4], s[90:91] offset:256",
        "global_load_dword v62, %[lane4], s[90:91] offset:512",
        "global_load_dword v63, %[lane4], s[90:91] offset:768",
        "s_mov_b64 s[36:37], %[eb]",
        "s_mov_b32 s34, 0",
        "s_load_dwordx16 s[40:55], s[36:37], s34",
        "s_waitcnt lgkmcnt(0)",
    ]
    lines += issue_rows(0, 0)
    lines.append("s_add_u32 s34, s34, 64")
    lines.append("s_load_dwordx16 s[56:71], s[36:37], s34")
    lines.append("s_waitcnt vmcnt(4)")
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

    body = "\n".join(f'      "{l}\\n"  \\' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(48, 128))
    sclob = ", ".join(f'"s{i}"' for i in range(34, 92))
    return f'''#define {name}(acc, lane16, lane4, eb, bp, bstride, ncols)  \\
  asm volatile(  \\
{body}
      : [acc0] "+v"(acc[0]), [acc1] "+v"(acc[1]), [acc2] "+v"(acc[2]), [acc3] "+v"(acc[3]),  \\
        [acc4] "+v"(acc[4]), [acc5] "+v"(acc[5]), [acc6] "+v"(acc[6]), [acc7] "+v"(acc[7])   \\
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [eb] "s"(eb), [bp] "s"(bp),  \\
        [bstride] "s"(bstride), [ncols] "s"(ncols)  \\
      : {vclob},  \\
        {sclob}, "scc", "memory")
'''


HEADER = """// Generated by tools/gen_sparse_asm.py -- do not edit by hand.
// Inner loop of k_score_sparse for continuous feature blocks (see the
// generator's docstring for the layout, the pipeline and the fixed registers).
"""

if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fastselect_amd", "csrc",
                        "fs_sparse_asm.inc")
    open(path, "w").write(HEADER + gen())
    print("wrote", os.path.normpath(path))
