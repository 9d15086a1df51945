"""Exhaustive LDS bank-conflict check of the swizzles used by the HIP kernels, against the MI355X
lane groups of /opt/skills/guides/MI355X_MICROARCH.md §LDS (ds_read_b128: four non-contiguous 16-lane groups;
ds_read_b64 / ds_read_b64_tr_b16: two 32-lane halves; 64 x 4-byte banks = one 256-byte bank row).

    python tools/lds_swizzle_check.py
"""
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]
S = [0, 2, 3, 1]


def attn_swz(row, ch):  # csrc/attention.hip
    return ch ^ (((row & 3) << 2) | S[(row >> 2) & 3])


def attn_ok():
    # 16-B row reads: lane (g, r) reads row R + r, chunk 4 s + g   (frag_row / Offs::row)
    for R in (0, 16, 48):
        for s in range(4):
            for grp in B128_GROUPS:
                slots = {attn_swz(R + (l & 15), 4 * s + (l >> 4)) for l in grp}
                assert len(slots) == 16, ("attn row", R, s)
    # transposed reads: lane (g, i): q = i >> 2, p = i & 3, row 4 g + q (+16), chunk 2 dt + (p >> 1), 8-B half p & 1
    for R in (0, 32):
        for dt in range(8):
            for half in (range(0, 32), range(32, 64)):
                slots = set()
                for l in half:
                    g, i = l >> 4, l & 15
                    q, p = i >> 2, i & 3
                    row = R + 4 * g + q
                    slots.add(2 * attn_swz(row, 2 * dt + (p >> 1)) + (p & 1))
                assert len(slots) == 32, ("attn tr", R, dt)


def tn_ok():
    # csrc/gemm_tn.hip BK32: 64-B rows, chunk ^ S((row >> 2) & 3); BK64: 128-B rows, chunk ^ ((row >> 1) & 7)
    for R in (0, 16, 32):
        for grp in B128_GROUPS:
            slots = {((R + (l & 15)) * 64 % 256) // 16 + ((l >> 4) ^ S[((R + (l & 15)) >> 2) & 3]) for l in grp}
            assert len(slots) == 16, ("tn32", R)
            for ks in range(2):
                slots = {((R + (l & 15)) * 128 % 256) // 16 + ((4 * ks + (l >> 4)) ^ (((R + (l & 15)) >> 1) & 7))
                         for l in grp}
                assert len(slots) == 16, ("tn64", R, ks)


if __name__ == "__main__":
    attn_ok()
    tn_ok()
    print("all LDS swizzles conflict-free on the MI355X lane groups")
