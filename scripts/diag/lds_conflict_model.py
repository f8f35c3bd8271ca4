"""Bank-conflict model of the pair-split kernel's LDS accesses at A16/O32/LPR4
(split_kernel<16,32,4>, kernel_split.h), from the lane groups and bank rules
of MI355X_MICROARCH.md §LDS: extra LDS cycles per wave, per access pattern.
Host-only; compare the total with SQ_LDS_BANK_CONFLICT / waves
(profiles/r03_split_lds_conflicts.txt).

    python scripts/diag/lds_conflict_model.py
"""

# ds_read_b128: four 16-lane groups; bank = (dword address) mod 64
G128 = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
G128 += [[x + 32 for x in g] for g in G128]


def extra_b128(addrs):
    extra = 0
    for g in G128:
        banks = {}
        for ln in g:
            a = addrs[ln]
            if a is None:
                continue
            for k in range(4):
                banks.setdefault((a + k) % 64, set()).add(a + k)
        extra += max([len(v) for v in banks.values()] or [1]) - 1
    return extra


def extra_b32(addrs):
    """ds_read_b32 / ds_write_b32: two 32-lane halves, bank = dword mod 32"""
    extra = 0
    for half in (range(32), range(32, 64)):
        banks = {}
        for ln in half:
            a = addrs[ln]
            if a is not None:
                banks.setdefault(a % 32, set()).add(a)
        extra += max([len(v) for v in banks.values()] or [1]) - 1
    return extra


A, O, LPR = 16, 32, 4
R, D = 16, 2 + 2 * O + 2 * (A - 1)   # rows per wave, packed row length (96)


def row_writes(col):
    """the pair phase's packed-row writes; col(r, j) = dword of column j of row r"""
    t = 0
    for i in range(O // LPR):   # obstacle bearings and distances
        t += extra_b32([col(ln // LPR, 2 + ln % LPR + LPR * i) for ln in range(64)])
        t += extra_b32([col(ln // LPR, 2 + O + ln % LPR + LPR * i) for ln in range(64)])
    for i in range((A - 1 + LPR - 1) // LPR):   # other agents (the spare slot: target)
        on = [(ln % LPR) + LPR * i < A - 1 for ln in range(64)]
        t += extra_b32([col(ln // LPR, 2 + 2 * O + ln % LPR + LPR * i) if on[ln] else None
                        for ln in range(64)])
        t += extra_b32([col(ln // LPR, 2 + 2 * O + A - 1 + ln % LPR + LPR * i) if on[ln] else None
                        for ln in range(64)])
    return t


def store_reads(col):
    """the store phase: lane i of the tile reads 16-byte piece i (linear)"""
    n4, t = R * D // 4, 0
    for k in range(0, n4, 64):
        ad = []
        for ln in range(64):
            i = ln + k
            ad.append(None if i >= n4 else col(i // (D // 4), 4 * (i % (D // 4))))
        t += extra_b128(ad)
    return t


def bond_writes(bs):
    t = 0
    for i in range((A - 1 + LPR - 1) // LPR):
        t += extra_b32([bs * (ln // LPR) + (ln % LPR) + LPR * i
                        if (ln % LPR) + LPR * i < A - 1 else None for ln in range(64)])
    return t


def main():
    print("packed rows (per wave): row writes / store-phase reads, extra LDS cycles")
    for dp in (96, 100, 104, 108):
        c = lambda r, j, dp=dp: r * dp + j
        print(f"  row stride {dp:3d}: writes {row_writes(c):4d}  store reads {store_reads(c):3d}")
    xor = lambda r, j: r * D + 4 * ((j >> 2) ^ (r & 7)) + (j & 3)
    print(f"  stride 96, 16-byte pieces XOR-swizzled by row & 7: writes {row_writes(xor)} "
          f" store reads {store_reads(xor)}  (costs ~40 VALU per wave of address math)")
    print("bond-term writes (row stride 15, as built):", bond_writes(A - 1),
          "; stride 20:", bond_writes(20))


if __name__ == "__main__":
    main()
