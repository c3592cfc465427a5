"""LDS bank-conflict model of the attention kernels' [64][64] bf16 tile images (128-B rows):
counts extra LDS cycles of the ds_read_b128 row fragments (frag_row) and the
ds_read_b64_tr_b16 transposed fragments (frag_tr) for an XOR swizzle of the 16-B chunk index,
using the lane groups of MI355X_MICROARCH.md's LDS table, and searches all linear XORs of the
row bits for one conflict-free on both.  python tools/attn_swizzle_check.py"""
import itertools
# ds_read_b128 lane groups
G128 = [[0,1,2,3,12,13,14,15]+list(range(20,28)), list(range(4,12))+[16,17,18,19,28,29,30,31]]
G128 += [[g+32 for g in grp] for grp in G128]
GTR = [list(range(32)), list(range(32,64))]

def conflicts_row(f):
    tot = 0
    for row0 in range(0, 64, 16):
        for s in range(2):
            for grp in G128:
                slots = {}
                for l in grp:
                    row = row0 + (l & 15); ch = 4*s + (l >> 4)
                    a = row*128 + ((ch ^ f[row]) << 4)
                    slot = (a % 256) // 16
                    slots[slot] = slots.get(slot, 0) + 1
                tot += max(slots.values()) - 1
    return tot

def conflicts_tr(f):
    tot = 0
    for t in range(4):
        for s in range(2):
            for hi in (0, 16):
                for grp in GTR:
                    slots = {}
                    for l in grp:
                        G, i = l >> 4, l & 15
                        q, p = i >> 2, i & 3
                        ch = 2*t + (p >> 1)
                        ra = 32*s + 4*G + q + hi
                        a = ra*128 + ((ch ^ f[ra]) << 4) + (p & 1)*8
                        b = (a % 256) // 8   # 8-B bank pair
                        slots[b] = slots.get(b, 0) + 1
                    tot += max(slots.values()) - 1
    return tot

def f_from(M):
    f = []
    for row in range(64):
        v = 0
        for o in range(3):
            bit = 0
            for ib in range(6):
                if (M[o] >> ib) & 1:
                    bit ^= (row >> ib) & 1
            v |= bit << o
        f.append(v)
    return f

cur_row = [((r >> 1) & 7) for r in range(64)]
cur_tr = [(((r >> 1) & 3) << 1) for r in range(64)]
print("swz_row: row", conflicts_row(cur_row), "tr", conflicts_tr(cur_row))
print("swz_tr:  row", conflicts_row(cur_tr), "tr", conflicts_tr(cur_tr))
best = None
for M in itertools.product(range(64), repeat=3):
    f = f_from(M)
    c = conflicts_row(f) + conflicts_tr(f)
    if best is None or c < best[0]:
        best = (c, M, conflicts_row(f), conflicts_tr(f))
        if c == 0:
            break
print("best", best)
