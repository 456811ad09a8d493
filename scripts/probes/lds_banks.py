"""LDS bank-conflict check of the dense engine's swizzles (robustgrape_amd/csrc/grape_dense.hpp sidx, sidx16).

Model (/opt/skills/guides/MI355X_MICROARCH.md, LDS table): an 8-byte access per lane occupies two dword banks;
  ds_read_b64                    two 32-lane groups, bank = dword % 64
  ds_read2st64_b64 / ds_write_b64   four 16-lane groups, bank = dword % 32
Each extra distinct dword on a bank within a group costs one LDS cycle.  Prints the worst extra cycles of one
access over every (k-step, tile, column block) for each fragment / tile pattern, for the round-2 swizzles and
the round-6 ones.  python scripts/probes/lds_banks.py
"""
N = 64


def conflicts(addrs, groups, nbanks):
    extra = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for dw in (a // 4, a // 4 + 1):
                banks.setdefault(dw % nbanks, set()).add(dw)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


G32 = [list(range(0, 32)), list(range(32, 64))]
G16 = [list(range(i, i + 16)) for i in range(0, 64, 16)]


def worst(f):
    w64 = w16 = 0
    for s in range(16):
        for t in range(4):
            for w in range(4):
                addrs = [8 * f(lane, s, t, w) for lane in range(64)]
                w64 = max(w64, conflicts(addrs, G32, 64))
                w16 = max(w16, conflicts(addrs, G16, 32))
    return w64, w16


def swz_r2(row):
    return ((row & 15) << 1) ^ ((row & 1) << 4)


def swz_r6(row):
    return (row & 15) | ((row & 1) << 4)


def patterns64(sidx):
    return {
        "A fragment of L": lambda l, s, t, w: sidx(16 * t + (l & 15), 4 * s + (l >> 4)),
        "A fragment of L^T": lambda l, s, t, w: sidx(4 * s + (l >> 4), 16 * t + (l & 15)),
        "B fragment of R": lambda l, s, t, w: sidx(4 * s + (l >> 4), 16 * w + (l & 15)),
        "B fragment of R^T": lambda l, s, t, w: sidx(16 * w + (l & 15), 4 * s + (l >> 4)),
        "C tile store / load": lambda l, s, t, w: sidx(16 * t + (l >> 4) + 4 * (s % 4), 16 * w + (l & 15)),
    }


def patterns16(s16):
    return {
        "16 x 16 C store": lambda l, s, t, w: s16((l >> 4) + 4 * (s % 4), l & 15),
        "64 x 16 C store": lambda l, s, t, w: s16(16 * t + (l >> 4) + 4 * (s % 4), l & 15),
        "16 x 16 A fragment": lambda l, s, t, w: s16(l & 15, 4 * (s % 4) + (l >> 4)),
        "64 x 16 A fragment": lambda l, s, t, w: s16(16 * t + (l & 15), 4 * (s % 4) + (l >> 4)),
    }


if __name__ == "__main__":
    for tag, swz, m16 in (("round 2", swz_r2, 14), ("round 6", swz_r6, 15)):
        def sidx(row, col, swz=swz):
            return row * N + (col ^ swz(row))

        def s16(row, col, m16=m16):
            return row * 16 + (col ^ (row & m16))

        assert all(len({sidx(r, c) for c in range(N)}) == N for r in range(N))
        print(f"-- {tag}: extra LDS cycles per access (ds_read_b64 model / 16-lane ds_read2st64_b64 model)")
        for name, f in list(patterns64(sidx).items()) + list(patterns16(s16).items()):
            a, b = worst(f)
            print(f"   {name:22s} {a} / {b}")
