"""LDS bank-conflict model of the audio conv1 fused backward (conv_c1p.hip,
c1p8_bwd_wgrad_kernel): the B-fragment ds_read_b128 of the parity/shift input copies.

gfx950 LDS: 64 banks x 4 B; a ds_read_b128 is served in 4 passes of 16 lanes with the lane
groups below; a pass costs as many cycles as the largest number of distinct 16-byte addresses
that share one bank window (equal addresses broadcast).  Searches the row / copy strides and
prints the best (cycles per MFMA step for both tap tiles, bytes of LDS).

    python tools/lds_bank_sim.py
"""
G1 = [0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27]
G2 = [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]
GROUPS = [G1, G2, [x + 32 for x in G1], [x + 32 for x in G2]]


def tap(tt, col):
    t = 16 * tt + col
    if t >= 30:
        t = 0
    ky, k2 = t // 6, t % 6 - 2
    return k2 & 1, (k2 >> 1 if k2 >= 0 else -1) + 1, ky


def cycles(RS, CA, CB, tt, TH=16, W=112):
    segs = W // 16
    tot = n = 0
    for ks in range(TH * segs // 4):
        addrs = []
        for lane in range(64):
            gq, col = lane >> 4, lane & 15
            kb = 4 * ks + gq
            r, P0 = kb // segs, 8 * (kb % segs)
            bb, ba, ky = tap(tt, col)
            addrs.append(bb * CB + ba * CA + (r + ky) * RS + P0 * 2)
        for g in GROUPS:
            win = {}
            for l in g:
                win.setdefault((addrs[l] // 16) % 16, set()).add(addrs[l])
            tot += max(len(v) for v in win.values())
        n += 1
    return tot / n


def main():
    print("dense copies (RS 128, CA 2560, CB 7680):",
          cycles(128, 2560, 7680, 0) + cycles(128, 2560, 7680, 1))
    res = []
    for rsp in range(9):
        RS = 128 + 16 * rsp
        for cap in range(16):
            CA = 20 * RS + 16 * cap
            for cbp in range(16):
                CB = 3 * CA + 16 * cbp
                res.append((cycles(RS, CA, CB, 0) + cycles(RS, CA, CB, 1), 2 * CB, RS, CA, CB))
    res.sort()
    for r in res[:8]:
        print("cycles %.1f  lds %d B  RS %d CA %d CB %d" % r)


if __name__ == "__main__":
    main()
