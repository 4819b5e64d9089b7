"""LDS bank-conflict model of the conv transforms (sconv.hip), not a test: every LDS instruction of
k_sconv_rfft2<N, BT> / k_sconv_irfft2<N> with its lane -> address map, serviced by the gfx950 lane
groups and bank rules of MI355X_MICROARCH.md section LDS (b32: 2 x 32 lanes, mod 32; b64 read:
2 x 32 lanes, mod 64; b64 write: 4 x 16 contiguous lanes, mod 32).  Prints LDS-array cycles per
workgroup (ideal vs modelled) for the layout's strides, and searches padded strides.

python tools/probes/sconv_lds_banks.py            # current strides vs the best found
"""
import itertools
from collections import defaultdict

GROUPS = {
    "r32": ([list(range(0, 32)), list(range(32, 64))], 32, 1),
    "r64": ([list(range(0, 32)), list(range(32, 64))], 64, 2),
    "w32": ([list(range(0, 32)), list(range(32, 64))], 32, 1),
    "w64": ([list(range(16 * i, 16 * i + 16)) for i in range(4)], 32, 2),
}


def cycles(kind, addrs):
    """addrs: 64 dword addresses (None = inactive lane); LDS cycles of one wave instruction."""
    groups, mod, width = GROUPS[kind]
    tot = 0
    for g in groups:
        banks = defaultdict(set)
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            for k in range(width):
                banks[(a + k) % mod].add(a + k)
        tot += max((len(s) for s in banks.values()), default=0) or 0
    return tot


def wave_instrs(nthreads, total, lane_fn):
    """the lanes of each wave / trip of `for (i = tid; i < total; i += nthreads)`"""
    for base in range(0, total, nthreads):
        for w0 in range(base, min(base + nthreads, total), 64):
            yield [lane_fn(w0 + l) if w0 + l < min(base + nthreads, total) else None for l in range(64)]


def rfft_cost(N, BT, RS, IS, ZH, ZS):
    NT = 512 if N == 32 else 1024
    H = N // 2 + 1
    c = i = 0
    # P1: img fill (b32 write)
    for ad in wave_instrs(NT, BT * N * N, lambda x: (x % BT) * IS + (x // BT // N) * RS + (x // BT) % N):
        c += cycles("w32", ad); i += 2
    # P2 / P3: rows: read img[w] (b32), write Z[kb] (b64)
    for w in range(N):
        for ad in wave_instrs(NT, BT * N, lambda x, w=w: (x % BT) * IS + (x // BT) * RS + w):
            c += cycles("r32", ad); i += 2
    for kb in range(H):
        for ad in wave_instrs(NT, BT * N, lambda x, kb=kb: 2 * ((x % BT) * ZS + (x // BT) * ZH + kb)):
            c += cycles("w64", ad); i += 4
    # P4: columns: read Z[h] (b64)
    for h in range(N):
        for ad in wave_instrs(NT, BT * H, lambda x, h=h: 2 * ((x % BT) * ZS + h * ZH + x // BT)):
            c += cycles("r64", ad); i += 2
    return c, i


def irfft_cost(N, RS, IS, YH, ZH, ZS, BT=8):
    NT = 512 if N == 32 else 1024
    H = N // 2 + 1
    c = i = 0
    # Q1: Ys fill (b64 write), f = ka H + kb
    for ad in wave_instrs(NT, BT * N * H, lambda x: 2 * ((x % BT) * ZS + (x // BT // H) * YH + (x // BT) % H)):
        c += cycles("w64", ad); i += 4
    # Q2 / Q3: columns: read Ys[ka] (b64), write Zs[h] (b64)
    for ka in range(N):
        for ad in wave_instrs(NT, BT * H, lambda x, ka=ka: 2 * ((x % BT) * ZS + ka * YH + x // BT)):
            c += cycles("r64", ad); i += 2
    for h in range(N):
        for ad in wave_instrs(NT, BT * H, lambda x, h=h: 2 * ((x % BT) * ZS + h * ZH + x // BT)):
            c += cycles("w64", ad); i += 4
    # Q4 / Q5: rows: read Zs[kb] (b64, kb = 0 .. N/2), write out[w] (b32)
    for kb in range(N // 2 + 1):
        for ad in wave_instrs(NT, BT * N, lambda x, kb=kb: 2 * ((x % BT) * ZS + (x // BT) * ZH + kb)):
            c += cycles("r64", ad); i += 2
    for w in range(N):
        for ad in wave_instrs(NT, BT * N, lambda x, w=w: (x % BT) * IS + (x // BT) * RS + w):
            c += cycles("w32", ad); i += 2
    # Q6: epilogue reads (b32), twice (two channels) for GroupSort: counted once
    for ad in wave_instrs(NT, BT * N * N, lambda x: (x % BT) * IS + (x // BT // N) * RS + (x // BT) % N):
        c += cycles("r32", ad); i += 2
    return c, i


def split_costs(N, BT, RS, IS, YH, ZH, ZS, inverse):
    return irfft_cost(N, RS, IS, YH, ZH, ZS) if inverse else rfft_cost(N, BT, RS, IS, ZH, ZS)


def main():
    for N in (8, 16, 32):
        H = N // 2 + 1
        RS, IS, ZS = N + 1, N * (N + 1) + 1, N * H + 1
        cases = [(BT, False) for BT in ((16, 4) if N != 8 else (16,))] + [(8, True)]
        for BT, inv in cases:
            name = f"irfft2<{N}>" if inv else f"rfft2<{N},{BT}>"
            cur = split_costs(N, BT, RS, IS, H, H, ZS, inv)
            # the real-image strides (RS, IS) and the complex ones (YH, ZH, ZS) touch disjoint
            # instructions: search them apart, each with the other at the current value
            bi = min(((split_costs(N, BT, rs, isx, H, H, ZS, inv)[0], BT * isx, rs, isx)
                      for rs in range(N, N + 5) for isx in range(N * rs, N * rs + 33)))
            yhs = range(H, H + 5) if inv else [H]
            bz = min(((split_costs(N, BT, RS, IS, yh, zh, zs, inv)[0], BT * zs, yh, zh, zs)
                      for yh in yhs for zh in range(H, H + 5) for zs in range(N * max(yh, zh), N * max(yh, zh) + 17)))
            both = split_costs(N, BT, bi[2], bi[3], bz[2], bz[3], bz[4], inv)
            print(f"{name}: current {cur[0]} LDS cycles (conflict-free {cur[1]}); best RS={bi[2]} IS={bi[3]} "
                  f"YH={bz[2]} ZH={bz[3]} ZS={bz[4]}: {both[0]}", flush=True)


if __name__ == "__main__":
    main()


def irfft_inplace_cost(N, ZS, NCH=2, BT=8, NT=512):
    """k_sconv_irfft2 since r05: both channels in place in one complex buffer (channel stride BT ZS)."""
    H = N // 2 + 1
    CS = BT * ZS
    c = i = 0
    NL = NCH * BT * N * H

    def ys(x):      # load: ch, bt, f
        ch, r = divmod(x, BT * N * H)
        return 2 * (ch * CS + (r % BT) * ZS + r // BT)
    for ad in wave_instrs(NT, NL, ys):
        c += cycles("w64", ad); i += 4

    def col(x, k):
        ch, r = divmod(x, BT * H)
        return 2 * (ch * CS + (r % BT) * ZS + k * H + r // BT)
    for k in range(N):
        for kind in ("r64", "w64"):
            for ad in wave_instrs(NT, NCH * BT * H, lambda x, k=k: col(x, k)):
                c += cycles(kind, ad); i += 2 if kind == "r64" else 4

    def row(x):
        ch, r = divmod(x, BT * N)
        return 2 * (ch * CS + (r % BT) * ZS + (r // BT) * H)
    for kb in range(N // 2 + 1):
        for ad in wave_instrs(NT, NCH * BT * N, lambda x, kb=kb: row(x) + 2 * kb):
            c += cycles("r64", ad); i += 2
    for w in range(N):
        for ad in wave_instrs(NT, NCH * BT * N, lambda x, w=w: row(x) + w):
            c += cycles("w32", ad); i += 2
    # epilogue: each channel's pixel (bt, h, w), idx -> bt fastest
    for ch in range(NCH):
        for ad in wave_instrs(NT, BT * N * N, lambda x, ch=ch: 2 * (ch * CS + (x % BT) * ZS + (x // BT // N) * H) + (x // BT) % N):
            c += cycles("r32", ad); i += 2
    return c, i


def search_inplace():
    for N, NT in ((8, 256), (16, 512), (32, 512)):
        H = N // 2 + 1
        for nch in (2, 1):
            res = sorted((irfft_inplace_cost(N, zs, nch, 8, NT)[0], zs) for zs in range(N * H, N * H + 33))
            print(f"irfft2 in place N={N} NCH={nch}: ideal {irfft_inplace_cost(N, N * H + 1, nch, 8, NT)[1]}, "
                  f"best {res[:4]}, ZS={N * H + 1}: {irfft_inplace_cost(N, N * H + 1, nch, 8, NT)[0]}", flush=True)


def rfft_inplace_cost(N, BT, ZS, NCH, NT):
    """k_sconv_rfft2 since r05: real input in place in the complex buffer (row stride 2H floats)."""
    H = N // 2 + 1
    CS = BT * ZS
    c = i = 0

    def pix(ch, bt, h):
        return 2 * (ch * CS + bt * ZS + h * H)
    for ch in range(NCH):
        for ad in wave_instrs(NT, BT * N * N, lambda x, ch=ch: pix(ch, x % BT, x // BT // N) + (x // BT) % N):
            c += cycles("w32", ad); i += 2

    def row(x):
        ch, r = divmod(x, BT * N)
        return pix(ch, r % BT, r // BT)
    for w in range(N):
        for ad in wave_instrs(NT, NCH * BT * N, lambda x, w=w: row(x) + w):
            c += cycles("r32", ad); i += 2
    for kb in range(H):
        for ad in wave_instrs(NT, NCH * BT * N, lambda x, kb=kb: row(x) + 2 * kb):
            c += cycles("w64", ad); i += 4

    def col(x, h):
        ch, r = divmod(x, BT * H)
        return 2 * (ch * CS + (r % BT) * ZS + h * H + r // BT)
    for h in range(N):
        for ad in wave_instrs(NT, NCH * BT * H, lambda x, h=h: col(x, h)):
            c += cycles("r64", ad); i += 2
    return c, i


def search_rfft_inplace():
    for N, BT, NCH, NT in ((8, 16, 1, 512), (8, 16, 2, 512), (16, 16, 1, 512), (16, 16, 2, 512),
                           (32, 8, 2, 512), (32, 4, 1, 512), (8, 4, 1, 512), (16, 4, 1, 512)):
        H = N // 2 + 1
        res = sorted((rfft_inplace_cost(N, BT, zs, NCH, NT)[0], zs) for zs in range(N * H, N * H + 33))
        print(f"rfft2 in place N={N} BT={BT} NCH={NCH}: ideal {rfft_inplace_cost(N, BT, N * H + 1, NCH, NT)[1]}, "
              f"best {res[:4]}", flush=True)
