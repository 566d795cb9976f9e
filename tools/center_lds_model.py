#!/usr/bin/env python3
"""LDS bank model of the 2^13-tile center kernel's exchanges (ntt_wave.hip Eng<13, 3, 13>):
which element each lane of a half-wave writes / reads in every exchange (Eng::lane_bit, lbq), and
the worst bank conflict degree under the padded layout word = e + (e >> s).  Prints the degree of
each exchange for pad shifts 3..9, then searches every split of the 13 stages into 5 rounds and
every register window per round (the last forward round at bits [0, 3)) for the arrangement with
the fewest conflicts.  (Result: the engine's own arrangement, 1 / 2 / 2 / 2, is the best; no
round layout or pad shift removes the 2-way conflicts of the middle exchanges.)"""
import itertools

TB, R, M = 13, 3, 13
NR = (M + R - 1) // R


def s_lo(q, inv):
    return max(0, M - R * (NR - q)) if inv else max(0, M - 1 - R * q - (R - 1))


def lbq(q, inv):
    return min(s_lo(q, inv), TB - R)


def lane_bit_lb(lb, i):   # non-column mapping (the center's M = TB)
    return i if i < lb else i + R


def degree(lbw, lbr, pad=lambda e: e + (e >> 5)):
    worst = 0
    for lb in (lbw, lbr):
        for k in range(1 << R):
            banks = {}
            for lane in range(32):
                e = k << lb
                for i in range(5):
                    if (lane >> i) & 1:
                        e |= 1 << lane_bit_lb(lb, i)
                b = pad(e) % 32
                banks[b] = banks.get(b, 0) + 1
            worst = max(worst, max(banks.values()))
    return worst


def main():
    for inv in (False, True):
        for q in range(NR - 1):
            row = [degree(lbq(q, inv), lbq(q + 1, inv), lambda e, s=s: e + (e >> s)) for s in range(3, 10)]
            print("inv" if inv else "fwd", q, "windows", lbq(q, inv), lbq(q + 1, inv), "degree by pad shift 3..9:", row)
    best = []
    for sizes in itertools.product((1, 2, 3), repeat=NR):
        if sum(sizes) != M:
            continue
        hi, chunks = M - 1, []
        for sz in sizes:
            chunks.append((hi - sz + 1, hi))
            hi -= sz
        opts = [[lb for lb in range(0, TB - R + 1) if lb <= lo and h < lb + R] for lo, h in chunks]
        if 0 not in opts[-1]:
            continue
        opts[-1] = [0]
        for lbs in itertools.product(*opts):
            d = [degree(lbs[q], lbs[q + 1]) for q in range(NR - 1)]
            best.append((sum(d), max(d), sizes, lbs, d))
    best.sort()
    print("best round layouts (sum, max, stage split, windows, per-exchange degree):")
    for b in best[:5]:
        print(" ", b)


if __name__ == "__main__":
    main()
