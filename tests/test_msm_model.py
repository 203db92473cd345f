"""CPU: the index arithmetic of the RLC bucket sums (cess_amd/csrc/k_rlc.hip,
k_msm_*; host layout in host_rlc.cpp msm_sums) on a scalar model of G1.

Points are modelled by their discrete logarithms in Z_r, so every group
operation is exact integer arithmetic and the bucket result must equal
sum_i r_i s_i mod r.  The model restates the kernels' formulas: 8-bit window
digits of the 128-bit scalar (k[0] least significant), bucket id
(seg * 16 + w) * 256 + d, chunking by msm_chunk (>= 64 entries, <= 32 chunks
per bucket), the window running sums over digit blocks [16q, 16q + 16) with
the (16q - 1) correction, and the 2^(8w) weights.  The GPU tests
(tests/test_gpu_rlc.py) check the real kernels against per-record multiples.
"""
import random

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
WIN, DIG = 16, 256


def msm_chunk(cnt):
    return max(64, (cnt + 31) // 32)


def digit(k4, w):
    return (k4[w >> 2] >> (8 * (w & 3))) & 255


def bucket_sums(records, nseg):
    """records: (seg, scalar words k4, point-log) -> per-segment sums."""
    nb = nseg * WIN * DIG
    cnt = [0] * nb
    for seg, k4, _ in records:
        for w in range(WIN):
            d = digit(k4, w)
            if d:
                cnt[(seg * WIN + w) * DIG + d] += 1
    start, items, e, it = [0] * nb, [0] * (nb + 1), 0, 0
    for b in range(nb):
        start[b], items[b] = e, it
        e += cnt[b]
        if cnt[b]:
            it += -(-cnt[b] // msm_chunk(cnt[b]))
    items[nb] = it
    idx, cur = [None] * e, list(start)
    for j, (seg, k4, _) in enumerate(records):
        for w in range(WIN):
            d = digit(k4, w)
            if d:
                b = (seg * WIN + w) * DIG + d
                idx[cur[b]] = j
                cur[b] += 1
    # k_msm_items: work item j -> its bucket by binary search, its chunk
    part = [0] * it
    for j in range(it):
        lo, hi = 0, nb
        while hi - lo > 1:
            mid = (lo + hi) >> 1
            if items[mid] <= j:
                lo = mid
            else:
                hi = mid
        b = lo
        L, t = msm_chunk(cnt[b]), j - items[b]
        s, en = start[b] + t * L, start[b] + min(cnt[b], (t + 1) * L)
        assert s < en
        part[j] = sum(records[idx[q]][2] for q in range(s, en)) % R
    bsum = [sum(part[items[b]:items[b + 1]]) % R for b in range(nb)]
    # k_msm_window / k_msm_wsum / k_msm_finish
    out = []
    for seg in range(nseg):
        total = 0
        for w in range(WIN):
            sw = seg * WIN + w
            W = 0
            for q in range(16):
                acc = sm = 0
                for d in range(16 * q + 15, 16 * q - 1, -1):
                    if d:
                        acc = (acc + bsum[sw * DIG + d]) % R
                    sm = (sm + acc) % R
                W += sm + (16 * q - 1) * acc
            total += (W % R) << (8 * w)
        out.append(total % R)
    return out


def test_bucket_model_equals_direct_sums():
    rng = random.Random(5)
    nseg = 3
    records = []
    for i in range(5000):
        k = rng.randrange(1 << 128) | 1
        k4 = [(k >> (32 * w)) & 0xFFFFFFFF for w in range(4)]
        records.append((rng.randrange(nseg), k4, rng.randrange(R)))
    # a heavy bucket (many equal digits) so chunking splits it
    for i in range(3000):
        k = 0x0101010101010101_0101010101010101
        records.append((0, [(k >> (32 * w)) & 0xFFFFFFFF for w in range(4)], rng.randrange(R)))
    got = bucket_sums(records, nseg)
    for seg in range(nseg):
        want = sum(sum(k4[w] << (32 * w) for w in range(4)) * s for sg, k4, s in records if sg == seg) % R
        assert got[seg] == want


def test_msm_chunk_bounds():
    for cnt in (1, 63, 64, 65, 2047, 2048, 2049, 10 ** 5, 16 * 10 ** 6):
        L = msm_chunk(cnt)
        n_items = -(-cnt // L)
        assert L >= 64 and n_items <= 32 and (n_items - 1) * L < cnt <= n_items * L
