"""CPU model of the tile GEMM's stream-K tail (gemm_prefill.hip tail_plan / sk_owner and the kernel's
segment walk): every K-tile of every tail tile is computed exactly once, a tile's segments are
workgroups sk_owner(first)..sk_owner(last) in K order, partial slots (tile + workgroup) never
collide and stay inside the [sk + P] workspace, and the plan keeps >= 16 K-tiles per workgroup."""
import pytest

TM = TN = 256
BK = 64


def sk_owner(it, P, I):
    u = it * P // I
    while u + 1 < P and (u + 1) * I // P <= it:
        u += 1
    while u > 0 and u * I // P > it:
        u -= 1
    return u


def tail_plan(M, N, K, cus):
    T = -(-M // TM) * (N // TN)
    if T % cus == 0:
        return None
    ntot, L = K // BK, T % cus
    sk = L
    if L * ntot < 16 * cus and T >= L + cus:
        sk = L + cus
    I = sk * ntot
    P = min(cus, I // 16)
    saved = (-(-T // cus) - (T - sk) / cus - I / (P * ntot)) * ntot
    if P < 2 or saved < 8.0:
        return None
    return T - sk, sk, P


def segments(sk, P, ntot):
    I = sk * ntot
    for u in range(P):
        it, end = u * I // P, (u + 1) * I // P
        while it < end:
            tu = it // ntot
            kb = it - tu * ntot
            ke = min(end - tu * ntot, ntot)
            yield u, tu, kb, ke
            it = tu * ntot + ke


@pytest.mark.parametrize("M,N,K", [(512, 4096, 4096), (2304, 4096, 4096), (2304, 4096, 14336), (768, 6144, 4096),
                                   (1024, 28672, 4096), (4608, 4096, 4096), (3072, 6144, 4096), (300, 512, 1024),
                                   (1000, 768, 768), (2560, 1024, 2048)])
def test_stream_k_partition(M, N, K):
    cus = 256
    plan = tail_plan(M, N, K, cus)
    if plan is None:
        return
    dpn, sk, P = plan
    ntot = K // BK
    assert (dpn % cus) == 0 and P <= cus
    assert sk * ntot // P >= 16
    cover = {}
    slots = set()
    for u, tu, kb, ke in segments(sk, P, ntot):
        assert 0 <= kb < ke <= ntot
        for k in range(kb, ke):
            assert (tu, k) not in cover
            cover[(tu, k)] = u
        whole = kb == 0 and ke == ntot
        if not whole:
            uf = sk_owner(tu * ntot, P, sk * ntot)
            ul = sk_owner(tu * ntot + ntot - 1, P, sk * ntot)
            assert uf <= u <= ul
            slot = tu + u
            assert slot not in slots and slot < sk + P
            slots.add(slot)
            # the combine reads slots tu + uf .. tu + ul: exactly this tile's segments
            assert all(tu + v in slots or v > u for v in range(uf, ul + 1))
    assert len(cover) == sk * ntot
