"""Host-side lean (split-KV) prefill work lists (ops.attention.prefill_lean_list), on CPU: every KV
block of every (sequence, tile) walk is assigned exactly once, split tiles get consecutive partial
slots in chunk order with one merge record each, items come longest first, and steps whose walks
are already balanced get no lean list."""
import numpy as np
import pytest

from financial_chatbot_llm_amd.ops import attention as A


def _walks(cu, ctx, G, causal=True):
    TQ = 256 // G
    out = {}
    for s, (n, c) in enumerate(zip(np.diff(cu).tolist(), ctx)):
        for t in range((n + TQ - 1) // TQ):
            last = min((t + 1) * TQ, n) - 1
            kv_end = min(c, c - n + last + 1) if causal else c
            out[(s, t)] = (kv_end + A.KV_BS - 1) // A.KV_BS
    return out


@pytest.mark.parametrize("shape", [
    [(220, 4600)],                                    # one decide behind a long cached context
    [(230, 4700), (210, 4500)],
    [(600, 4200)],
    [(9, 5200)] * 3 + [(220, 4600)],
    [(1600, 3400)] + [(220, 4600)] * 8,               # balanced enough: no lean list
    [(4096, 4096)],
])
@pytest.mark.parametrize("causal", [True, False])
def test_lean_list_covers_every_block_once(shape, causal, monkeypatch):
    monkeypatch.setattr(A, "LEAN_COST_GATE", False)      # the list's structure; the gate is below
    G, Hkv = 4, 8
    cu = np.array([0] + list(np.cumsum([q for q, _ in shape])), np.int64)
    ctx = [c for _, c in shape]
    walks = _walks(cu, ctx, G, causal)
    ln = A.prefill_lean_list(cu, np.array(ctx), G, Hkv, causal)
    if ln is None:
        total = sum(walks.values())
        C = max(A.LEAN_MIN_CHUNK, -(-total * Hkv // 256))
        assert max(walks.values()) <= C                  # nothing needed splitting
        return
    assert ln[0, 0] == -1
    ni, nm, nslots = int(ln[0, 1]), int(ln[0, 2]), int(ln[0, 3])
    items, merges = ln[1:1 + ni], ln[1 + ni:1 + ni + nm]
    assert len(ln) == 1 + ni + nm
    lengths = items[:, 3] - items[:, 2]
    assert (lengths > 0).all() and (np.diff(lengths) <= 0).all()    # LPT order
    cover = {}
    for s, t, b0, b1, slot, _ in items.tolist():
        for b in range(b0, b1):
            assert (s, t, b) not in cover
            cover[(s, t, b)] = slot
    assert len(cover) == sum(walks.values())
    assert all((s, t, b) in cover for (s, t), nb in walks.items() for b in range(nb))
    used = set()
    for s, t, slot0, k, _, _ in merges.tolist():
        chunks = sorted((b0, slot) for ss, tt, b0, b1, slot, _ in items.tolist() if (ss, tt) == (s, t))
        assert [slot for _, slot in chunks] == list(range(slot0, slot0 + k))   # chunk order = slot order
        used.update(range(slot0, slot0 + k))
        assert k >= 2
    assert used == set(range(nslots))
    whole = [(s, t) for s, t, b0, b1, slot, _ in items.tolist() if slot < 0]
    assert all(b0 == 0 and b1 == walks[(s, t)] for s, t, b0, b1, slot, _ in items.tolist() if slot < 0)
    assert len(set(whole)) == len(whole)


def test_lpt_makespan():
    assert A._lpt_makespan([5, 4, 3, 3, 3], 2) == 10.0      # LPT: 5 | 4, 3 -> 4+3 | 5+3 | 7+3
    assert A._lpt_makespan([7, 1], 4) == 7.0
    assert A._lpt_makespan([2] * 8, 4) == 4.0


@pytest.mark.parametrize("shape,split", [
    ([(220, 4600)], True),                            # one decide: 4 tiles x 8 heads on 256 CUs
    ([(230, 4700), (210, 4500)], True),
    ([(600, 4200)], True),
    # more chunks than CUs: a second round behind the longest whole tiles -- measured slower split
    # (profiles/r6_prefill_attn_pair_barrier_rejected.jsonl pf3_prod vs pf3_q)
    ([(600, 3600)] + [(220, 4600)] * 4, False),
    ([(220, 4600)] * 4 + [(9, 5200)] * 16, False),
])
def test_lean_cost_gate_decisions(shape, split):
    cu = np.array([0] + list(np.cumsum([q for q, _ in shape])), np.int64)
    ln = A.prefill_lean_list(cu, np.array([c for _, c in shape]), 4, 8)
    assert (ln is not None) == split
