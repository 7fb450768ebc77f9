"""K15: filtered exact top-k over an HBM-resident corpus (user_id == u AND date >= t)."""
from __future__ import annotations

from typing import Tuple

import torch

from . import _native as N

SORT_CAP = 8192


def filtered_topk_ref(corpus, user_codes, dates, queries, q_user, q_floor, ks, kmax):
    nq = queries.shape[0]
    ids = torch.full((nq, kmax), -1, dtype=torch.int32, device=corpus.device)
    scores = torch.zeros((nq, kmax), dtype=torch.float32, device=corpus.device)
    counts = torch.zeros((nq,), dtype=torch.int32, device=corpus.device)
    for i in range(nq):
        mask = (user_codes == q_user[i]) & (dates >= q_floor[i])
        rows = torch.nonzero(mask).flatten()
        if rows.numel() == 0:
            continue
        s = corpus[rows].float() @ queries[i].float()
        # descending score, ties by smaller row id (rows are ascending -> stable sort)
        order = torch.sort(-s, stable=True).indices
        k = min(int(ks[i]), rows.numel(), kmax)
        ids[i, :k] = rows[order[:k]].to(torch.int32)
        scores[i, :k] = s[order[:k]]
        counts[i] = k
    return ids, scores, counts


class _Workspace:
    def __init__(self):
        self.key = None

    def get(self, nq: int, cap: int, device):
        key = (nq, cap, str(device))
        if self.key != key:
            self.counts = torch.empty((nq,), dtype=torch.int32, device=device)
            self.cand = torch.empty((nq, cap), dtype=torch.int32, device=device)
            self.scores = torch.empty((nq, cap), dtype=torch.float32, device=device)
            self.key = key
        return self.counts, self.cand, self.scores


_WS = _Workspace()


def filtered_topk(corpus: torch.Tensor, user_codes: torch.Tensor, dates: torch.Tensor, queries: torch.Tensor,
                  q_user: torch.Tensor, q_floor: torch.Tensor, ks: torch.Tensor, kmax: int,
                  cap: int = 65536) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """-> (row ids [nq,kmax] int32, scores [nq,kmax] f32, counts [nq] int32), best first."""
    nq, D = queries.shape
    if not N.use_native(corpus):
        return filtered_topk_ref(corpus, user_codes, dates, queries, q_user.tolist(), q_floor.tolist(),
                                 ks.tolist(), kmax)
    if nq > 64:  # kernel handles 64 queries per launch
        parts = [filtered_topk(corpus, user_codes, dates, queries[i:i + 64], q_user[i:i + 64], q_floor[i:i + 64],
                               ks[i:i + 64], kmax, cap) for i in range(0, nq, 64)]
        return tuple(torch.cat(x) for x in zip(*parts))
    cap = max(SORT_CAP, min(cap, corpus.shape[0]))
    counts, cand, scores = _WS.get(nq, cap, corpus.device)
    out_ids = torch.full((nq, kmax), -1, dtype=torch.int32, device=corpus.device)
    out_scores = torch.zeros((nq, kmax), dtype=torch.float32, device=corpus.device)
    out_count = torch.empty((nq,), dtype=torch.int32, device=corpus.device)
    queries = queries.to(torch.bfloat16).contiguous()
    # converted inputs bound to names: as N.ptr(x.to(...)) temporaries they would be freed before
    # the launch and the next conversion could reuse (overwrite) their memory on the stream
    qu, qf, kk = q_user.to(torch.int32).contiguous(), q_floor.to(torch.int64).contiguous(), ks.to(torch.int32).contiguous()
    N.call("penny_filtered_topk", N.ptr(corpus), N.ptr(user_codes), N.ptr(dates), corpus.shape[0], D,
           N.ptr(queries), N.ptr(qu), N.ptr(qf), N.ptr(kk), nq, kmax, N.ptr(counts), N.ptr(cand), N.ptr(scores), cap,
           N.ptr(out_ids), N.ptr(out_scores), N.ptr(out_count), N.stream())
    oc = out_count.cpu()
    big = (oc < 0).nonzero().flatten().tolist()
    for i in big:  # > SORT_CAP candidates: finish on device with torch.topk
        total = -int(oc[i])
        k = min(int(ks[i]), total, kmax)
        if total <= cap:
            s, j = torch.topk(scores[i, :total], k)
            out_ids[i, :k], out_scores[i, :k] = cand[i, :total][j], s
        else:
            mask = (user_codes == q_user[i]) & (dates >= q_floor[i])
            full = (corpus.float() @ queries[i].float()).masked_fill(~mask, float("-inf"))
            s, j = torch.topk(full, k)
            out_ids[i, :k], out_scores[i, :k] = j.to(torch.int32), s
        oc[i] = k
    return out_ids, out_scores, oc.to(corpus.device)
